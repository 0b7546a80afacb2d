# GPU-box pass: rocprofv3 --kernel-trace --stats over tools/run_one.py for each
# non-bench config (C3 CSR-3, hugebubbles stand-in, C4 shard, C5, C3 fp32),
# summaries under gpurun_out/<TAG>_kstats/; each run also times 20 cold launches
# (Infinity Cache evicted by a 512 MiB read before each: cold_us).
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/gpu_kstats.sh [TAG] ["cfg cfg ..."]
set -o pipefail
TAG=${1:-r01}; CFGS=${2:-"c3 c3h c4 c5 c3:f32"}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/${TAG}_kstats
export PYTHONUNBUFFERED=1
O=$R/gpurun_out/${TAG}_kstats
cd /tmp && export TMPDIR=/tmp
for cfg in $CFGS; do
  name=${cfg/:/_}
  echo "== $cfg"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run \
    -- python3 $R/heterogeneous-spmv_amd/tools/run_one.py --config $cfg --iters 100 --cold 20 \
    > $O/${name}_run.log 2>&1 || exit $?
  grep '^{' $O/${name}_run.log > $O/${name}_run.json
  cp $O/prof_$name/*kernel_stats.csv $O/${name}_kernel_stats.csv
  head -c 300 $O/${name}_run.json; echo
done
