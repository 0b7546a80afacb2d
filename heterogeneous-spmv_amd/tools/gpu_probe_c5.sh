# GPU-box pass: the C5 column-sort design probe (tools/probes/csort_proto.hip).
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/gpu_probe_c5.sh TAG [lib]
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== csort probe"
timeout -k 10 400 heterogeneous-spmv_amd/build/probes/csort_proto 2000000 50 > $O/csort.jsonl 2> $O/csort.err || { cat $O/csort.err; exit 1; }
cat $O/csort.jsonl | cut -c1-300
if [ "$2" = lib ]; then
echo "== library c5"
timeout -k 10 300 python3 heterogeneous-spmv_amd/tools/run_one.py --config c5 --iters 50 > $O/c5_run.log 2>&1 || { tail $O/c5_run.log; exit 1; }
grep '^{' $O/c5_run.log | cut -c1-400
fi
