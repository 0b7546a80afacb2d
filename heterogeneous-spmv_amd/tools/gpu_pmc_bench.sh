# GPU-box pass: rocprofv3 PMC passes (size-resolved fabric reads, FETCH_SIZE,
# WRITE_SIZE) over a short bench.py run, summarised per launch by
# pmc_summary.py into gpurun_out/<TAG>_<workload>_pmc.json (warm) and
# ..._cold_pmc.json (the cold leg's launches).  One pass per counter group.
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/gpu_pmc_bench.sh TAG [bench args]
set -o pipefail
TAG=${1:-r02}; BARGS=${2:-}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1
P=$R/gpurun_out/$TAG/pmc
bash heterogeneous-spmv_amd/tools/host_info.sh gpurun_out/$TAG/host.txt
# only the headline launches (+ the cold leg, last): no plan legs, no C4
PB="python3 $R/bench.py --no-cpu --no-plans --no-scaling-ref --steps 50 --warmup 10 --cold-steps 10 $BARGS"
timeout -k 10 300 python3 bench.py --no-cpu --no-plans --no-scaling-ref --steps 50 --warmup 10 --cold-steps 10 $BARGS > gpurun_out/$TAG/bench_pmc_plain.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
echo "== rocprof RDREQ" && timeout -k 10 -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $P/rdreq -o bench -- $PB > $R/gpurun_out/$TAG/rocprof_rdreq.log 2>&1 &&
echo "== rocprof FETCH_SIZE" && timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o bench -- $PB > $R/gpurun_out/$TAG/rocprof_fetch.log 2>&1 &&
echo "== rocprof WRITE_SIZE" && timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o bench -- $PB > $R/gpurun_out/$TAG/rocprof_write.log 2>&1 &&
echo "== rocprof TCC requests" && timeout -k 10 -s KILL 300 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $P/tcc -o bench -- $PB > $R/gpurun_out/$TAG/rocprof_tcc.log 2>&1 &&
echo "== rocprof kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o bench -- $PB > $R/gpurun_out/$TAG/rocprof_kt.log 2>&1 || exit 1
cp $P/kt/*kernel_stats.csv $R/gpurun_out/$TAG/bench_kernel_stats.csv 2>/dev/null
cd $R && W=$(python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/$TAG/bench_pmc_plain.log') if l.startswith('{')][-1];r=d['roofline'];print(d['config']['workload_key'], r['alg_bytes_per_launch'], r['launches_per_spmv'])") &&
set -- $W &&
python3 heterogeneous-spmv_amd/tools/pmc_summary.py --fetch $P/fetch --write $P/write --rdreq $P/rdreq --extra $P/tcc --kernel-substr hspmv_ --per-spmv $3 --workload $1 --skip-last 10 --last 50 --alg-bytes $2 -o gpurun_out/${TAG}/${TAG}_$1_pmc.json &&
python3 heterogeneous-spmv_amd/tools/pmc_summary.py --fetch $P/fetch --write $P/write --rdreq $P/rdreq --extra $P/tcc --kernel-substr hspmv_ --per-spmv $3 --workload $1-cold --last 10 --alg-bytes $2 -o gpurun_out/${TAG}/${TAG}_$1-cold_pmc.json &&
cat gpurun_out/${TAG}/${TAG}_$1_pmc.json
