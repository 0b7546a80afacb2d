# GPU-box check: smoke, GPU tests, bench, rocprofv3 kernel trace + PMC passes
# (size-resolved fabric reads, WRITE_SIZE, FETCH_SIZE) and their summaries.
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/gpu_check.sh [TAG] [bench args]
set -o pipefail
TAG=${1:-r01}; BARGS=${2:-}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
P=$R/gpurun_out/prof_$TAG
PB="python3 $R/bench.py --no-cpu --steps 50 --warmup 10 --cold-steps 10 $BARGS"
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log &&
echo "== pytest gpu" && { timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } &&
echo "== bench" && timeout -k 10 300 python bench.py $BARGS > gpurun_out/bench_$TAG.log 2>&1 && cat gpurun_out/bench_$TAG.log &&
cd /tmp && export TMPDIR=/tmp &&
echo "== rocprof kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o bench -- python3 $R/bench.py --no-cpu $BARGS > $R/gpurun_out/rocprof_trace.log 2>&1 &&
echo "== rocprof RDREQ" && timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $P/rdreq -o bench -- $PB > $R/gpurun_out/rocprof_rdreq.log 2>&1 &&
echo "== rocprof FETCH_SIZE" && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o bench -- $PB > $R/gpurun_out/rocprof_fetch.log 2>&1 &&
echo "== rocprof WRITE_SIZE" && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o bench -- $PB > $R/gpurun_out/rocprof_write.log 2>&1 &&
cd $R && W=$(python3 -c "import json;d=json.loads(open('gpurun_out/bench_$TAG.log').read().strip().splitlines()[-1]);print(d['config']['workload_key'], d['roofline']['alg_bytes_per_launch'])") &&
set -- $W &&
python3 heterogeneous-spmv_amd/tools/pmc_summary.py --fetch $P/fetch --write $P/write --rdreq $P/rdreq --workload $1 --skip-last 10 --last 50 --alg-bytes $2 -o gpurun_out/${TAG}_$1_pmc.json &&
python3 heterogeneous-spmv_amd/tools/pmc_summary.py --fetch $P/fetch --write $P/write --rdreq $P/rdreq --workload $1-cold --last 10 --alg-bytes $2 -o gpurun_out/${TAG}_$1-cold_pmc.json &&
cat $P/trace/*kernel_stats.csv | cut -c1-250
