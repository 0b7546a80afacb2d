# GPU-box check: smoke, GPU tests, bench, rocprofv3 kernel trace + PMC passes.
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/gpu_check.sh [TAG]
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
P=$R/gpurun_out/prof_$TAG
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log &&
echo "== pytest gpu" && { timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } &&
echo "== bench" && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && cat gpurun_out/bench.log &&
cd /tmp && export TMPDIR=/tmp &&
echo "== rocprof kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o bench -- python3 $R/bench.py --no-cpu > $R/gpurun_out/rocprof_trace.log 2>&1 &&
echo "== rocprof FETCH_SIZE" && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o bench -- python3 $R/bench.py --no-cpu --steps 50 --warmup 10 --cold-steps 10 > $R/gpurun_out/rocprof_fetch.log 2>&1 &&
echo "== rocprof WRITE_SIZE" && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o bench -- python3 $R/bench.py --no-cpu --steps 50 --warmup 10 --cold-steps 10 > $R/gpurun_out/rocprof_write.log 2>&1 &&
cd $R && ls -R $P | head -30 && cat $P/trace/*kernel_stats.csv | cut -c1-250
