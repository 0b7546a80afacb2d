# GPU-box: GPU tests then the kernel sweep.  Usage: bash .../gpu_sweep.sh TAG [configs]
set -o pipefail
TAG=${1:-sweep}; CFG=${2:-c2,c3,c4,c5}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "== pytest gpu" && { timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } &&
echo "== sweep" && timeout -k 10 900 python heterogeneous-spmv_amd/tools/sweep.py --configs $CFG --out gpurun_out/$TAG.jsonl > gpurun_out/$TAG.log 2>&1; rc=$?; cat gpurun_out/$TAG.log | cut -c1-330; exit $rc
