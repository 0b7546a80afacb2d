# GPU-box: GPU tests (unless SKIP_TESTS=1) then the kernel sweep.
# Usage: [SKIP_TESTS=1] bash .../gpu_sweep.sh TAG [configs] [extra sweep args]
set -o pipefail
TAG=${1:-sweep}; CFG=${2:-c2,c3,c4,c5}; EXTRA=${3:-}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest gpu"
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -30 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
echo "== sweep"
timeout -k 10 900 python heterogeneous-spmv_amd/tools/sweep.py --configs $CFG $EXTRA --out gpurun_out/$TAG.jsonl > gpurun_out/$TAG.log 2>&1; rc=$?
cut -c1-330 gpurun_out/$TAG.log; exit $rc
