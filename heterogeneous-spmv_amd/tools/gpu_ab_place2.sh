# GPU-box check + A/B of the placement trials (hspmv_create_on_device): the
# CSR-3 / full-size parity tests, then identical C3 handles with trials
# (default 4 sets) and without (HSPMV_PLACEMENT=0), and the chunk size /
# y store policy with trials on.
# Usage: bash heterogeneous-spmv_amd/tools/gpu_ab_place2.sh TAG
set -o pipefail
TAG=${1:-place2}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=heterogeneous-spmv_amd/build/libhspmv.so
T=heterogeneous-spmv_amd/tools
echo "== pytest" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_xdict.py -m gpu -x -q -k "csr3 or xdict or full_size" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] &&
echo "== ab c3" && timeout -k 10 500 python $T/ab.py \
  --libs "$L,$L,$L,$L#HSPMV_PLACEMENT=0,$L#HSPMV_PLACEMENT=0,$L@327680#HSPMV_PF=1,$L@327680#HSPMV_PF=1#HSPMV_YNT=0,$L#HSPMV_YNT=0" \
  --configs c3,c4,c3h --rounds 5 --out gpurun_out/ab_${TAG}.jsonl 2>&1 | grep -v amdgpu.ids
