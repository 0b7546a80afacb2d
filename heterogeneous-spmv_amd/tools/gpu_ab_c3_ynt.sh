# GPU-box check + A/B after the 64-row aligned CSR-3 tasks: the CSR-3 parity
# tests, then (one process each) y store policy and chunk size on C3 fp64 /
# fp32, and the y store policy on the STREAM configurations.
# Usage: bash heterogeneous-spmv_amd/tools/gpu_ab_c3_ynt.sh TAG
set -o pipefail
TAG=${1:-ynt}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=heterogeneous-spmv_amd/build/libhspmv.so
T=heterogeneous-spmv_amd/tools
echo "== pytest csr3" && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_xdict.py -m gpu -x -q -k "csr3 or xdict or full_size" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] &&
echo "== ab c3" && timeout -k 10 500 python $T/ab.py \
  --libs "$L,$L#HSPMV_TASK_FILL=0,$L#HSPMV_YNT=0,$L#HSPMV_YNT=0#HSPMV_PF=0,$L@327680#HSPMV_PF=1#HSPMV_YNT=0,$L@393216#HSPMV_PF=1#HSPMV_YNT=0,$L@524288#HSPMV_PF=1#HSPMV_YNT=0" \
  --configs c3,c3:f32 --rounds 5 --out gpurun_out/ab_${TAG}_c3.jsonl 2>&1 | grep -v amdgpu.ids &&
echo "== ab stream" && timeout -k 10 400 python $T/ab.py \
  --libs "$L,$L#HSPMV_YNT=0" --configs c4,c3h,c2 --rounds 5 --out gpurun_out/ab_${TAG}_stream.jsonl 2>&1 | grep -v amdgpu.ids
