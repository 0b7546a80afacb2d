# GPU-box repeat A/B: identical handles (same library, same flags) created
# one after another in one process, to separate placement effects (where the
# handle's arrays land in HBM) from kernel changes.  C3 fp64.
# Usage: bash heterogeneous-spmv_amd/tools/gpu_ab_placement.sh TAG
set -o pipefail
TAG=${1:-place}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=heterogeneous-spmv_amd/build/libhspmv.so
T=heterogeneous-spmv_amd/tools
V="$L@327680#HSPMV_PF=1#HSPMV_YNT=0"
echo "== ab c3 repeats" && timeout -k 10 500 python $T/ab.py \
  --libs "$L,$L,$L,$V,$V,$V,$L@327680#HSPMV_PF=1,$L" \
  --configs c3 --rounds 5 --out gpurun_out/ab_${TAG}.jsonl 2>&1 | grep -v amdgpu.ids
