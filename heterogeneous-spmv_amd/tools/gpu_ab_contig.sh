# GPU-box A/B: physically contiguous device allocations (HSPMV_CONTIG=1,
# hipDeviceMallocContiguous) against plain hipMalloc, alternating identical
# handles in one process (C3 fp64 / fp32, C4 shard, honeycomb).
# Usage: bash heterogeneous-spmv_amd/tools/gpu_ab_contig.sh TAG
set -o pipefail
TAG=${1:-contig}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=heterogeneous-spmv_amd/build/libhspmv.so
T=heterogeneous-spmv_amd/tools
C="$L#HSPMV_CONTIG=1"
echo "== ab contig" && timeout -k 10 600 python $T/ab.py \
  --libs "$L,$C,$L,$C,$L,$C" \
  --configs c3,c3:f32,c4,c3h --rounds 5 --out gpurun_out/ab_${TAG}.jsonl 2>&1 | grep -v amdgpu.ids
