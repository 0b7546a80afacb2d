# GPU-box A/B of C3's block order and stream cache policy with x
# dictionaries, one process: default (4-block XCD chunks), full XCD remap
# (each XCD a contiguous eighth), dispatch order, nontemporal col/val streams,
# full remap + nontemporal, 8-wave dictionary blocks.
# Usage: bash heterogeneous-spmv_amd/tools/gpu_ab_c3_order.sh TAG
set -o pipefail
TAG=${1:-order}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=heterogeneous-spmv_amd/build/libhspmv.so
T=heterogeneous-spmv_amd/tools
# flags: 1<<22 XCD_REMAP, 1<<14 NO_XCD_REMAP, 1<<12 NONTEMPORAL
echo "== ab c3 order" && timeout -k 10 500 python $T/ab.py \
  --libs "$L,$L@4194304,$L@16384,$L#HSPMV_NT=1,$L@4198400,$L#HSPMV_XD_WAVES=8" \
  --configs c3,c3:f32 --rounds 5 --out gpurun_out/ab_${TAG}.jsonl 2>&1 | grep -v amdgpu.ids
