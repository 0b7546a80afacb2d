# GPU-box A/B of C3 with the x-dictionary staging waves at raised issue
# priority (diag builds: HSPMV_DIAG=64 -> s_setprio 3, 128 -> s_setprio 1),
# one process, rounds interleaved.
# Usage: bash heterogeneous-spmv_amd/tools/gpu_ab_c3_prio.sh TAG
set -o pipefail
TAG=${1:-prio}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B=heterogeneous-spmv_amd/build
T=heterogeneous-spmv_amd/tools
echo "== ab c3 prio" && timeout -k 10 500 python $T/ab.py \
  --libs "$B/libhspmv.so,$B/diag64/libhspmv.so,$B/diag128/libhspmv.so" \
  --configs c3,c3:f32 --rounds 6 --out gpurun_out/ab_${TAG}.jsonl 2>&1 | grep -v amdgpu.ids
