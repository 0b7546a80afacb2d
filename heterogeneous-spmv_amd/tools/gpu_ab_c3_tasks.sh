# GPU-box A/B of C3's task cut, chunk size and y store policy (x
# dictionaries, one process): default (super-row-packed 60-row tasks, U = 4,
# prefetch, nontemporal y), full 64-row tasks (HSPMV_TASK_FILL=1), cached y
# stores, U = 3 / 5 / 6 with prefetch.
# Usage: bash heterogeneous-spmv_amd/tools/gpu_ab_c3_tasks.sh TAG
set -o pipefail
TAG=${1:-tasks}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=heterogeneous-spmv_amd/build/libhspmv.so
T=heterogeneous-spmv_amd/tools
# flags: HSPMV_U(u) = u << 16
echo "== ab c3 tasks" && timeout -k 10 500 python $T/ab.py \
  --libs "$L,$L#HSPMV_TASK_FILL=1,$L#HSPMV_YNT=0,$L@196608#HSPMV_PF=1,$L@327680#HSPMV_PF=1,$L@393216#HSPMV_PF=1,$L#HSPMV_TASK_FILL=1#HSPMV_YNT=0" \
  --configs c3,c3:f32 --rounds 5 --out gpurun_out/ab_${TAG}.jsonl 2>&1 | grep -v amdgpu.ids
