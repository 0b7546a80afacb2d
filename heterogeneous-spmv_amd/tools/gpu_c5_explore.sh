# GPU-box exploration of the C5 column-sorted kernel: LDS atomic throughput
# by slot type (tools/probes/lds_atomic_probe.hip), then C5 csort variants in one
# process (tools/ab.py; rounds interleaved).
# Usage: bash heterogeneous-spmv_amd/tools/gpu_c5_explore.sh TAG [VARIANTS]
set -o pipefail
TAG=${1:-c5x}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
B=heterogeneous-spmv_amd/build
T=heterogeneous-spmv_amd/tools
L=$B/diagenv/libhspmv.so  # reads the HSPMV_* A/B knobs
V=${2:-"$L,$L#HSPMV_CSORT_PF=1,$L#HSPMV_CSORT_U=8,$L#HSPMV_CSORT_U=8#HSPMV_CSORT_PF=1"}
bash heterogeneous-spmv_amd/tools/host_info.sh gpurun_out/host_${TAG}.txt
if [ -n "$LDS_PROBE" ]; then
  echo "== lds probe" && timeout -k 10 120 $B/probes/lds_atomic_probe > gpurun_out/lds_probe_${TAG}.jsonl && cat gpurun_out/lds_probe_${TAG}.jsonl || exit 1
fi
echo "== ab c5" && timeout -k 10 600 python $T/ab.py --libs "$V" --configs ${CONFIGS:-c5} --rounds 6 \
  --out gpurun_out/ab_${TAG}.jsonl 2>&1 | grep -v amdgpu.ids
