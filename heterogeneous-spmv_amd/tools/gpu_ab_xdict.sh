# GPU-box A/B of block x dictionaries (HSPMV_XDICT=0/1) in one process per
# kernel choice, after the XD parity test.  Usage: bash .../gpu_ab_xdict.sh TAG
set -o pipefail
TAG=${1:-xd}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=heterogeneous-spmv_amd/build/libhspmv.so
T=heterogeneous-spmv_amd/tools
echo "== pytest xdict" && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "xdict or col16 or golden" --timeout 240 > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] &&
echo "== ab auto" && timeout -k 10 400 python $T/ab.py --libs "$L#HSPMV_XDICT=0,$L#HSPMV_XDICT=1" --configs c3,c4,c3m,l4k,c2 --rounds 5 --out gpurun_out/ab_${TAG}_auto.jsonl 2>&1 | grep -v amdgpu.ids &&
echo "== ab stream" && timeout -k 10 300 python $T/ab.py --libs "$L#HSPMV_XDICT=0,$L#HSPMV_XDICT=1" --configs c3,c5 --kernel stream --rounds 5 --out gpurun_out/ab_${TAG}_stream.jsonl 2>&1 | grep -v amdgpu.ids
