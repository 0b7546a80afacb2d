# GPU-box: C3 occupancy and store-path A/Bs of round 3, one process each
# (diag-env library), plus the per-workgroup timeline (diag-512 build) and
# the dictionary / CSR3 GPU tests.
# Usage (repo root): bash heterogeneous-spmv_amd/tools/gpu_c3_occupancy.sh TAG
set -o pipefail
TAG=${1:-c3occ}
R=$GRAFT_REPO_ROOT; D=$R/gpurun_out/$TAG; mkdir -p $D
export PYTHONUNBUFFERED=1
E=$R/heterogeneous-spmv_amd/build/diagenv/libhspmv.so
HSPMV_LIB=$R/heterogeneous-spmv_amd/build/diag512/libhspmv.so timeout -k 10 200 \
  python3 $R/heterogeneous-spmv_amd/tools/block_trace.py --configs c3 --out $D/block_trace.jsonl || exit 1
timeout -k 10 400 python3 $R/heterogeneous-spmv_amd/tools/ab.py \
  --libs "$E,$E#HSPMV_XD_BPC=-1,$E#HSPMV_XD_BPC=7,$E#HSPMV_XD_BPC=8" \
  --configs c3,c3:f32 --rounds 5 --out $D/ab_c3_xd_bpc.jsonl || exit 1
timeout -k 10 400 python3 $R/heterogeneous-spmv_amd/tools/ab.py \
  --libs "$E,$E#HSPMV_NT=1#HSPMV_YNT=0,$E#HSPMV_YNT=0,$E#HSPMV_NT=1" \
  --configs c3 --rounds 5 --out $D/ab_c3_nt_ynt.jsonl || exit 1
cd $R && timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 \
  -k "xdict or csr3 or c3 or stencil" > $D/pytest.log 2>&1
rc=$?; tail -3 $D/pytest.log; exit $rc
