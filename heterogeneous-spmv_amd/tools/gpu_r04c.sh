#!/bin/bash
# GPU-box pass (round 4 c): csort column-part / crowded-row balancing, A/B in
# one process (diag-env library), then per-workgroup timelines with it on.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04c; mkdir -p $O
cd $R; T=heterogeneous-spmv_amd/tools; E=heterogeneous-spmv_amd/build/diagenv/libhspmv.so
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -4 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step csort_tests 300 python -u -m pytest tests/test_csort.py -x -q --timeout 200 --timeout-method thread
step ab_balance 400 python $T/ab.py --libs "$E#HSPMV_CSORT_BALANCE=-1,$E" --configs c5,c5r --rounds 5 --out $O/ab_c5_balance.jsonl
step trace 240 python $T/csort_trace.py --configs c5,c5r --per-wg --out $O/csort_trace_wg_balanced.jsonl
step ab_c3_py 500 python $T/ab.py --libs "$E,$E#HSPMV_CSR3_PY=1,$E#HSPMV_CSR3_PY=2,$E#HSPMV_CSR3_PY=4,$E#HSPMV_CSR3_PY=8" --configs c3,c3:f32 --rounds 5 --out $O/ab_c3_py.jsonl
step ab_c5_fin 300 python $T/ab.py --libs "$E,$E#HSPMV_CSORT_FIN_ROWS=4,$E#HSPMV_CSORT_FIN_ROWS=1" --configs c5,c5r --rounds 5 --out $O/ab_c5_fin_rows.jsonl
