#!/bin/bash
# GPU-box pass (round 4 j): csort gather-lane quad packing -- tests, A/B in
# one process (diag-env library), timelines with the build's quad-sector
# counts.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04j; mkdir -p $O
cd $R; T=heterogeneous-spmv_amd/tools; E=heterogeneous-spmv_amd/build/diagenv/libhspmv.so
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -4 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step csort_tests 300 python -u -m pytest tests/test_csort.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "csort or c5"
step ab_pack 400 python $T/ab.py --libs "$E#HSPMV_CSORT_PACK=-1,$E,$E#HSPMV_CSORT_PACK=-1,$E" --configs c5,c5r --rounds 7 --out $O/ab_c5_pack.jsonl
step trace 240 python $T/csort_trace.py --configs c5,c5r --per-wg --out $O/csort_trace_wg_pack.jsonl
