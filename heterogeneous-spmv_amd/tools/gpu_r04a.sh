#!/bin/bash
# GPU-box pass (round 4): the gpu test suite, the bench line, then the csort
# per-workgroup timelines of C5 / c5r with the build's cost terms (diag-env
# library).  Stops at the first step that ends in anything but 0 / 1 (a test
# failure still lets the measurements run; a fault, abort or timeout does not).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04a; mkdir -p $O
cd $R
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -3 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step gputest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 300 python bench.py
step trace 240 python heterogeneous-spmv_amd/tools/csort_trace.py --configs c5,c5r --per-wg --out $O/csort_trace_wg.jsonl
