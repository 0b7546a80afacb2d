#!/bin/bash
# GPU-box pass (round 4 o): STREAM launch shapes for short rows (groups per
# wave x chunk size x waves per workgroup) on the honeycomb (hugebubbles
# stand-in), the tall / diagonal zoo shapes and the banded configs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04o; mkdir -p $O
cd $R; T=heterogeneous-spmv_amd/tools
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -4 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step short_grid 900 python -u $T/sweep.py --configs c3h,tall,diag,c4,c2,l4k --grid short --rounds 3 --iters 20 --out $O/sweep_short_rows.jsonl
