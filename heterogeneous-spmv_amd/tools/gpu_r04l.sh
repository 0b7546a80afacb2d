#!/bin/bash
# GPU-box pass (round 4 l): AUTO planner regret over a matrix zoo
# (tools/auto_regret.py): the BASELINE configurations, then shapes the
# planner was not fitted to.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04l; mkdir -p $O
cd $R; T=heterogeneous-spmv_amd/tools
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -4 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step regret_extra 500 python -u $T/auto_regret.py --zoo urand8,urand32,blocks32,arrow,wide,tall,diag,c5d --out $O/auto_regret_extra.jsonl
step regret_base 600 python -u $T/auto_regret.py --zoo c2,c3,c3h,c4,c5,c5r,mix,d24,d64,d512 --out $O/auto_regret_base.jsonl
