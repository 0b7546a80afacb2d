#!/bin/bash
# GPU-box pass (round 4 y): AUTO planner regret in fp32 (the reference's
# value type) over the zoo.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04y; mkdir -p $O
cd $R; T=heterogeneous-spmv_amd/tools
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -2 $O/$name.log | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step regret_f32_a 600 python -u $T/auto_regret.py --zoo c2:f32,c3:f32,c3h:f32,c4:f32,mix:f32,d24:f32,d64:f32,d512:f32 --out $O/auto_regret_f32_a.jsonl
step regret_f32_b 600 python -u $T/auto_regret.py --zoo urand8:f32,urand32:f32,blocks32:f32,arrow:f32,wide:f32,tall:f32,diag:f32 --out $O/auto_regret_f32_b.jsonl
