#!/bin/bash
# GPU-box pass (round 4 z): the csort x-size threshold (256 KiB): planner
# regret on the shapes it moves (fp32 mix) or must not move (tall, C5, c2),
# and the csort / planner / zoo tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04z; mkdir -p $O
cd $R; T=heterogeneous-spmv_amd/tools
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -2 $O/$name.log | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_csort.py tests/test_planner.py tests/test_zoo.py tests/test_density.py -x -q --timeout 200 --timeout-method thread
step regret 700 python -u $T/auto_regret.py --zoo mix:f32,tall:f32,blocks32:f32,d64:f32,c2:f32,c4:f32,mix,tall,c5 --out $O/auto_regret_threshold.jsonl
