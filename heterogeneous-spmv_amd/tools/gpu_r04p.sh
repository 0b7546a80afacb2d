#!/bin/bash
# GPU-box pass (round 4 p): STREAM waves per workgroup 1 / 2 / 4 on C4's
# shards at 8 / 4 / 2 ranks and whole, C2 and the honeycomb (7 rounds, one
# process per config).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04p; mkdir -p $O
cd $R; T=heterogeneous-spmv_amd/tools
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -4 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step waves 900 python -u $T/sweep.py --configs c4,c4p4,c4p2,c4p1,c2,c3h,l4k --grid waves --rounds 7 --iters 20 --out $O/sweep_stream_waves.jsonl
