#!/bin/bash
# GPU-box pass (round 4 u): the x-slab span condition -- parity tests that
# touch slabs, and the deterministic-handle grid again.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04u; mkdir -p $O
cd $R; T=heterogeneous-spmv_amd/tools
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -4 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_gpu_parity.py tests/test_csort.py tests/test_planner.py tests/test_zoo.py -x -q --timeout 200 --timeout-method thread -k "slab or c5 or csort or planner or zoo or deterministic"
step det 600 python -u $T/sweep.py --configs c5,c5r,mix --grid det --rounds 3 --iters 20 --out $O/sweep_deterministic.jsonl
