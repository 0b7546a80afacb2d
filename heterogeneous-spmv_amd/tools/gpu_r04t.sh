#!/bin/bash
# GPU-box pass (round 4 t): deterministic handles on the power-law configs
# (row kernels with / without the CSR-3 maps, x slabs on / off).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04t; mkdir -p $O
cd $R; T=heterogeneous-spmv_amd/tools
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -4 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step det 600 python -u $T/sweep.py --configs c5,c5r,mix,urand8 --grid det --rounds 3 --iters 20 --out $O/sweep_deterministic.jsonl
