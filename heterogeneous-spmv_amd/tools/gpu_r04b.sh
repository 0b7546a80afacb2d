#!/bin/bash
# GPU-box pass (round 4 b): CSR-3 parity (SSR plan with dictionaries), the
# bench line, and the CPU baseline's process settings A/B (host CPUs only).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04b; mkdir -p $O
cd $R
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -3 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
step parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "csr3"
step bench 300 python bench.py --no-cpu
step cpu_ab 400 python heterogeneous-spmv_amd/tools/cpu_baseline_ab.py --out $O/cpu_baseline_ab.jsonl --budget 6
