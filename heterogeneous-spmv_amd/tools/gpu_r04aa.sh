#!/bin/bash
# GPU-box pass (round 4 aa): the full gpu test suite, smoke, the bench line
# and the rocprofv3 kernel-trace summary of the same bench command.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04aa; mkdir -p $O
cd $R
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -3 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
bash heterogeneous-spmv_amd/tools/host_info.sh $O/host.txt > /dev/null 2>&1
step gputest 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
cd /tmp && export TMPDIR=/tmp
echo "== rocprof bench"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 $R/bench.py > $O/rocprof_bench.log 2>&1
rc=$?; echo "   rc=$rc"; cp $O/prof_bench/*kernel_stats.csv $O/bench_kernel_stats.csv 2>/dev/null; head -5 $O/bench_kernel_stats.csv | cut -c1-200
