#!/bin/bash
# The one GPU-box pass script: a list of steps, each under its own time limit,
# logs under gpurun_out/TAG/.  A step that fails with a test failure (rc 1)
# is reported and the pass goes on; any other failure (a fault, an abort, a
# time limit) ends the pass there -- no GPU step runs after it.
#
# Usage (from the repo root):
#   bash heterogeneous-spmv_amd/tools/gpu_round.sh TAG STEP [STEP ...]
# Steps:
#   gputest[:KEXPR]     pytest -m gpu (optionally -k KEXPR)
#   tests:FILES[:KEXPR] pytest on the given test files (comma separated), gpu+cpu
#   smoke               __graft_entry__.smoke()
#   bench[:ARGS]        python bench.py ARGS (ARGS: commas become spaces)
#   rocprof[:ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS
#   rocprofleg[:ARGS]   the same with --marker-trace --kernel-rename: kernels
#                       reported per bench leg (bench.py's roctx ranges)
#   kstats:CFGS         tools/gpu_kstats.sh over run_one.py (CFGS comma separated)
#   kstat1:NAME:ARGS    rocprofv3 --kernel-trace --stats over run_one.py ARGS (';' for spaces)
#   pmc:CFG             tools/gpu_pmc_bench.sh TAG_CFG --config CFG (PMC traffic summary)
#   ab:ARGS             tools/ab.py ARGS (commas inside ARGS: use ';' for spaces)
#   py:NAME:SECS:ARGS   python ARGS (';' for spaces), log NAME, limit SECS
set -o pipefail
TAG=${1:?TAG}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O
T=heterogeneous-spmv_amd/tools
export PYTHONUNBUFFERED=1
bash $T/host_info.sh $O/host.txt > /dev/null 2>&1

run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; (cd $R && timeout -k 10 $secs "$@") > $O/$name.log 2>&1; local rc=$?
  echo "   rc=$rc"; tail -4 $O/$name.log | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: $name rc=$rc"; exit $rc; fi
}
PYT=(python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider)

for step in "$@"; do
  kind=${step%%:*}; arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  case $kind in
    gputest)
      if [ -n "$arg" ]; then run gputest 900 "${PYT[@]}" tests -m gpu -k "$arg"
      else run gputest 900 "${PYT[@]}" tests -m gpu; fi ;;
    tests)
      files=${arg%%:*}; k=""; [ "$files" != "$arg" ] && k=${arg#*:}
      if [ -n "$k" ]; then run tests 600 "${PYT[@]}" ${files//,/ } -k "$k"
      else run tests 600 "${PYT[@]}" ${files//,/ }; fi ;;
    smoke)
      run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      run bench 400 python bench.py ${arg//,/ }
      grep '^{' $O/bench.log | cut -c1-1200 ;;
    rocprof)
      echo "== rocprof"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
        --output-format csv -d $O/prof_bench -o bench -- python3 $R/bench.py ${arg//,/ }) \
        > $O/rocprof_bench.log 2>&1
      rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/rocprof_bench.log; exit $rc; }
      cp $O/prof_bench/*kernel_stats.csv $O/bench_kernel_stats.csv 2>/dev/null
      head -6 $O/bench_kernel_stats.csv | cut -c1-200 ;;
    rocprofleg)
      echo "== rocprofleg"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace \
        --kernel-rename --stats --output-format csv -d $O/prof_leg -o bench -- python3 $R/bench.py ${arg//,/ }) \
        > $O/rocprof_leg.log 2>&1
      rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/rocprof_leg.log; exit $rc; }
      grep '^{' $O/rocprof_leg.log > $O/bench_leg.json
      cp $O/prof_leg/*kernel_stats.csv $O/bench_leg_kernel_stats.csv 2>/dev/null
      head -12 $O/bench_leg_kernel_stats.csv | cut -c1-200 ;;
    kstat1)
      name=${arg%%:*}; rargs=${arg#*:}
      echo "== kstat1 $name"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $O/prof_$name -o run -- python3 $R/$T/run_one.py ${rargs//;/ }) > $O/${name}_run.log 2>&1
      rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/${name}_run.log; exit $rc; }
      grep '^{' $O/${name}_run.log | cut -c1-300
      cp $O/prof_$name/*kernel_stats.csv $O/${name}_kernel_stats.csv 2>/dev/null ;;
    kstats)
      run kstats 1200 bash $T/gpu_kstats.sh $TAG "${arg//,/ }" ;;
    pmc)
      run pmc_$arg 900 bash $T/gpu_pmc_bench.sh ${TAG}_$arg "--config $arg" ;;
    ab)
      run ab 900 python $T/ab.py ${arg//;/ } ;;
    py)
      name=${arg%%:*}; rest=${arg#*:}; secs=${rest%%:*}; pargs=${rest#*:}
      run $name $secs python ${pargs//;/ } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
