# GPU-box: arbitrary PMC passes for run_one.py cases.
# Usage: bash .../gpu_pmc2.sh TAG "PASS1 COUNTERS;PASS2 COUNTERS;..." "ARGS1" "ARGS2" ...
set -o pipefail
TAG=$1; PASSES=$2; shift 2
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/$TAG
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
i=0
for args in "$@"; do
  i=$((i+1)); D=$R/gpurun_out/$TAG/case$i
  echo "== case$i: $args"; echo "$args" > $D.args 2>/dev/null || { mkdir -p $D; echo "$args" > $D.args; }
  timeout -k 10 300 python3 $R/heterogeneous-spmv_amd/tools/run_one.py $args > $D.json 2>&1 || exit 1
  p=0
  IFS=';' read -ra PS <<< "$PASSES"
  for pass in "${PS[@]}"; do
    p=$((p+1))
    timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $D/p$p -o run -- python3 $R/heterogeneous-spmv_amd/tools/run_one.py $args > $D.p$p.log 2>&1
    rc=$?
    case $rc in 124|134|137|139) echo "fatal rc=$rc on pass $p"; exit $rc;; esac
    echo "  pass $p ($pass): rc=$rc"
  done
done
