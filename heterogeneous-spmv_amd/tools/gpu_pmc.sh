# GPU-box: PMC passes (FETCH_SIZE | WRITE_SIZE | TCC_HIT_sum+TCC_MISS_sum) for
# a list of run_one.py argument sets.  Usage: bash .../gpu_pmc.sh TAG "ARGS1" "ARGS2" ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/$TAG
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
i=0
for args in "$@"; do
  i=$((i+1)); D=$R/gpurun_out/$TAG/case$i
  echo "== case$i: $args" && echo "$args" > $R/gpurun_out/$TAG/case$i.args
  timeout -k 10 300 python3 $R/heterogeneous-spmv_amd/tools/run_one.py $args > $R/gpurun_out/$TAG/case$i.json 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/heterogeneous-spmv_amd/tools/run_one.py $args > /dev/null 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 $R/heterogeneous-spmv_amd/tools/run_one.py $args > /dev/null 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 $R/heterogeneous-spmv_amd/tools/run_one.py $args > /dev/null 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $D/hit -o run -- python3 $R/heterogeneous-spmv_amd/tools/run_one.py $args > /dev/null 2>&1 || exit 1
  cat $R/gpurun_out/$TAG/case$i.json | cut -c1-400
done
