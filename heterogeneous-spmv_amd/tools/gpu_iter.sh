# GPU-box pass for one development iteration: selected GPU tests, then a
# rocprofv3 kernel trace of tools/run_one.py for each listed config.
# Usage (from the repo root):
#   bash heterogeneous-spmv_amd/tools/gpu_iter.sh TAG "<pytest args>" "<cfg> <cfg> ..." [run_one args]
set -o pipefail
TAG=${1:-r02}; PT=${2:-}; CFGS=${3:-}; RARGS=${4:-}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O
export PYTHONUNBUFFERED=1
if [ -n "$PT" ]; then
  echo "== pytest $PT"
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $PT > $O/pytest.log 2>&1
  rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -40; [ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
for cfg in $CFGS; do
  name=${cfg//:/_}
  echo "== $cfg"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o run \
    -- python3 $R/heterogeneous-spmv_amd/tools/run_one.py --config $cfg --iters 100 --cold 20 $RARGS \
    > $O/${name}_run.log 2>&1 || { tail -20 $O/${name}_run.log; exit 1; }
  grep '^{' $O/${name}_run.log > $O/${name}_run.json
  cp $O/prof_$name/*kernel_stats.csv $O/${name}_kernel_stats.csv
  python3 -c "
import json,csv,sys
d=json.load(open('$O/${name}_run.json'))
print({k: d[k] for k in ('config','t_min_us','t_avg_us','cold_us','gbps_min') if k in d}, d['info']['kernel_name'])
for r in csv.DictReader(open('$O/${name}_kernel_stats.csv')):
    print('   ', r['Name'][:90], r['Calls'], r['AverageNs'])
"
done
