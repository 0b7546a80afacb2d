# GPU-box pass for one round checkpoint: host CPU facts, GPU tests, the
# default bench line (C3 at N = 1), and a rocprofv3 kernel trace of the same
# bench command.  Every GPU step has its own time limit; the first failure
# ends the script.
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/gpu_round.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-r02}; KEXPR=${2:-}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O
export PYTHONUNBUFFERED=1
bash heterogeneous-spmv_amd/tools/host_info.sh $O/host.txt
echo "== pytest gpu"
if [ -n "$KEXPR" ]; then KARGS=(-k "$KEXPR"); else KARGS=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARGS[@]}" > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench (default)"
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-1500
cd /tmp && export TMPDIR=/tmp
echo "== rocprofv3 kernel trace of the bench"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 $R/bench.py --no-cpu > $O/bench_trace.log 2>&1 || exit 1
cp $O/trace/*kernel_stats.csv $O/bench_kernel_stats.csv 2>/dev/null
cut -c1-200 $O/bench_kernel_stats.csv
