# GPU-box: quick sweep with the normal library and the three ablation builds.
set -o pipefail
CFG=${1:-c3,c4,b27}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for d in 0 1 2 3; do
  if [ $d -eq 0 ]; then unset HSPMV_LIB; else export HSPMV_LIB=$R/heterogeneous-spmv_amd/build/diag$d/libhspmv.so; fi
  echo "== diag $d"
  timeout -k 10 600 python heterogeneous-spmv_amd/tools/sweep.py --configs $CFG --quick --out gpurun_out/diag_$d.jsonl > gpurun_out/diag_$d.log 2>&1 || { tail -5 gpurun_out/diag_$d.log; exit 1; }
done
