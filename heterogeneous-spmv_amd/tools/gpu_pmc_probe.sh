# GPU-box: the counter passes of gpu_pmc2.sh on the bandwidth probe (bw_probe2 SEG 0).
# Usage: bash .../gpu_pmc_probe.sh TAG "PASS1;PASS2;..." SEG
set -o pipefail
TAG=$1; PASSES=$2; SEG=${3:-640}
R=$GRAFT_REPO_ROOT; D=$R/gpurun_out/$TAG/probe$SEG; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
p=0
IFS=';' read -ra PS <<< "$PASSES"
for pass in "${PS[@]}"; do
  p=$((p+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $D/p$p -o run -- $R/heterogeneous-spmv_amd/build/probes/bw_probe2 $SEG 0 > $D/p$p.log 2>&1
  rc=$?
  case $rc in 124|134|137|139) echo "fatal rc=$rc on pass $p"; exit $rc;; esac
  echo "  pass $p ($pass): rc=$rc"
done
