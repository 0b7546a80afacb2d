# GPU-box: where the y-store cost of a streaming SpMV goes -- TCP / TCC / SQ
# counters of bw_probe6's base (no stores) and y.wave kernels (reg_only set),
# one rocprofv3 --pmc pass each.
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/gpu_pmc_ystore.sh TAG
set -o pipefail
TAG=${1:-ystore}
R=$GRAFT_REPO_ROOT; D=$R/gpurun_out/$TAG; mkdir -p $D
B=$R/heterogeneous-spmv_amd/build/probes/bw_probe6
cd /tmp && export TMPDIR=/tmp
P=(
 "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum"
 "TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum"
 "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_WR"
 "TCC_BUSY_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum"
 "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TOTAL_WRITE_sum"
)
i=0
for pass in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $D/p$i -o y -- $B 27 8388608 1 > $D/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $pass"
  case $rc in 0) ;; *) echo "fatal rc=$rc"; exit $rc;; esac
done
