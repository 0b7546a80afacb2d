# GPU-box: stall / pipeline counters of the C5 column-sorted kernel (one
# rocprofv3 --pmc pass each, run_one.py c5), to find what bounds the sweep.
# Usage: bash heterogeneous-spmv_amd/tools/gpu_pmc_c5.sh TAG [run_one args]
set -o pipefail
TAG=${1:-c5pmc}; shift
ARGS=${*:-"--config c5 --iters 30"}
R=$GRAFT_REPO_ROOT; D=$R/gpurun_out/$TAG; mkdir -p $D
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
P=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_RD"
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
 "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
 "TD_TD_BUSY_sum TD_TC_STALL_sum TCC_BUSY_sum TCC_TAG_STALL_sum TCC_REQ_sum TCC_HIT_sum"
 "SQ_WAVES SQ_CYCLES SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
)
timeout -k 10 300 python3 $R/heterogeneous-spmv_amd/tools/run_one.py $ARGS > $D/run.json 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- python3 $R/heterogeneous-spmv_amd/tools/run_one.py $ARGS > $D/kt.log 2>&1 || exit 1
i=0
for pass in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $D/p$i -o run -- python3 $R/heterogeneous-spmv_amd/tools/run_one.py $ARGS > $D/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $pass"
  case $rc in 124|134|137|139) echo "fatal rc=$rc"; exit $rc;; esac
done
