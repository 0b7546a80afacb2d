#!/bin/bash
# GPU-box pass (round 4 w): L1 gather calibration (tools/probes/gather_probe.hip):
# timing per address pattern, then two rocprofv3 --pmc passes over the same
# binary (TCP / GRBM, then TD / TCC / SQ), summarised per kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04w; mkdir -p $O
cd $R/heterogeneous-spmv_amd || exit 1
timeout -k 10 120 /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probes/gather_probe.hip -o $O/gather_probe || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $O/gather_probe > $O/timing.jsonl 2> $O/timing.err || exit $?
cat $O/timing.jsonl
P=(
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
 "TD_TD_BUSY_sum TD_TC_STALL_sum TCC_REQ_sum TCC_HIT_sum SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD"
)
i=0
for pass in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $pass --output-format csv -d $O/pmc/p$i -o run -- $O/gather_probe > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $pass"
  case $rc in 0) ;; *) echo "stop rc=$rc"; exit $rc;; esac
done
python3 $R/heterogeneous-spmv_amd/tools/pmc_kernels.py $O/pmc > $O/pmc_per_kernel.jsonl && cut -c1-300 $O/pmc_per_kernel.jsonl
