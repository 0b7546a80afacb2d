# GPU-box pass: the texture-data (TD) cost of register loads, LDS-DMA loads
# and C5-like gathers (tools/probes/td_probe.hip), plain, then TD/TCP counters.
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/gpu_td_probe.sh TAG
set -o pipefail
TAG=${1:-td}
R=$GRAFT_REPO_ROOT; D=$R/gpurun_out/$TAG; mkdir -p $D
B=$R/heterogeneous-spmv_amd/build/probes/td_probe
timeout -k 10 120 $B > $D/td.jsonl 2> $D/td.err || { cat $D/td.err; exit 1; }
cat $D/td.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o td -- $B > $D/kt.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $D/p1 -o td -- $B > $D/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD --output-format csv -d $D/p2 -o td -- $B > $D/p2.log 2>&1 || exit 1
echo done
