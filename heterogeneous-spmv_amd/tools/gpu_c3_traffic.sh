# GPU-box: C3 fabric traffic per kernel variant, one process (ab.py, diag-env
# library, --rounds 1) under separate rocprofv3 --pmc passes; pmc_variants.py
# attributes the dispatches to the handles.  Answers where C3's bytes above
# the model (tools/l2_model.py) come from, on one box.
# Usage: bash heterogeneous-spmv_amd/tools/gpu_c3_traffic.sh TAG [CONFIG]
set -o pipefail
TAG=${1:-c3traffic}; CFG=${2:-c3}
R=$GRAFT_REPO_ROOT; D=$R/gpurun_out/$TAG; mkdir -p $D
export PYTHONUNBUFFERED=1
bash $R/heterogeneous-spmv_amd/tools/host_info.sh $D/host.txt
E=$R/heterogeneous-spmv_amd/build/diagenv/libhspmv.so
V=${VARIANTS:-"$E,$E#HSPMV_PF=0,$E@16777216,$E@4194304,$E#HSPMV_XDICT=0,$E#HSPMV_NT=1,$E"}
NAMES=${VNAMES:-"default,pf0,xcd_chunk1,xcd_contig,no_xdict,nt1,default_again"}
AB="$R/heterogeneous-spmv_amd/tools/ab.py --libs $V --configs $CFG --rounds 1 --iters 30"
timeout -k 10 300 python3 $AB > $D/ab.jsonl 2> $D/ab.err || exit 1
cat $D/ab.jsonl
cd /tmp && export TMPDIR=/tmp
P=(
 "TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_REQ_sum"
 "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
 "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
 "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
 "TCC_NORMAL_EVICT_sum TCC_NORMAL_WRITEBACK_sum TCC_PROBE_sum TCC_STREAMING_REQ_sum"
)
i=0
for pass in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $D/p$i -o run -- python3 $AB > $D/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $pass"
  case $rc in 0) ;; *) echo "stop rc=$rc"; break;; esac
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- python3 $AB > $D/kt.log 2>&1 || exit 1
cd $R && python3 heterogeneous-spmv_amd/tools/pmc_variants.py $D --names $NAMES --iters 30 --alg-bytes ${ALG:-662227600} > $D/variants.jsonl && cat $D/variants.jsonl | cut -c1-400
