# GPU-box PMC diagnosis of C3's box-dependent traffic: address-translation
# (UTCL1) and DRAM-vs-total fabric read counters per launch, for plain and
# physically contiguous (HSPMV_CONTIG=1) allocations.  Two passes each.
# Usage (from the repo root): bash heterogeneous-spmv_amd/tools/gpu_pmc_tlb.sh TAG
set -o pipefail
TAG=${1:-tlb}
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/$TAG; mkdir -p $O
export PYTHONUNBUFFERED=1
RUN="python3 $R/heterogeneous-spmv_amd/tools/run_one.py --config c3 --iters 50"
cd /tmp && export TMPDIR=/tmp
for V in plain contig; do
  if [ $V = contig ]; then export HSPMV_CONTIG=1; else unset HSPMV_CONTIG; fi
  echo "== $V tcp" && timeout -k 10 -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d $O/$V/tcp -o run -- $RUN > $O/${V}_tcp.log 2>&1 &&
  echo "== $V tcc" && timeout -k 10 -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/$V/tcc -o run -- $RUN > $O/${V}_tcc.log 2>&1 || exit 1
done
cd $R && python3 - "$O" <<'PY'
import csv, glob, json, sys, collections
O = sys.argv[1]
out = {}
for v in ("plain", "contig"):
    per = collections.defaultdict(list)
    for f in glob.glob(f"{O}/{v}/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "hspmv_csr3" in r["Kernel_Name"]:
                per[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out[v] = {k: sum(x[-40:]) / len(x[-40:]) for k, x in per.items() if x}
print(json.dumps(out, indent=1))
json.dump(out, open(f"{O}/summary.json", "w"), indent=1)
PY
