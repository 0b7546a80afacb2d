#!/usr/bin/env python3
"""Per-kernel, per-dispatch mean of every counter in a rocprofv3 --pmc output
tree (any kernels; counters from several passes merged by kernel name).

    python heterogeneous-spmv_amd/tools/pmc_kernels.py gpurun_out/TAG/probe640
"""
import csv
import glob
import json
import re
import sys

vals = {}
for f in glob.glob(sys.argv[1] + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))
        m = re.search(r"seg_read<(\d+), (\w+)>", r["Kernel_Name"])
        if m:
            k = f"seg_read<{m.group(1)},{m.group(2)}>"
        d = vals.setdefault(k, {}).setdefault(r["Counter_Name"], {})
        d[int(r["Dispatch_Id"])] = d.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
for k, cs in vals.items():
    print(json.dumps({"kernel": k, "counters": {c: sum(v.values()) / len(v) for c, v in cs.items()}}))
