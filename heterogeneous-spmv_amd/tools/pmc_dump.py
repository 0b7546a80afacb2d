#!/usr/bin/env python3
"""Per-dispatch mean of every counter in a gpu_pmc2.sh output dir (hspmv kernels)."""
import csv
import glob
import json
import sys
from pathlib import Path

for case in sorted(Path(sys.argv[1]).glob("case*.args")):
    d = case.with_suffix("")
    js = json.loads(Path(str(d) + ".json").read_text().strip().splitlines()[-1])
    vals = {}
    for f in glob.glob(str(d) + "/p*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "hspmv" not in r["Kernel_Name"]:
                continue
            vals.setdefault(r["Counter_Name"], {}).setdefault(int(r["Dispatch_Id"]), 0.0)
            vals[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    mean = {k: sum(v.values()) / len(v) for k, v in vals.items()}
    print(json.dumps({"args": case.read_text().strip(), "t_min_us": round(js["t_min_us"], 2),
                      "alg_bytes": js["alg_bytes"], "counters": mean}))
