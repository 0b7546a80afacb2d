#!/usr/bin/env python3
"""Tabulates a gpu_pmc.sh output directory: per case the kernel time, the
algorithmic bytes, the FETCH_SIZE/WRITE_SIZE traffic (raw and with the gfx950
x2 FETCH correction of MI355X_MICROARCH.md §HBM) and the L2 hit rate.

    python heterogeneous-spmv_amd/tools/pmc_table.py gpurun_out/pmc1 [-o profiles/x.json]
"""
import argparse
import csv
import glob
import json
from pathlib import Path


def per_dispatch_mean(d, counters, substr="hspmv"):
    f = glob.glob(str(d) + "/*counter_collection.csv")[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if substr not in r["Kernel_Name"] or r["Counter_Name"] not in counters:
            continue
        vals.setdefault(r["Counter_Name"], {}).setdefault(int(r["Dispatch_Id"]), 0.0)
        vals[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("-o", "--out", default="")
    a = ap.parse_args()
    rows = []
    for args_file in sorted(Path(a.dir).glob("case*.args")):
        case = args_file.with_suffix("")
        js = json.loads(Path(str(case) + ".json").read_text().strip().splitlines()[-1])
        fetch = per_dispatch_mean(case / "fetch", ["FETCH_SIZE"])["FETCH_SIZE"] * 1024
        write = per_dispatch_mean(case / "write", ["WRITE_SIZE"])["WRITE_SIZE"] * 1024
        h = per_dispatch_mean(case / "hit", ["TCC_HIT_sum", "TCC_MISS_sum"])
        alg = js["alg_bytes"]
        rec = {"args": args_file.read_text().strip(), "t_min_us": round(js["t_min_us"], 2),
               "alg_bytes": alg, "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
               "hbm_bytes_corrected": 2 * fetch + write,
               "corrected_over_alg": round((2 * fetch + write) / alg, 3),
               "raw_over_alg": round((fetch + write) / alg, 3),
               "l2_hit": round(h["TCC_HIT_sum"] / (h["TCC_HIT_sum"] + h["TCC_MISS_sum"]), 3),
               "kernel": js["info"]["kernel_name"], "chunk_u": js["info"]["chunk_u"]}
        rows.append(rec)
        print(json.dumps(rec))
    if a.out:
        Path(a.out).write_text(json.dumps(rows, indent=1) + "\n")


if __name__ == "__main__":
    main()
