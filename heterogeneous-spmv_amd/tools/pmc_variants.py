#!/usr/bin/env python3
"""Per-handle counters of one ab.py run (--rounds 1) under rocprofv3 --pmc.

ab.py launches, in order: one SpMV per handle (the y check), then for each
handle 3 warm-up + ITERS timed SpMVs.  The hspmv_ dispatches of every pass
are taken in dispatch order, the first n_handles dropped, and the rest cut
into n_handles groups of 3 + ITERS; each handle's counters are the mean over
its timed launches (x launches_per_spmv).  The timed groups are the
last n_handles x (3 + ITERS) x lps dispatches.

    python heterogeneous-spmv_amd/tools/pmc_variants.py DIR --names a,b,c --iters 30 [--lps 1]
"""
import argparse
import csv
import glob
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--names", required=True)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--lps", type=int, default=1, help="launches per SpMV")
    ap.add_argument("--alg-bytes", type=float, default=0.0)
    a = ap.parse_args()
    names = a.names.split(",")
    nh = len(names)
    per = {n: defaultdict(float) for n in names}
    for f in sorted(glob.glob(a.dir + "/p*/*counter_collection.csv")):
        disp = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if "hspmv_" not in r["Kernel_Name"]:
                continue
            d = disp[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        g = (3 + a.iters) * a.lps
        if len(disp) < nh * g:
            raise SystemExit(f"{f}: {len(disp)} dispatches, expected >= {nh * g}")
        ids = sorted(disp)[-nh * g:]  # the timed rounds come last
        for i, n in enumerate(names):
            timed = ids[i * g + 3 * a.lps:(i + 1) * g]
            for c in disp[timed[0]]:
                per[n][c] = sum(disp[k][c] for k in timed) / a.iters
    for n in names:
        c = dict(per[n])
        rd = 128 * c.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) + \
            32 * c.get("TCC_EA0_RDREQ_32B_sum", 0)
        wr = 1024 * c.get("WRITE_SIZE", 0)
        rec = {"variant": n, "read_bytes_rdreq": round(rd), "write_bytes": round(wr),
               "traffic": round(rd + wr),
               "counters": {k: round(v, 1) for k, v in sorted(c.items())}}
        if a.alg_bytes:
            rec["traffic_over_alg"] = round((rd + wr) / a.alg_bytes, 4)
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
