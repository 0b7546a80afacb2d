#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into HBM bytes per SpMV launch.

Usage:
  pmc_summary.py --fetch DIR_OR_CSV --write DIR_OR_CSV [--rdreq DIR_OR_CSV]
                 --workload KEY [--kernel-substr hspmv_csr] [--skip-first N]
                 [--take N] [--alg-bytes B] -o profiles/rNN_<workload>_pmc.json

With --rdreq (a pass of TCC_EA0_RDREQ_128B_sum, _64B_sum, _32B_sum) the read
bytes come from the size-resolved fabric requests, 128*n128 + 64*n64 +
32*n32 -- the calibration the guide asks for ("other access widths are
uncalibrated: calibrate on a known byte count"): on this kernel's dword +
dwordx2 streams it equals the known byte count exactly
(profiles/r01_pmc7_probe_vs_kernels: seg_read<2> 629.1 MB = 52.4 M x 12 B),
while 2*FETCH_SIZE reads 0.72-1.0x of it.  Both are recorded; traffic uses
the calibrated one.

Counters are collected in separate passes (FETCH_SIZE uses 3 TCC slots,
WRITE_SIZE 2: MI355X_MICROARCH.md, rocprofv3 PMC slots) and corrected as that
guide's HBM section prescribes: both are in KiB; on gfx950 FETCH_SIZE reports
1/2 of the bytes of a wide coalesced streaming read, so it is doubled:
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
FETCH_SIZE counts L2->fabric requests, so Infinity-Cache hits are included.
"""
from __future__ import annotations

import argparse
import csv
import json
from pathlib import Path


def find_csv(p: str) -> Path:
    path = Path(p)
    if path.is_file():
        return path
    c = sorted(path.rglob("*counter_collection.csv"))
    if not c:
        raise SystemExit(f"no *counter_collection.csv under {p}")
    return c[0]


def per_dispatch(csv_path: Path, counter: str, substr: str):
    vals = {}
    with open(csv_path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            if substr not in row.get("Kernel_Name", ""):
                continue
            d = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or len(vals))
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--rdreq", default="")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--kernel-substr", default="hspmv_csr")
    ap.add_argument("--skip-first", type=int, default=0)
    ap.add_argument("--take", type=int, default=0)
    ap.add_argument("--last", type=int, default=0, help="use only the last N dispatches")
    ap.add_argument("--skip-last", type=int, default=0, help="drop the last N dispatches")
    ap.add_argument("--alg-bytes", type=float, default=0.0)
    ap.add_argument("--per-spmv", type=int, default=1,
                    help="consecutive matching dispatches that form one SpMV (summed)")
    ap.add_argument("--extra", default="",
                    help="a pass with any other counters: each is reported per SpMV")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    fc, wc = find_csv(a.fetch), find_csv(a.write)
    K = max(1, a.per_spmv)

    def sel(v):
        v = [sum(v[i:i + K]) for i in range(0, len(v) - K + 1, K)]
        v = v[a.skip_first:]
        if a.skip_last:
            v = v[:-a.skip_last]
        if a.last:
            v = v[-a.last:]
        if a.take:
            v = v[:a.take]
        return v

    f = sel(per_dispatch(fc, "FETCH_SIZE", a.kernel_substr))
    w = sel(per_dispatch(wc, "WRITE_SIZE", a.kernel_substr))
    if not f or not w:
        raise SystemExit("no matching dispatches")
    fetch_kib = sum(f) / len(f)
    write_kib = sum(w) / len(w)
    hbm_guide = (2.0 * fetch_kib + write_kib) * 1024.0
    out = {"workload": a.workload, "kernel_substr": a.kernel_substr,
           "dispatches": [len(f), len(w)], "fetch_size_kib": fetch_kib,
           "write_size_kib": write_kib, "hbm_bytes_guide": hbm_guide,
           "hbm_bytes_per_launch": hbm_guide,
           "correction": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE = 1/2 streamed bytes)",
           "source": f"rocprofv3 --pmc FETCH_SIZE ({fc.name}) / --pmc WRITE_SIZE ({wc.name})"}
    if a.rdreq:
        rc = find_csv(a.rdreq)
        n = {}
        for sz in (128, 64, 32):
            v = sel(per_dispatch(rc, f"TCC_EA0_RDREQ_{sz}B_sum", a.kernel_substr))
            n[sz] = sum(v) / len(v) if v else 0.0
        rd = 128.0 * n[128] + 64.0 * n[64] + 32.0 * n[32]
        out.update({"rdreq_128b": n[128], "rdreq_64b": n[64], "rdreq_32b": n[32],
                    "read_bytes_rdreq": rd, "hbm_bytes_per_launch": rd + write_kib * 1024.0,
                    "correction": "128*RDREQ_128B + 64*RDREQ_64B + 32*RDREQ_32B + WRITE_SIZE*1024 "
                                  "(size-resolved fabric reads, calibrated on a known byte count)",
                    "source": f"rocprofv3 --pmc TCC_EA0_RDREQ_{{128B,64B,32B}}_sum ({rc.name}) / "
                              f"--pmc WRITE_SIZE ({wc.name}); FETCH_SIZE ({fc.name}) kept as hbm_bytes_guide"})
    if a.extra:
        ec = find_csv(a.extra)
        names = set()
        with open(ec) as f:
            for row in csv.DictReader(f):
                if a.kernel_substr in row.get("Kernel_Name", ""):
                    names.add(row["Counter_Name"])
        ex = {}
        for nm in sorted(names):
            v = sel(per_dispatch(ec, nm, a.kernel_substr))
            if v:
                ex[nm] = sum(v) / len(v)
        out["extra_counters_per_spmv"] = ex
        out["extra_source"] = ec.name
    out["dispatches_per_spmv"] = K
    hbm = out["hbm_bytes_per_launch"]
    if a.alg_bytes:
        out["alg_bytes_per_launch"] = a.alg_bytes
        out["traffic_over_alg"] = hbm / a.alg_bytes
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
