#!/usr/bin/env python3
"""Handle creation time (host planning + upload + derived tables) per
config: what a caller pays once before the first SpMV (the reference's
drivers print their preprocessing time the same way, e.g. "reordered in").

    python heterogeneous-spmv_amd/tools/create_time.py [--configs c3,c5,c4p1,c3h,c2]
"""
import argparse
import json
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent))

import torch  # noqa: E402,F401  (load order: torch's HIP runtime first)

import hspmv  # noqa: E402
from sweep import build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c5,c5r,c4p1,c3h,c2")
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    for cfg in a.configs.split(","):
        t0 = time.perf_counter()
        A, maps, desc = build(cfg)
        gen_s = time.perf_counter() - t0
        times = []
        for _ in range(a.repeat):
            t0 = time.perf_counter()
            op = hspmv.SpMV(A, maps, device=0)
            op.synchronize()
            times.append(time.perf_counter() - t0)
            info = op.info
            op.close()
        print(json.dumps({"config": cfg, "m": A.m, "nnz": A.nnz, "kernel": info["kernel_name"],
                          "x_dict": info["x_dict"], "csort_parts": info["csort_parts"],
                          "create_s": [round(t, 3) for t in times], "generate_s": round(gen_s, 2),
                          "desc": desc}), flush=True)


if __name__ == "__main__":
    main()
