#!/usr/bin/env python3
"""Runs ONE (config, variant) SpMV for a fixed number of launches -- the
workload under rocprofv3 --pmc / --kernel-trace passes.

    python heterogeneous-spmv_amd/tools/run_one.py --config c3 --kernel stream --u 4 --iters 50
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))

import hspmv  # noqa: E402
from hspmv import gen  # noqa: E402
from sweep import build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--u", type=int, default=0)
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--pf", action="store_true")
    ap.add_argument("--nt", action="store_true")
    ap.add_argument("--noxcd", action="store_true")
    ap.add_argument("--mi355x-maps", action="store_true")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--options", default="", help='hspmv_options as JSON, e.g. {"deterministic": 2}')
    ap.add_argument("--cold", type=int, default=0,
                    help="also time N launches each after a 512 MiB read (Infinity Cache evicted)")
    a = ap.parse_args()
    A, maps, desc = build(a.config)
    if a.kernel == "csr3" and (maps is None or a.mi355x_maps):
        maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "mi355x"))
    if a.kernel != "csr3" and a.kernel != "auto":
        maps = None
    op = hspmv.SpMV(A, maps, kernel=a.kernel, chunk_u=a.u, lanes=a.lanes, prefetch=a.pf,
                    nontemporal=a.nt, xcd_remap=False if a.noxcd else None,
                    options=json.loads(a.options) if a.options else None)
    op.set_x(gen.rand_x(A.n, 42).astype(A.val.dtype))
    t = op.run(warmup=3, iters=a.iters)
    b = op.info["alg_bytes"]  # x counted as the distinct columns read
    out = {"config": a.config, "desc": desc, "info": op.info, "t_min_us": t["t_min"] * 1e6,
           "t_avg_us": t["t_avg"] * 1e6, "alg_bytes": b, "gbps_min": b / t["t_min"] * 1e-9,
           "gbps_avg": b / t["t_avg"] * 1e-9}
    if a.cold:
        # cold: a 512 MiB read before every launch evicts the 256 MiB
        # Infinity Cache; each launch timed alone by the library's events
        import torch
        flush = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
        cold = []
        for _ in range(a.cold):
            flush.sum()
            torch.cuda.synchronize()
            cold.append(op.run(warmup=0, iters=1)["t_min"])
        del flush
        med = float(np.median(cold))
        out.update({"cold_us": med * 1e6, "cold_min_us": min(cold) * 1e6, "gbps_cold": b / med * 1e-9})
    print(json.dumps(out))
    op.close()


if __name__ == "__main__":
    main()
