#!/usr/bin/env python3
"""Cold-launch A/B of launch shapes in ONE process.

    python heterogeneous-spmv_amd/tools/cold_ab.py --config c2 [--rounds 20] [--out F.jsonl]

A cold launch follows a 512 MiB read that evicts the 256 MiB Infinity Cache
(bench.py's `cold` leg).  Variants of the same matrix, each its own handle:
the planner's default (XCD-contiguous block order and one-wave workgroups for
a cache-resident C2), dispatch order (xcd_remap=False), two-wave workgroups
(hspmv_options.stream_waves = 2), and both.  Rounds interleave the variants;
per variant the median / min cold launch and the warm t_min are reported,
and y is checked bitwise against the default's (the launch shape never
changes a row's sum).
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))

import torch  # noqa: E402  (load order: torch's HIP runtime first)

import hspmv  # noqa: E402
from hspmv import gen  # noqa: E402
from sweep import build  # noqa: E402

VARIANTS = [
    ("default", {}, {}),
    ("dispatch_order", {"xcd_remap": False}, {}),
    ("waves2", {}, {"stream_waves": 2}),
    ("dispatch_order+waves2", {"xcd_remap": False}, {"stream_waves": 2}),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    A, maps, desc = build(a.config)
    x = gen.rand_x(A.n, 42).astype(A.val.dtype)
    ops = []
    for name, kw, opts in VARIANTS:
        op = hspmv.SpMV(A, maps, options=opts or None, **kw)
        op.set_x(x)
        ops.append((name, op))
    ys = [op(x) for _, op in ops]
    flush = torch.ones(64 << 20, dtype=torch.float64, device="cuda")
    cold = {n: [] for n, _ in ops}
    for _ in range(a.rounds):
        for name, op in ops:
            flush.sum()
            torch.cuda.synchronize()
            cold[name].append(op.run(warmup=0, iters=1)["t_min"] * 1e6)
    out = []
    for (name, op), y in zip(ops, ys):
        warm = op.run(warmup=3, iters=50)
        info = op.info
        rec = {"config": a.config, "desc": desc, "variant": name,
               "cold_med_us": round(float(np.median(cold[name])), 3),
               "cold_min_us": round(float(np.min(cold[name])), 3),
               "warm_min_us": round(warm["t_min"] * 1e6, 3), "warm_avg_us": round(warm["t_avg"] * 1e6, 3),
               "kernel": info["kernel_name"], "waves_per_block": info["waves_per_block"],
               "xcd_remap": info["xcd_remap"], "blocks": info["blocks"],
               "y_bitwise_equal_to_default": bool(np.array_equal(y, ys[0]))}
        out.append(rec)
        print(json.dumps(rec), flush=True)
        op.close()
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in out))


if __name__ == "__main__":
    main()
