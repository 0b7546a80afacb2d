#!/usr/bin/env python3
"""Kernel sweep over the BASELINE.json configurations on one GPU.

For every config (C2 Laplacian CSR fp64, C3 27-pt RCM CSR-3 fp64, C4 banded
per-GPU shard fp64, C5 power-law CSR-3 fp32) and every kernel variant, times
the SpMV with HIP events around each launch (hspmv_run, reference protocol)
in interleaved rounds inside ONE process (cdna_hip_programming.md §5.4 rule
24), checks y against the oracle once per variant, and prints one JSON line
per (config, variant): median/min kernel time, algorithmic GB/s, GFLOP/s and
fraction of the 8 TB/s HBM peak.

    python heterogeneous-spmv_amd/tools/sweep.py [--configs c2,c3,c4,c5]
           [--rounds 3] [--iters 30] [--out profiles/rNN_sweep.jsonl]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(REPO / "oracle"))

import hspmv  # noqa: E402
from hspmv import dist as hdist  # noqa: E402
from hspmv import gen  # noqa: E402

PEAK = 8000.0


def build(cfg):
    if cfg == "c2":
        A = gen.laplace2d(1000, 1000)
        return A, None, "C2 5-pt Laplacian 1000^2 CSR fp64"
    if cfg == "c3":
        A = gen.stencil27(125)
        maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "volta"))
        return A, maps, "C3 27-pt 125^3 RCM CSR-3 fp64 (ssrs=20, srs=10)"
    if cfg == "c4":
        sh = hdist.build_shard("c4", 0, 8)
        return sh.A, None, "C4 banded 2e7 rows, rank-0 shard of 8 (2.5M rows) fp64"
    if cfg == "c5":
        A = gen.powerlaw(2_000_000, seed=1234, dtype=np.float32)
        maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "mi355x"))
        return A, maps, "C5 power-law 2e6 rows CSR-3 fp32"
    raise ValueError(cfg)


def variants(cfg, A, maps, full=False):
    """Kernel variants to time.  Default: the tuning grid over chunk size U,
    prefetch and XCD remap for STREAM and CSR3, plus the VECTOR widths."""
    d = A.nnz / A.m
    v = []
    lanes = [4, 8] if d < 16 else [16, 64]
    for L in lanes:
        v.append((f"vector{L}", dict(kernel="vector", lanes=L), None))
    m3 = maps if maps is not None else hspmv.build_csr3_maps(A, *hspmv.csr3_params(d, "mi355x"))
    tag3 = "csr3" if maps is not None else "csr3-mi355x"
    for u in (2, 3, 4, 6, 8):
        for pf in (False, True):
            sfx = f"-u{u}" + ("-pf" if pf else "")
            v.append(("stream" + sfx, dict(kernel="stream", chunk_u=u, prefetch=pf), None))
            v.append((tag3 + sfx, dict(kernel="csr3", chunk_u=u, prefetch=pf), m3))
    v.append(("stream-auto", dict(kernel="stream"), None))
    v.append((tag3 + "-auto", dict(kernel="csr3"), m3))
    v.append(("stream-auto-noxcd", dict(kernel="stream", xcd_remap=False), None))
    v.append((tag3 + "-auto-noxcd", dict(kernel="csr3", xcd_remap=False), m3))
    v.append(("stream-auto-nt", dict(kernel="stream", nontemporal=True), None))
    if cfg == "c5":
        v.append(("stream-nosplit", dict(kernel="stream", split_rows=False), None))
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4,c5")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import oracle
    lines = []
    for cfg in a.configs.split(","):
        t0 = time.time()
        A, maps, desc = build(cfg)
        x = gen.rand_x(A.n, 42).astype(A.val.dtype)
        y_ref = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
        absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
        print(f"# {cfg}: {desc} m={A.m} nnz={A.nnz} built in {time.time() - t0:.1f}s",
              file=sys.stderr, flush=True)
        ops = []
        for name, kw, mp in variants(cfg, A, maps):
            op = hspmv.SpMV(A, mp, **kw)
            op.set_x(x)
            op.spmv()
            y = op.get_y()
            err = np.abs(y.astype(np.float64) - y_ref.astype(np.float64))
            tol = (1e-6 if A.val.dtype == np.float64 else 1e-4) * np.abs(y_ref) + \
                  (1e-12 if A.val.dtype == np.float64 else 1e-5) * absrow
            ok = bool(np.all(err <= tol))
            ops.append((name, op, ok, mp))
        times = {name: [] for name, *_ in ops}
        for _ in range(a.rounds):
            for name, op, ok, mp in ops:
                t = op.run(warmup=3, iters=a.iters)
                times[name].append((t["t_min"], t["t_avg"]))
        for name, op, ok, mp in ops:
            tmin = min(t[0] for t in times[name])
            tmed = float(np.median([t[1] for t in times[name]]))
            nssr, nsr = (mp.n_ssr, mp.n_sr) if mp is not None else (0, 0)
            b = hspmv.alg_bytes(A.m, A.n, A.nnz, A.val.dtype, nssr, nsr)
            rec = {"config": cfg, "variant": name, "ok": ok, "m": A.m, "nnz": A.nnz,
                   "dtype": str(A.val.dtype), "kernel": op.info["kernel_name"],
                   "t_min_us": round(tmin * 1e6, 3), "t_avg_us": round(tmed * 1e6, 3),
                   "gbps_min": round(b / tmin * 1e-9, 1), "gbps_avg": round(b / tmed * 1e-9, 1),
                   "gflops_min": round(2 * A.nnz / tmin * 1e-9, 1), "frac_peak": round(b / tmin * 1e-9 / PEAK, 4),
                   "chunk_u": op.info["chunk_u"], "waves_per_block": op.info["waves_per_block"],
                   "n_split_rows": op.info["n_split_rows"], "desc": desc}
            lines.append(rec)
            print(json.dumps(rec), flush=True)
            op.close()
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in lines))


if __name__ == "__main__":
    main()
