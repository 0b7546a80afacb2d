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

import torch  # noqa: E402,F401  (device arrays shared by all variants)

import hspmv  # noqa: E402
from hspmv import dist as hdist  # noqa: E402
from hspmv import gen  # noqa: E402

PEAK = 8000.0


def build(cfg):
    if cfg.endswith(":f32"):  # any config in fp32 (the reference's own dtype)
        A, maps, desc = build(cfg[:-4])
        return A.astype(np.float32), maps, desc + " [fp32]"
    if cfg == "c2":
        A = gen.laplace2d(1000, 1000)
        return A, None, "C2 5-pt Laplacian 1000^2 CSR fp64"
    if cfg == "c3":
        A = gen.stencil27(125)
        maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "volta"))
        return A, maps, "C3 27-pt 125^3 RCM CSR-3 fp64 (ssrs=20, srs=10)"
    if cfg == "c3m":  # C3's matrix with the MI355X CSR-3 grouping (64, 4)
        A = gen.stencil27(125)
        maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "mi355x"))
        return A, maps, "C3 27-pt 125^3 RCM CSR-3 fp64 (mi355x grouping ssrs=64, srs=4)"
    if cfg.startswith("c2s"):  # C2's matrix, CSR-3 grouping (ssrs, srs) = c2s<ssrs>x<srs>
        ssrs, srs = (int(v) for v in cfg[3:].split("x"))
        A = gen.laplace2d(1000, 1000)
        return A, hspmv.build_csr3_maps(A, ssrs, srs), f"C2 CSR-3 fp64 (ssrs={ssrs}, srs={srs})"
    if cfg.startswith("c3s"):  # C3's matrix, CSR-3 grouping (ssrs, srs) = c3s<ssrs>x<srs>
        ssrs, srs = (int(v) for v in cfg[3:].split("x"))
        A = gen.stencil27(125)
        maps = hspmv.build_csr3_maps(A, ssrs, srs)
        return A, maps, f"C3 27-pt 125^3 RCM CSR-3 fp64 (ssrs={ssrs}, srs={srs})"
    if cfg in ("c3g", "c4g"):  # CSR-3 maps with exactly STREAM's 64-row groups, 4 per block
        A = gen.stencil27(125) if cfg == "c3g" else hdist.build_shard("c4", 0, 8).A
        inner = np.append(np.arange(0, A.m, 64), A.m).astype(np.int32)
        nsr = len(inner) - 1
        outer = np.append(np.arange(0, nsr, 4), nsr).astype(np.int32)
        return A, hspmv.Csr3Maps(outer, inner), f"{cfg}: CSR-3 maps = 64-row groups x 4"
    if cfg.startswith("c4s"):  # C4's shard, CSR-3 grouping c4s<ssrs>x<srs>
        ssrs, srs = (int(v) for v in cfg[3:].split("x"))
        sh = hdist.build_shard("c4", 0, 8)
        return sh.A, hspmv.build_csr3_maps(sh.A, ssrs, srs), f"C4 shard CSR-3 ({ssrs}, {srs})"
    if cfg == "c4":
        sh = hdist.build_shard("c4", 0, 8)
        return sh.A, None, "C4 banded 2e7 rows, rank-0 shard of 8 (2.5M rows) fp64"
    if cfg.startswith("c4p"):  # C4's rank-0 shard at P ranks (c4p2 / c4p4), or the whole (c4p1)
        P = int(cfg[3:])
        sh = hdist.build_shard("c4", 0, P)
        return sh.A, None, f"C4 banded 2e7 rows, rank-0 shard of {P} fp64"
    if cfg == "b27":  # diagnostic: C3's row length with a C4-like (local) gather
        A = gen.banded(1_953_125, per_row=27, half=32, seed=5)
        return A, None, "diag: banded 1.95M rows, 27 nnz/row within +-32, fp64"
    if cfg == "s27n":  # diagnostic: C3's stencil in natural (non-RCM) order
        A = gen.stencil27(125, rcm=False)
        return A, None, "diag: 27-pt 125^3 natural order fp64"
    if cfg == "l4k":  # diagnostic: HBM-resident 5-pt Laplacian (three x windows per group)
        A = gen.laplace2d(4000, 4000)
        return A, None, "diag: 5-pt Laplacian 4000^2 CSR fp64 (HBM-resident)"
    if cfg in ("c3h", "c3hm"):  # DIMACS10 hugebubbles-00000 stand-in (degree-3 mesh, RCM)
        A = gen.honeycomb(4280, 4280)
        if cfg == "c3h":
            return A, None, "C3 alt: honeycomb 4280^2 RCM (18.3M rows, 54.9M nnz) CSR fp64"
        maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "volta"))
        return A, maps, "C3 alt: honeycomb 4280^2 RCM CSR-3 fp64 (volta grouping)"
    if cfg.startswith("d") and cfg[1:].isdigit():  # mid/high density band: d<k> nnz per row
        k = int(cfg[1:])
        m = max(50_000_000 // k, 1000)
        A = gen.banded(m, per_row=k, half=k, seed=21, chunk=max((1 << 22) // (2 * k + 1), 256))
        return A, None, f"density band: {m} rows x {k} nnz within +-{k}, CSR fp64 (~50M nnz)"
    if cfg == "mix":  # SuiteSparse-like mixed row lengths (Pareto, 8..4000), band +-4000
        import scipy.sparse as sp
        rng = np.random.default_rng(31)
        m = 1_000_000
        lens = np.minimum((8 * (rng.pareto(1.2, m) + 1)).astype(np.int64), 4000)
        rows = np.repeat(np.arange(m, dtype=np.int64), lens)
        ci = np.clip(rows + rng.integers(-4000, 4001, rows.shape[0]), 0, m - 1)
        S = sp.csr_matrix((rng.uniform(-1, 1, ci.shape[0]), (rows, ci)), shape=(m, m))
        S.sum_duplicates()
        S.sort_indices()
        A = hspmv.CsrMatrix.from_scipy(S, np.float64)
        return A, None, (f"mixed rows: {m} rows, Pareto lengths 8..4000 (mean {A.nnz / m:.0f}), "
                         "band +-4000, CSR fp64")
    if cfg in ("c5", "c5r"):  # c5r: the same matrix RCM-permuted (helpers/converter.m:8,14)
        A = gen.powerlaw(2_000_000, seed=1234, dtype=np.float32, rcm=cfg == "c5r")
        maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "mi355x"))
        return A, maps, "C5 power-law 2e6 rows CSR-3 fp32" + (" RCM-permuted" if cfg == "c5r" else "")
    import auto_regret  # the planner-regret zoo's shapes (urand8, diag, tall, ...)
    if cfg in auto_regret.EXTRA:
        return auto_regret.build(cfg)
    raise ValueError(cfg)


class DeviceMatrix:
    """One device copy of A (+ x, y) in torch tensors; handles borrow it."""

    def __init__(self, A, x):
        import torch
        self.torch = torch
        self.A = A
        self.rp = torch.from_numpy(A.row_ptr).cuda()
        self.ci = torch.from_numpy(A.col_idx).cuda()
        self.val = torch.from_numpy(A.val).cuda()
        self.x = torch.from_numpy(np.ascontiguousarray(x)).cuda()
        self.y = torch.empty(A.m, dtype=self.val.dtype, device="cuda")
        self.maps = {}

    def spmv(self, maps, **kw):
        torch = self.torch
        meta = hspmv.CsrMatrix(self.A.m, self.A.n, np.zeros(1, np.int32), np.zeros(0, np.int32),
                               np.zeros(0, self.A.val.dtype))
        cs = hspmv._lib.Csr(self.A.m, self.A.n, self.A.nnz, self.rp.data_ptr(), self.ci.data_ptr(),
                            self.val.data_ptr(), hspmv.api.dtype_code(self.A.val.dtype))
        mdev = None
        if maps is not None:
            key = id(maps)
            if key not in self.maps:
                self.maps[key] = (torch.from_numpy(maps.outer).cuda(),
                                  torch.from_numpy(maps.inner).cuda(), maps)
            o, i, _ = self.maps[key]
            mdev = hspmv._lib.Csr3Maps(maps.n_ssr, maps.n_sr, o.data_ptr(), i.data_ptr())
        op = hspmv.SpMV.from_device(cs, mdev, meta, device=0, **kw)
        op.bind_x_device(self.x.data_ptr())
        op.bind_y_device(self.y.data_ptr())
        return op


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
    v.append(("stream-auto-xcd", dict(kernel="stream", xcd_remap=True), None))
    v.append((tag3 + "-auto-xcd", dict(kernel="csr3", xcd_remap=True), m3))
    v.append(("stream-auto-nt", dict(kernel="stream", nontemporal=True), None))
    v.append(("stream-auto-c32", dict(kernel="stream", col16=False), None))
    v.append((tag3 + "-auto-c32", dict(kernel="csr3", col16=False), m3))
    if cfg == "c5":
        v.append(("stream-nosplit", dict(kernel="stream", split_rows=False), None))
    return v


def xcd_variants(A, maps):
    d = A.nnz / A.m
    m3 = maps if maps is not None else hspmv.build_csr3_maps(A, *hspmv.csr3_params(d, "mi355x"))
    v = [("stream-auto", dict(kernel="stream"), None), ("csr3-auto", dict(kernel="csr3"), m3),
         ("stream-xcdfull", dict(kernel="stream", xcd_remap=True), None),
         ("csr3-xcdfull", dict(kernel="csr3", xcd_remap=True), m3)]
    for s in (1, 2, 4, 8, 16, 32, 64, 128):
        v.append((f"stream-xcd{s}", dict(kernel="stream", xcd_chunk=s), None))
        v.append((f"csr3-xcd{s}", dict(kernel="csr3", xcd_chunk=s), m3))
    return v


def group_variants(A):
    v = [("stream-auto", dict(kernel="stream"), None)]
    for g in (1, 2, 4, 8, 16):
        for u in (0, 2, 4, 6):
            for pf in (False, True):
                name = f"stream-g{g}" + (f"-u{u}" if u else "") + ("-pf" if pf else "")
                v.append((name, dict(kernel="stream", groups_per_wave=g, chunk_u=u, prefetch=pf), None))
    return v


def short_row_variants(A):
    """STREAM launch shapes for short rows: groups per wave x chunk size x
    waves per workgroup (hspmv_options.stream_waves)."""
    v = [("stream-auto", dict(kernel="stream"), None)]
    for w in (1, 2, 4):
        for g in (1, 2, 4):
            for u in (0, 2, 4):
                name = f"stream-w{w}-g{g}" + (f"-u{u}" if u else "")
                v.append((name, dict(kernel="stream", groups_per_wave=g, chunk_u=u,
                                     options={"stream_waves": w}), None))
    return v


def waves_variants(A):
    """STREAM waves per workgroup at the planner's other choices."""
    v = [("stream-auto", dict(kernel="stream"), None)]
    for w in (1, 2, 4):
        v.append((f"stream-w{w}", dict(kernel="stream", options={"stream_waves": w}), None))
    return v


def det_variants(A, maps):
    """Deterministic handles (options deterministic=1: no csort) against AUTO:
    the row kernels with and without the CSR-3 maps, x slabs on / off."""
    v = [("auto", dict(kernel="auto"), maps)]
    for tag, mp in (("maps", maps), ("nomaps", None)):
        if tag == "maps" and maps is None:
            continue
        v.append((f"det-{tag}", dict(kernel="auto", options={"deterministic": 1}), mp))
        v.append((f"det-{tag}-noslabs", dict(kernel="auto", options={"deterministic": 1, "x_slabs": -1}), mp))
    v.append(("det-stream", dict(kernel="stream", options={"deterministic": 1}), None))
    return v


def c16_variants(A, maps):
    """16-bit column offsets (default) vs 32-bit columns, over chunk sizes."""
    d = A.nnz / A.m
    m3 = maps if maps is not None else hspmv.build_csr3_maps(A, *hspmv.csr3_params(d, "mi355x"))
    v = []
    for c16 in (True, False):
        t = "" if c16 else "-c32"
        for u in (0, 2, 3, 4, 6, 8):
            tag = f"-u{u}" if u else "-auto"
            v.append((f"stream{tag}{t}", dict(kernel="stream", chunk_u=u, col16=c16), None))
        v.append((f"csr3-auto{t}", dict(kernel="csr3", col16=c16), m3))
        v.append((f"stream-auto-nt{t}", dict(kernel="stream", nontemporal=True, col16=c16), None))
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4,c5")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--out", default="")
    ap.add_argument("--quick", action="store_true", help="only stream u4/u6 + csr3 auto")
    ap.add_argument("--grid", default="main", choices=["main", "xcd", "groups", "c16", "short", "waves", "det"],
                    help="xcd: the XCD chunk grid (blocks per XCD turn) at the auto chunk size")
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
        vs = {"main": lambda: variants(cfg, A, maps), "xcd": lambda: xcd_variants(A, maps),
              "groups": lambda: group_variants(A),
              "c16": lambda: c16_variants(A, maps), "short": lambda: short_row_variants(A),
              "waves": lambda: waves_variants(A), "det": lambda: det_variants(A, maps)}[a.grid]()
        if a.quick:
            vs = [v for v in vs if v[0] in ("stream-u4", "stream-u6", "stream-u8", "stream-auto",
                                          "stream-auto-noxcd", "csr3-auto", "csr3-mi355x-auto")]
        # every variant reads the SAME device arrays (borrowed pointers), so
        # the comparison is not skewed by where each copy was allocated
        dev = DeviceMatrix(A, x)
        for name, kw, mp in vs:
            op = dev.spmv(mp, **kw)
            dev.y.fill_(float("nan"))  # a row the kernel skips cannot pass
            torch.cuda.synchronize()  # the fill runs on torch's stream, the SpMV on its own
            op.spmv()
            op.synchronize()
            y = dev.y.cpu().numpy()
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
            b = op.info["alg_bytes"]  # x counted as the distinct columns read
            rec = {"config": cfg, "variant": name, "ok": ok, "m": A.m, "nnz": A.nnz,
                   "dtype": str(A.val.dtype), "kernel": op.info["kernel_name"],
                   "t_min_us": round(tmin * 1e6, 3), "t_avg_us": round(tmed * 1e6, 3),
                   "gbps_min": round(b / tmin * 1e-9, 1), "gbps_avg": round(b / tmed * 1e-9, 1),
                   "gflops_min": round(2 * A.nnz / tmin * 1e-9, 1), "frac_peak": round(b / tmin * 1e-9 / PEAK, 4),
                   "chunk_u": op.info["chunk_u"], "waves_per_block": op.info["waves_per_block"],
                   "n_split_rows": op.info["n_split_rows"], "xcd_chunk": op.info["xcd_remap"],
                   "groups": op.info["groups_per_wave"], "col16": op.info["col16"],
                   "x_slabs": op.info["x_slabs"], "x_dict": op.info["x_dict"],
                   "format_gbps_min": round(op.info["format_bytes"] / tmin * 1e-9, 1),
                   "desc": desc}
            lines.append(rec)
            print(json.dumps(rec), flush=True)
            op.close()
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in lines))


if __name__ == "__main__":
    main()
