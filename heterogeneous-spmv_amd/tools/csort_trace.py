#!/usr/bin/env python3
"""Per-workgroup timeline of one column-sorted (csort) launch: start / end
(s_memrealtime, 100 MHz) and XCD of every workgroup, from the diagnostic
library (build/diagenv/libhspmv.so, HSPMV_CSORT_TRACE=1).  Shows whether a
launch is bound by its slowest workgroups (a tail) or by the rate of all.

    python heterogeneous-spmv_amd/tools/csort_trace.py --configs c5,c5r [--env K=V,...] --out F.json
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))

import torch  # noqa: E402,F401  (load order: torch's HIP runtime first)

from ab import load  # noqa: E402
from hspmv import _lib, gen  # noqa: E402
from sweep import build  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c5,c5r")
    ap.add_argument("--lib", default=str(HERE.parent / "build" / "diagenv" / "libhspmv.so"))
    ap.add_argument("--env", default="", help="extra A/B knobs K=V,K=V for the handle")
    ap.add_argument("--out", default="")
    ap.add_argument("--per-wg", action="store_true", help="every workgroup + the build's cost terms")
    a = ap.parse_args()
    L = load(a.lib)
    L.hspmv_diag_csort_trace.restype = C.c_int
    L.hspmv_diag_csort_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    out = []
    for cfg in a.configs.split(","):
        A, maps, desc = build(cfg)
        x = gen.rand_x(A.n, 42).astype(A.val.dtype)
        env = {"HSPMV_CSORT_TRACE": "1"}
        env.update(dict(kv.split("=", 1) for kv in a.env.split(",") if kv))
        os.environ.update(env)
        cs, ms = A.c_struct(), (maps.c_struct() if maps is not None else None)
        h = C.c_void_p()
        assert L.hspmv_create_on_device(C.byref(h), C.byref(cs), C.byref(ms) if ms else None, 0, None, 0) == 0
        for k in env:
            os.environ.pop(k, None)
        assert L.hspmv_set_x(h, x.ctypes.data) == 0
        t = _lib.Timing()
        assert L.hspmv_run(h, 3, 10, C.byref(t)) == 0
        buf = np.zeros((4096, 3), np.uint64)
        n = L.hspmv_diag_csort_trace(h, buf.ctypes.data, 4096)
        assert n > 0, "no csort trace (kernel not csort?)"
        tr = buf[:n]
        st = (tr[:, 0] - tr[:, 0].min()).astype(np.float64) * TICK_US
        en = (tr[:, 1] - tr[:, 0].min()).astype(np.float64) * TICK_US
        dur = en - st
        xcc = (tr[:, 2] & 0xF).astype(int)
        slow = np.argsort(-dur)[:8]
        rec = {"config": cfg, "env": env, "t_min_us": round(t.t_min * 1e6, 2), "n_wg": int(n),
               "span_us": round(float(en.max()), 2),
               "start_us": {"max": round(float(st.max()), 2), "p99": round(float(np.percentile(st, 99)), 2)},
               "dur_us": {"min": round(float(dur.min()), 2), "median": round(float(np.median(dur)), 2),
                          "p90": round(float(np.percentile(dur, 90)), 2), "max": round(float(dur.max()), 2)},
               "end_us_median": round(float(np.median(en)), 2),
               "per_xcd_max_end_us": [round(float(en[xcc == i].max()), 2) if np.any(xcc == i) else None
                                      for i in range(8)],
               "slowest": [{"wg": int(j), "part": int(j % 2), "xcc": int(xcc[j]),
                            "start": round(float(st[j]), 2), "dur": round(float(dur[j]), 2)} for j in slow]}
        if a.per_wg:  # every workgroup, with build_csort's cost terms beside it
            L.hspmv_diag_csort_stats.restype = C.c_int
            L.hspmv_diag_csort_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
            stt = np.zeros((4096, 8), np.int64)
            ns = L.hspmv_diag_csort_stats(h, stt.ctypes.data, 4096)
            names = ["rows", "slices", "chunks", "entries", "quad_sectors", "sectors", "seg_chunks"]
            rec["per_wg"] = {"start_us": np.round(st, 2).tolist(), "dur_us": np.round(dur, 2).tolist(),
                             "xcc": xcc.tolist()}
            if ns == n:
                for i, nm in enumerate(names):
                    rec["per_wg"][nm] = stt[:n, i].tolist()
                # least squares: duration against the cost terms (+ constant)
                X = np.column_stack([stt[:n, 3], stt[:n, 4], stt[:n, 0], stt[:n, 6], np.ones(n)]).astype(float)
                coef, *_ = np.linalg.lstsq(X, dur, rcond=None)
                pred = X @ coef
                rec["fit"] = {"terms": ["entries", "quad_sectors", "rows", "seg_chunks", "const"],
                              "coef_us": [float(c) for c in coef],
                              "r2": float(1 - np.sum((dur - pred) ** 2) / np.sum((dur - dur.mean()) ** 2)),
                              "corr": {nm: float(np.corrcoef(stt[:n, i], dur)[0, 1]) for i, nm in enumerate(names)
                                       if np.std(stt[:n, i]) > 0}}
                for part in range(int(stt[:n, 0].size and 2)):
                    sel = np.arange(n) % 2 == part
                    rec.setdefault("by_part", []).append(
                        {"part": part, "dur_median": float(np.median(dur[sel])), "dur_max": float(dur[sel].max()),
                         "entries_median": float(np.median(stt[:n, 3][sel])),
                         "quad_sectors_median": float(np.median(stt[:n, 4][sel])),
                         "rows_median": float(np.median(stt[:n, 0][sel]))})
        print(json.dumps({k: v for k, v in rec.items() if k != "per_wg"}), flush=True)
        out.append(rec)
        L.hspmv_destroy(h)
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in out))


if __name__ == "__main__":
    main()
