#!/usr/bin/env python3
"""Per-workgroup timeline of one column-sorted (csort) launch: start / end
(s_memrealtime, 100 MHz), XCD and HW_ID (CU / shader array / engine) of
every workgroup, and each wave's end and chunk count, from the diagnostic
library (build/diagenv/libhspmv.so, HSPMV_CSORT_TRACE=1).  Shows whether a
launch is bound by its slowest workgroups (a tail) or by the rate of all,
and -- over --launches repeated launches -- whether a workgroup is slow
because of its work (slow every launch), its CU (the CU is slow whatever
runs on it) or neither.

    python heterogeneous-spmv_amd/tools/csort_trace.py --configs c5,c5r [--env K=V,...]
           [--launches 8] --out F.json
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
NW = 16          # waves per csort workgroup (kCsortThreads / 64)
SLOTS = 4 + 2 * NW  # kCsortTraceSlots (hspmv_internal.h)


def decode(tr):
    """start / end / duration (us from the launch's first start), XCC, a CU
    key from HW_ID (xcc, se, sh, cu), each wave's end (us from its
    workgroup's start), each wave's chunk count, and the slot-zeroing time."""
    t0 = tr[:, 0].min()
    st = (tr[:, 0] - t0).astype(np.float64) * TICK_US
    en = (tr[:, 1] - t0).astype(np.float64) * TICK_US
    xcc = (tr[:, 2] & 0xF).astype(int)
    hw = (tr[:, 2] >> np.uint64(32)).astype(np.int64)
    cu_key = xcc * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15)
    wave_end = (tr[:, 4:4 + NW] - tr[:, 0:1]).astype(np.float64) * TICK_US
    wave_chunks = tr[:, 4 + NW:4 + 2 * NW].astype(np.int64)
    zero_us = (tr[:, 3] - tr[:, 0]).astype(np.float64) * TICK_US
    return st, en, en - st, xcc, cu_key, wave_end, wave_chunks, zero_us

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c5,c5r")
    ap.add_argument("--lib", default=str(HERE.parent / "build" / "diagenv" / "libhspmv.so"))
    ap.add_argument("--env", default="", help="extra A/B knobs K=V,K=V for the handle")
    ap.add_argument("--out", default="")
    ap.add_argument("--per-wg", action="store_true", help="every workgroup + the build's cost terms")
    ap.add_argument("--launches", type=int, default=1,
                    help="repeat single launches and correlate durations by workgroup and by CU")
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
        buf = np.zeros((4096, SLOTS), np.uint64)
        n = L.hspmv_diag_csort_trace(h, buf.ctypes.data, 4096)
        assert n > 0, "no csort trace (kernel not csort?)"
        tr = buf[:n].copy()
        st, en, dur, xcc, cu_key, wave_end, wave_chunks, zero_us = decode(tr)
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
        # inside the workgroups: how far the last wave ends after the median
        # wave (intra-workgroup imbalance) and the slot-zeroing phase
        spread = wave_end.max(axis=1) - np.median(wave_end, axis=1)
        rec["waves"] = {"last_minus_median_wave_us": {"median": round(float(np.median(spread)), 2),
                                                       "max": round(float(spread.max()), 2)},
                        "slowest_wg_last_minus_median_us": [round(float(spread[j]), 2) for j in slow],
                        "slowest_wg_wave_end_us": [np.round(wave_end[j], 2).tolist() for j in slow[:3]],
                        "chunks_per_wave_minmax": [int(wave_chunks.min()), int(wave_chunks.max())],
                        "zero_us_median": round(float(np.median(zero_us)), 2)}
        if a.launches > 1:  # is a slow workgroup slow again?  is a CU slow whatever it runs?
            durs, keys = [dur], [cu_key]
            for _ in range(a.launches - 1):
                assert L.hspmv_run(h, 0, 1, C.byref(t)) == 0
                assert L.hspmv_diag_csort_trace(h, buf.ctypes.data, 4096) == n
                d2 = decode(buf[:n].copy())
                durs.append(d2[2])
                keys.append(d2[4])
            D = np.array(durs)
            K = np.array(keys)
            wg_corr = [float(np.corrcoef(D[i], D[i + 1])[0, 1]) for i in range(len(D) - 1)]
            same_cu = float(np.mean([np.mean(K[i] == K[0]) for i in range(1, len(K))]))
            # per-CU mean excess over the launch median, split into halves of
            # the launches: does a CU's excess in one half predict the other?
            exc = D - np.median(D, axis=1, keepdims=True)
            cu_ex = [{}, {}]
            for i in range(len(D)):
                for k, e in zip(K[i], exc[i]):
                    cu_ex[i % 2].setdefault(int(k), []).append(float(e))
            common = sorted(set(cu_ex[0]) & set(cu_ex[1]))
            cu_corr = (float(np.corrcoef([np.mean(cu_ex[0][k]) for k in common],
                                          [np.mean(cu_ex[1][k]) for k in common])[0, 1])
                       if len(common) > 8 else None)
            rec["launches"] = {"n": int(len(D)), "span_us": [round(float(v), 2) for v in D.max(axis=1)],
                               "wg_dur_corr_between_launches": [round(v, 3) for v in wg_corr],
                               "same_cu_as_first_launch": round(same_cu, 3),
                               "cu_excess_corr_between_halves": (round(cu_corr, 3) if cu_corr is not None
                                                                 else None),
                               "cus_seen": len(common),
                               "slowest_wg_each_launch": [int(np.argmax(d)) for d in D]}
        if a.per_wg:  # every workgroup, with build_csort's cost terms beside it
            L.hspmv_diag_csort_stats.restype = C.c_int
            L.hspmv_diag_csort_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
            stt = np.zeros((4096, 8), np.int64)
            ns = L.hspmv_diag_csort_stats(h, stt.ctypes.data, 4096)
            names = ["rows", "slices", "chunks", "entries", "quad_sectors", "sectors", "seg_chunks"]
            rec["per_wg"] = {"start_us": np.round(st, 2).tolist(), "dur_us": np.round(dur, 2).tolist(),
                             "xcc": xcc.tolist(), "cu_key": cu_key.tolist(),
                             "wave_end_max_us": np.round(wave_end.max(axis=1), 2).tolist(),
                             "wave_end_median_us": np.round(np.median(wave_end, axis=1), 2).tolist()}
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
