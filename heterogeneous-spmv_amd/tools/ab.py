#!/usr/bin/env python3
"""A/B timing of two or more libhspmv builds in ONE process on the same
matrices (box-to-box variance is ~3-5 %, larger than most kernel changes).

    python heterogeneous-spmv_amd/tools/ab.py --libs A.so,B.so [--configs c2,c3,c4,c5]
           [--kernel stream] [--rounds 5] [--out F.jsonl]

Each library is dlopen'ed privately; every handle owns its own device copy.
Rounds interleave the libraries; min and median kernel times are reported.
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

from hspmv import _lib, gen  # noqa: E402
from hspmv.api import _KERNELS  # noqa: E402
from auto_regret import build  # noqa: E402  (sweep.build + the planner zoo)


def load(path):
    h = C.CDLL(str(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        fn = getattr(h, name)
        fn.restype, fn.argtypes = res, args
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--configs", default="c2,c3,c4,c5")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--flags", type=int, default=0, help="extra hspmv flags (ORed)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    # each entry: path[@flags][#VAR=VALUE[#VAR2=VALUE2...]] (flags ORed with
    # --flags; the environment variables are set while that handle is created)
    entries, envs = [], []
    for e in a.libs.split(","):
        e, _, env = e.partition("#")
        envs.append([tuple(kv.split("=", 1)) for kv in env.split("#")] if env else None)
        entries.append((e.split("@")[0], int(e.split("@")[1]) if "@" in e else 0))
    cache = {}
    libs = [cache.setdefault(p, load(p)) for p, _ in entries]
    extra = [f for _, f in entries]
    names = [Path(p).parent.name + "/" + Path(p).name + (f"@{f}" if f else "") +
             "".join(f"#{k}={w}" for k, w in (v or [])) for (p, f), v in zip(entries, envs)]
    out = []
    for cfg in a.configs.split(","):
        A, maps, desc = build(cfg)
        x = gen.rand_x(A.n, 42).astype(A.val.dtype)
        cs, ms = A.c_struct(), (maps.c_struct() if maps is not None and a.kernel != "stream" else None)
        hs, places = [], []
        for L, fx, env in zip(libs, extra, envs):
            for k, w in env or []:
                os.environ[k] = w
            h = C.c_void_p()
            rc = L.hspmv_create_on_device(C.byref(h), C.byref(cs), C.byref(ms) if ms else None, 0,
                                          None, _KERNELS[a.kernel] | a.flags | fx)
            for k, _ in env or []:
                os.environ.pop(k, None)
            assert rc == 0, L.hspmv_last_error()
            assert L.hspmv_set_x(h, x.ctypes.data) == 0
            hs.append(h)
            inf = _lib.Info()
            assert L.hspmv_get_info_sized(h, C.byref(inf), C.sizeof(inf)) == 0
            places.append([round(v, 2) for v in inf.placement_us[:inf.placement_trials]] +
                          ([f"pick {inf.placement_pick}"] if inf.placement_trials else []))
        ys = []
        for L, h in zip(libs, hs):
            y = np.empty(A.m, dtype=A.val.dtype)
            assert L.hspmv_spmv(h) == 0 and L.hspmv_get_y(h, y.ctypes.data) == 0
            ys.append(y)
        same = [bool(np.array_equal(ys[0], y)) for y in ys]
        times = [[] for _ in libs]
        for _ in range(a.rounds):
            for i, (L, h) in enumerate(zip(libs, hs)):
                t = _lib.Timing()
                assert L.hspmv_run(h, 3, a.iters, C.byref(t)) == 0
                times[i].append((t.t_min, t.t_avg))
        # y again after the timed launches (racy paths: csort's atomic order,
        # chunk stealing): largest |y - y_first| relative to |y_first| + 1e-30
        rel = []
        for L, h in zip(libs, hs):
            y = np.empty(A.m, dtype=A.val.dtype)
            assert L.hspmv_get_y(h, y.ctypes.data) == 0
            d = np.abs(y.astype(np.float64) - ys[0].astype(np.float64))
            rel.append(float((d / (np.abs(ys[0].astype(np.float64)) + 1e-30)).max()) if A.m else 0.0)
        for i, (L, h) in enumerate(zip(libs, hs)):
            rec = {"config": cfg, "lib": names[i], "kernel": a.kernel,
                   "t_min_us": round(min(t[0] for t in times[i]) * 1e6, 3),
                   "t_med_us": round(float(np.median([t[1] for t in times[i]])) * 1e6, 3),
                   "y_equal_to_first": same[i], "max_rel_vs_first_after": rel[i],
                   "placement_us": places[i]}
            out.append(rec)
            print(json.dumps(rec), flush=True)
        for L, h in zip(libs, hs):
            L.hspmv_destroy(h)
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in out))


if __name__ == "__main__":
    main()
