#!/usr/bin/env python3
"""Per-workgroup timeline of the CSR3 kernel from the diag-512 build (make
diag DIAGS=512; HSPMV_DIAG & 512 in csrc/spmv_device.cuh): start and each
wave's end per workgroup (s_memrealtime, 100 MHz), XCD.  Shows the launch's
ramp-up and tail: how many workgroups are live over time, and how long a
workgroup lives.

    HSPMV_LIB=heterogeneous-spmv_amd/build/diag512/libhspmv.so \\
        python heterogeneous-spmv_amd/tools/block_trace.py --configs c3 [--out F.jsonl]
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

import hspmv  # noqa: E402
from hspmv import gen  # noqa: E402
from sweep import build  # noqa: E402

WAVES, SLOTS = 1 << 17, 8
TICK_US = 0.01


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    assert "diag512" in os.environ.get("HSPMV_LIB", ""), "set HSPMV_LIB to the diag512 build"
    L = hspmv.lib()
    L.hspmv_diag_trace.argtypes = [C.c_void_p, C.c_size_t]
    out = []
    for cfg in a.configs.split(","):
        A, maps, desc = build(cfg)
        op = hspmv.SpMV(A, maps)
        op.set_x(gen.rand_x(A.n, 42).astype(A.val.dtype))
        t = op.run(warmup=3, iters=10)
        assert L.hspmv_diag_trace_clear() == 0
        op.spmv()
        op.synchronize()
        buf = np.zeros(WAVES * SLOTS, dtype=np.uint64)
        assert L.hspmv_diag_trace(buf.ctypes.data, buf.nbytes) == 0
        tr = buf.reshape(WAVES, SLOTS).astype(np.int64)
        nb = int(np.count_nonzero(tr[:, 0]))
        tr = tr[:nb]
        t0 = tr[:, 0].min()
        st = (tr[:, 0] - t0) * TICK_US
        ends = np.where(tr[:, 1:5] > 0, (tr[:, 1:5] - t0) * TICK_US, np.nan)
        en = np.nanmax(ends, axis=1)
        life = en - st
        span = float(np.nanmax(en))
        # live workgroups over time (1 us bins)
        bins = np.arange(0.0, span + 1.0, 1.0)
        live = [int(np.sum((st <= b) & (en > b))) for b in bins]
        rec = {"config": cfg, "kernel": op.info["kernel_name"], "t_min_us": round(t["t_min"] * 1e6, 2),
               "workgroups": nb, "span_us": round(span, 2),
               "life_us": {p: round(float(np.nanpercentile(life, p)), 2) for p in (10, 50, 90, 99)},
               "last_start_us": round(float(st.max()), 2),
               "live_per_us": live,
               "end_spread_us": round(float(np.nanmax(ends) - np.nanmin(ends)), 2),
               "first_end_us": round(float(np.nanmin(en)), 2)}
        print(json.dumps({k: v for k, v in rec.items() if k != "live_per_us"}), flush=True)
        print("live:", " ".join(str(v) for v in live[::4]), flush=True)
        out.append(rec)
        op.close()
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in out))


if __name__ == "__main__":
    main()
