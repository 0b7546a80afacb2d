#!/usr/bin/env python3
"""Per-wave phase timing of the STREAM fp64 kernel from the diag-8 build
(make diag; HSPMV_DIAG & 8 in csrc/spmv_device.cuh).  Each wave's lane 0
stamps s_memtime at: start, row bounds loaded, first chunk's col/val
arrived, its x gather arrived, its row sums done, and the end; every stamp
waits for the wave's outstanding loads, so the phases are serialised.

    HSPMV_LIB=heterogeneous-spmv_amd/build/diag8/libhspmv.so \
        python heterogeneous-spmv_amd/tools/wave_trace.py --configs c4,c3
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


def q(a):
    return {p: float(np.percentile(a, p)) for p in (10, 50, 90)} if len(a) else {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c4,c3")
    ap.add_argument("--u", type=int, default=0)
    ap.add_argument("--kernel", default="stream")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    assert "diag8" in os.environ.get("HSPMV_LIB", ""), "set HSPMV_LIB to the diag8 build"
    L = hspmv.lib()
    L.hspmv_diag_trace.argtypes = [C.c_void_p, C.c_size_t]
    out = []
    for cfg in a.configs.split(","):
        A, maps, desc = build(cfg)
        op = hspmv.SpMV(A, maps if a.kernel == "csr3" else None, kernel=a.kernel, chunk_u=a.u)
        op.set_x(gen.rand_x(A.n, 42).astype(A.val.dtype))
        t = op.run(warmup=3, iters=10)
        assert L.hspmv_diag_trace_clear() == 0
        op.spmv()
        op.synchronize()
        buf = np.zeros(WAVES * SLOTS, dtype=np.uint64)
        assert L.hspmv_diag_trace(buf.ctypes.data, buf.nbytes) == 0
        tr = buf.reshape(WAVES, SLOTS).astype(np.int64)
        tr = tr[tr[:, 0] != 0]
        d = {k: tr[:, i + 1] - tr[:, i] for i, k in enumerate(["rp", "colval", "gather", "sums"])}
        d["rest"] = tr[:, 5] - tr[:, 4]
        d["life"] = tr[:, 5] - tr[:, 0]
        rec = {"config": cfg, "kernel": a.kernel, "desc": desc, "t_min_us": t["t_min"] * 1e6, "waves": int(len(tr)),
               "chunks_mean": float(tr[:, 7].mean()), "info_u": op.info["chunk_u"],
               "phases_cycles": {k: q(v) for k, v in d.items()},
               "mean_cycles": {k: float(v.mean()) for k, v in d.items()}}
        # start-time spread per XCD-local SE (HW_ID se_id, bits 13-15)
        t0 = tr[:, 0] - tr[:, 0].min()
        rec["start_span_cycles"] = q(t0)
        out.append(rec)
        print(json.dumps(rec), flush=True)
        op.close()
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in out))


if __name__ == "__main__":
    main()
