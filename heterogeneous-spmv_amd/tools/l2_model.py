#!/usr/bin/env python3
"""L2 model of the x-dictionary CSR3 kernel's workgroup -> XCD orders (CPU).

Each 256-row block (four 64-row wave tasks, the aligned plan) stages its x
dictionary runs, reads its row pointers, streams its 16-bit positions and
values and writes y.  tools/l2sim.c replays those line accesses through
eight per-XCD LRU caches (4 MiB, 128-byte lines, 16 ways) with `slots`
workgroups in flight per XCD, for several block orders, and prints the
modelled L2 misses per class (fabric reads) and bytes.

    python heterogeneous-spmv_amd/tools/l2_model.py [--config c3] [--slots 256]
"""
import argparse
import ctypes as C
import json
import subprocess
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))

import hspmv  # noqa: E402
from sweep import build  # noqa: E402

LINE = 128
CLASSES = ["x", "rp", "pos", "val", "y"]


def sim_lib():
    so = HERE / "l2sim.so"
    if not so.exists() or so.stat().st_mtime < (HERE / "l2sim.c").stat().st_mtime:
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", str(HERE / "l2sim.c"), "-o", str(so)])
    L = C.CDLL(str(so))
    L.l2sim.restype = C.c_int
    return L


def block_accesses(A, blk, runs, rows_per_block, val_bytes):
    """Per-block line lists (x staging, row pointers, positions, values, y)."""
    base = {"x": 0, "rp": 1 << 26, "pos": 2 << 26, "val": 3 << 26, "y": 4 << 26}
    nb = len(blk) - 1
    rp = A.row_ptr.astype(np.int64)
    lines, cls, off = [], [], [0]
    for b in range(nb):
        r0 = b * rows_per_block
        r1 = min(r0 + rows_per_block, A.m)
        seq, cs = [], []
        rec = runs[blk[b]:blk[b + 1]]
        # runs: {x_start, lds_off}, the last record a sentinel {0, total}
        for i in range(len(rec) - 1):
            xs, ln = int(rec[i, 0]), int(rec[i + 1, 1] - rec[i, 1])
            if ln <= 0:
                continue
            ls = np.arange(xs * val_bytes // LINE, (xs + ln - 1) * val_bytes // LINE + 1)
            seq.append(base["x"] + ls)
            cs.append(np.full(len(ls), 0, np.uint8))
        ls = np.arange(r0 * 4 // LINE, (r1 * 4) // LINE + 1)
        seq.append(base["rp"] + ls)
        cs.append(np.full(len(ls), 1, np.uint8))
        k0, k1 = int(rp[r0]), int(rp[r1])
        if k1 > k0:
            for name, w, c in (("pos", 2, 2), ("val", val_bytes, 3)):
                ls = np.arange(k0 * w // LINE, (k1 * w - 1) // LINE + 1)
                seq.append(base[name] + ls)
                cs.append(np.full(len(ls), c, np.uint8))
        ls = np.arange(r0 * val_bytes // LINE, (r1 * val_bytes - 1) // LINE + 1)
        seq.append(base["y"] + ls)
        cs.append(np.full(len(ls), 4, np.uint8))
        s = np.concatenate(seq)
        lines.append(s)
        cls.append(np.concatenate(cs))
        off.append(off[-1] + len(s))
    return (np.concatenate(lines).astype(np.uint64), np.concatenate(cls).astype(np.uint8),
            np.array(off, np.int64))


def order_chunk(nb, chunk, nxcd=8):
    """spmv_device.cuh xcd_chunk_remap: grid index -> block."""
    if chunk <= 1:
        return np.arange(nb, dtype=np.int32)
    span = nxcd * chunk
    j = np.arange(nb)
    i, x = j // nxcd, j % nxcd
    o = (i // chunk) * span + x * chunk + (i % chunk)
    full = (nb // span) * span
    o = np.where(j >= full, j, o)
    return o.astype(np.int32)


def order_contiguous(nb, nxcd=8):
    """XCD i takes blocks [i nb/8, (i+1) nb/8) in order."""
    per = -(-nb // nxcd)
    o = np.full(nb, -1, np.int64)
    lists = [list(range(i * per, min((i + 1) * per, nb))) for i in range(nxcd)]
    return interleave(lists, nb, nxcd)


def interleave(lists, nb, nxcd=8):
    """Grid index 8k + i runs lists[i][k]; leftovers fill the tail in order."""
    o = []
    k = 0
    while True:
        row = [lists[i][k] if k < len(lists[i]) else None for i in range(nxcd)]
        if all(v is None for v in row):
            break
        if any(v is None for v in row):  # unequal lengths: the rest in order
            rest = [v for i in range(nxcd) for v in lists[i][k:]]
            o.extend(rest)
            break
        o.extend(row)
        k += 1
    assert sorted(o) == list(range(nb))
    return np.array(o, np.int32)


def order_affinity(blk, runs, val_bytes, nxcd=8, slack=8, decay_blocks=512):
    """Greedy: blocks in row order, each to the XCD whose recently staged x
    lines it overlaps most, the XCDs' block counts kept within `slack`."""
    nb = len(blk) - 1
    owner = {}  # x line -> (xcd, block index when last staged)
    counts = [0] * nxcd
    lists = [[] for _ in range(nxcd)]
    for b in range(nb):
        rec = runs[blk[b]:blk[b + 1]]
        ls = []
        for i in range(len(rec) - 1):
            xs, ln = int(rec[i, 0]), int(rec[i + 1, 1] - rec[i, 1])
            if ln > 0:
                ls.extend(range(xs * val_bytes // LINE, (xs + ln - 1) * val_bytes // LINE + 1))
        score = [0] * nxcd
        for l in ls:
            o = owner.get(l)
            if o is not None and b - o[1] <= decay_blocks:
                score[o[0]] += 1
        lo = min(counts)
        cand = [i for i in range(nxcd) if counts[i] < lo + slack]
        best = max(cand, key=lambda i: (score[i], -counts[i]))
        lists[best].append(b)
        counts[best] += 1
        for l in ls:
            owner[l] = (best, b)
    return interleave(lists, nb, nxcd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--slots", type=int, default=256)
    ap.add_argument("--orders", default="chunk1,chunk4,contig,affinity")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    A, maps, desc = build(a.config)
    vb = A.val.dtype.itemsize
    plan = hspmv.xdict_plan(A, maps, options={"csr3_plan": 1})
    blk, runs, _ = plan
    nb = len(blk) - 1
    rows_per_block = -(-A.m // nb)
    lines, cls, off = block_accesses(A, blk, runs, 256, vb)
    L = sim_lib()
    res = []
    for name in a.orders.split(","):
        if name.startswith("chunk"):
            order = order_chunk(nb, int(name[5:]))
        elif name == "contig":
            order = order_contiguous(nb)
        elif name.startswith("affinity"):
            order = order_affinity(blk, runs, vb)
        hits = np.zeros(len(CLASSES), np.int64)
        miss = np.zeros(len(CLASSES), np.int64)
        rc = L.l2sim(C.c_int64(nb), order.ctypes.data_as(C.c_void_p), 8, a.slots,
                     off.ctypes.data_as(C.c_void_p), lines.ctypes.data_as(C.c_void_p),
                     cls.ctypes.data_as(C.c_void_p), 2048, 16, len(CLASSES),
                     hits.ctypes.data_as(C.c_void_p), miss.ctypes.data_as(C.c_void_p))
        assert rc == 0
        r = {"config": a.config, "order": name, "slots": a.slots, "blocks": nb,
             "rows_per_block": rows_per_block,
             "hits": dict(zip(CLASSES, hits.tolist())), "misses": dict(zip(CLASSES, miss.tolist())),
             "read_miss_MB": round(float(miss[:4].sum()) * LINE / 1e6, 1),
             "x_miss_MB": round(float(miss[0]) * LINE / 1e6, 1),
             "x_requests": int(hits[0] + miss[0])}
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in res))


if __name__ == "__main__":
    main()
