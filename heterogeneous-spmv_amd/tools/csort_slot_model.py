#!/usr/bin/env python3
"""CPU model behind the csort sweep-volume decision (r06).

The column-sorted kernel's x sweep volume is (row blocks per column part) x
(x bytes), and the row blocks per part are fixed by the CU count: 256 / H.
Fewer sweeps need more column parts H, whose blocks hold m H / 256 rows --
beyond the 20.4 K fp64 slots of a workgroup's LDS at H = 4 on C5 -- unless a
block gave slots only to the rows with entries in its part.  This counts,
for C5 and its RCM ordering, the share of rows with entries in each part and
the compacted slots per block that would need.

    python heterogeneous-spmv_amd/tools/csort_slot_model.py > profiles/r06/c5_slot_compaction_model.txt
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from hspmv import gen  # noqa: E402

LDS_SLOTS = 160 * 1024 // 8 - 2  # fp64 slots of one workgroup (hspmv_csort_build.cpp)


def main():
    for rcm in (False, True):
        A = gen.powerlaw(2_000_000, seed=1234, dtype=np.float32, rcm=rcm)
        lens = np.diff(A.row_ptr)
        rows = np.repeat(np.arange(A.m), lens)
        print("rcm", rcm, "m", A.m, "nnz", A.nnz, "len<=4:", np.mean(lens <= 4), "median", np.median(lens))
        for H in (2, 4, 8):
            part = (A.col_idx.astype(np.int64) * H // A.n)
            has = np.zeros((H, A.m), bool)
            has[part, rows] = True
            frac = has.mean(axis=1)
            blocks_per_part = 256 // H
            slots = A.m / blocks_per_part * frac
            print(f"  H={H}: rows with entries per part {np.round(frac, 3)}; "
                  f"compacted slots/block {slots.astype(int)} (cap {LDS_SLOTS})")


if __name__ == "__main__":
    main()
