import sys, numpy as np
sys.path.insert(0, "heterogeneous-spmv_amd")
from hspmv import gen
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
        print(f"  H={H}: rows with entries per part {np.round(frac,3)}; compacted slots/block {slots.astype(int)} (cap 20478)")
