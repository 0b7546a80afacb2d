"""Synthetic inputs for the BASELINE.json configurations.

No matrix can be fetched here, so every configuration has a seeded synthetic
stand-in with the shape the reference benchmarks:

* C1/C2  2-D 5-point Laplacian 1000 x 1000 (kron(I,T)+kron(T,I), T =
         tridiag(-1,2,-1)): m = 1,000,000, nnz = 4,996,000.
* C3     3-D 27-point stencil 125^3, values U(-1,1) seed 7, diagonal 27,
         RCM-permuted (scipy reverse_cuthill_mckee): nnz = 51,895,117.
* C4     banded: m = 20,000,000, 10 nonzeros per row at r+o, o drawn without
         replacement from [-32, 32], seed 11, values U(-1,1).
* C5     power-law: row degree min(4*(Pareto(1.5)+1), m/10), random columns,
         symmetrised + diagonal, seed 1234; c5r = the same matrix
         RCM-permuted, the ordering the reference benchmarks its inputs in
         (helpers/converter.m:8,14: symrcm -> .mtx.rcm.csr).

Generators that may be sharded take a row range [r0, r1) so that each rank of
a row-range partition builds only its own rows (global columns).
The .csr text writer follows helpers/converter.m:25-33 + sparse2csr.m.
"""
from __future__ import annotations

import numpy as np

from .api import CsrMatrix


# ------------------------------------------------------------------ x vectors

def rand_x(n: int, seed: int = 42, dtype=np.float64) -> np.ndarray:
    """U(-1,1) from splitmix64 (bit-identical to the CLI's --x rand:SEED)."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return (u * 2.0 - 1.0).astype(dtype)


# ------------------------------------------------------------------ matrices

def laplace2d(nx: int, ny: int, r0: int = 0, r1: int | None = None,
              dtype=np.float64) -> CsrMatrix:
    """Rows [r0, r1) of the 5-point Laplacian on an nx-by-ny grid (natural
    order, row = iy*nx + ix); columns sorted: r-nx, r-1, r, r+1, r+nx."""
    m = nx * ny
    r1 = m if r1 is None else r1
    rows = np.arange(r0, r1, dtype=np.int64)
    ix = rows % nx
    offs = [(-nx, rows >= nx), (-1, ix > 0), (0, np.ones_like(rows, bool)),
            (1, ix < nx - 1), (nx, rows < m - nx)]
    mask = np.stack([mk for _, mk in offs], axis=1)
    cols = np.stack([rows + o for o, _ in offs], axis=1)
    vals = np.broadcast_to(np.array([-1.0, -1.0, 4.0, -1.0, -1.0]), mask.shape)
    cnt = mask.sum(axis=1)
    rp = np.zeros(r1 - r0 + 1, np.int64)
    np.cumsum(cnt, out=rp[1:])
    return CsrMatrix(r1 - r0, m, rp.astype(np.int32), cols[mask].astype(np.int32),
                     vals[mask].astype(dtype))


def stencil27(n: int, seed: int = 7, rcm: bool = True, dtype=np.float64) -> CsrMatrix:
    """27-point stencil on n^3 (values U(-1,1), diagonal 27), RCM-permuted."""
    import scipy.sparse as sp
    N = n ** 3
    idx = np.arange(N, dtype=np.int64)
    iz, iy, ix = idx // (n * n), (idx // n) % n, idx % n
    rows, cols = [], []
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                ok = ((ix + dx >= 0) & (ix + dx < n) & (iy + dy >= 0) & (iy + dy < n)
                      & (iz + dz >= 0) & (iz + dz < n))
                rows.append(idx[ok])
                cols.append(idx[ok] + dx + dy * n + dz * n * n)
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    rng = np.random.default_rng(seed)
    v = rng.uniform(-1.0, 1.0, r.shape[0])
    v[r == c] = 27.0
    S = sp.csr_matrix((v, (r, c)), shape=(N, N))
    if rcm:
        from scipy.sparse.csgraph import reverse_cuthill_mckee
        perm = reverse_cuthill_mckee(S, symmetric_mode=True)
        S = S[perm][:, perm].tocsr()
    S.sort_indices()
    return CsrMatrix.from_scipy(S, dtype)


def honeycomb(nx: int, ny: int, seed: int = 5, rcm: bool = True, dtype=np.float64) -> CsrMatrix:
    """Brick-wall (honeycomb) lattice graph on nx x ny vertices: neighbours
    (i +- 1, j) and (i, j + 1) when i + j is even, else (i, j - 1); degree
    <= 3, no diagonal, values U(-1,1), RCM-permuted.  Stand-in for the
    reference's DIMACS10 bubble meshes (helpers/overhead.txt:33-34,
    hugebubbles-00000: 18,318,143 rows, 54,940,162 nnz, degree 3): at
    nx = ny = 4280 it has 18.3 M rows and 54.9 M nonzeros."""
    import scipy.sparse as sp
    N = nx * ny
    idx = np.arange(N, dtype=np.int64)
    i, j = idx % nx, idx // nx
    rows, cols = [], []
    ok = i + 1 < nx
    rows += [idx[ok], idx[ok] + 1]
    cols += [idx[ok] + 1, idx[ok]]
    ok = ((i + j) % 2 == 0) & (j + 1 < ny)
    rows += [idx[ok], idx[ok] + nx]
    cols += [idx[ok] + nx, idx[ok]]
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    del rows, cols, idx, i, j, ok
    rng = np.random.default_rng(seed)
    S = sp.csr_matrix((rng.uniform(-1.0, 1.0, r.shape[0]), (r, c)), shape=(N, N))
    del r, c
    if rcm:
        from scipy.sparse.csgraph import reverse_cuthill_mckee
        perm = reverse_cuthill_mckee(S, symmetric_mode=True)
        S = S[perm][:, perm].tocsr()
    S.sort_indices()
    return CsrMatrix.from_scipy(S, dtype)


def banded(m: int, per_row: int = 10, half: int = 32, seed: int = 11, r0: int = 0,
           r1: int | None = None, dtype=np.float64, chunk: int = 1 << 20) -> CsrMatrix:
    """Rows [r0, r1) of the C4 banded matrix: per_row distinct offsets per row
    from [-half, half] (per-row stream seeded by (seed, row chunk)), columns
    clipped to [0, m) with duplicates dropped, values U(-1,1)."""
    r1 = m if r1 is None else r1
    width = 2 * half + 1
    rps, cis, vas = [np.zeros(1, np.int64)], [], []
    base = 0
    c0 = (r0 // chunk) * chunk
    for cs in range(c0, r1, chunk):
        ce = min(cs + chunk, m)
        rng = np.random.default_rng([seed, cs // chunk])
        keys = rng.random((ce - cs, width), dtype=np.float32)
        offs = np.argsort(keys, axis=1)[:, :per_row].astype(np.int64) - half
        offs.sort(axis=1)
        vals = rng.uniform(-1.0, 1.0, (ce - cs, per_row))
        lo, hi = max(cs, r0), min(ce, r1)
        sl = slice(lo - cs, hi - cs)
        rows = np.arange(lo, hi, dtype=np.int64)[:, None]
        cols = rows + offs[sl]
        ok = (cols >= 0) & (cols < m)
        cnt = ok.sum(axis=1)
        rps.append(base + np.cumsum(cnt))
        base += int(cnt.sum())
        cis.append(cols[ok])
        vas.append(vals[sl][ok])
    rp = np.concatenate(rps)
    return CsrMatrix(r1 - r0, m, rp.astype(np.int32), np.concatenate(cis).astype(np.int32),
                     np.concatenate(vas).astype(dtype))


def powerlaw(m: int, alpha: float = 1.5, seed: int = 1234, dtype=np.float32,
             rcm: bool = False) -> CsrMatrix:
    """Scale-free rows: degree min(4*(Pareto(alpha)+1), m/10), random columns,
    symmetrised (A + A^T pattern) plus the diagonal, values U(-1,1).  rcm:
    the same matrix (same values) symmetrically permuted by reverse
    Cuthill-McKee, as the reference's converter orders its inputs
    (helpers/converter.m:8,14)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    deg = np.minimum((4 * (rng.pareto(alpha, m) + 1)).astype(np.int64), max(m // 10, 1))
    r = np.repeat(np.arange(m, dtype=np.int64), deg)
    c = rng.integers(0, m, r.shape[0], dtype=np.int64)
    d = np.arange(m, dtype=np.int64)
    rr = np.concatenate([r, c, d])
    cc = np.concatenate([c, r, d])
    S = sp.csr_matrix((np.ones(rr.shape[0], np.float32), (rr, cc)), shape=(m, m))
    S.sum_duplicates()
    S.sort_indices()
    S.data = rng.uniform(-1.0, 1.0, S.nnz).astype(np.float64)
    if rcm:
        from scipy.sparse.csgraph import reverse_cuthill_mckee
        perm = reverse_cuthill_mckee(S, symmetric_mode=True)
        S = S[perm][:, perm].tocsr()
        S.sort_indices()
    return CsrMatrix.from_scipy(S, dtype)


# ------------------------------------------------------------------ text I/O

def write_csr_text(path: str, A: CsrMatrix, index_base: int = 0) -> None:
    """helpers/converter.m:25-33: "m n nnz\\n", then "%d " row_ptr, "%d "
    col_ind, "%f " val lines (each ending with a space and newline)."""
    with open(path, "w") as f:
        f.write(f"{A.m} {A.n} {A.nnz}\n")
        f.write(" ".join(map(str, (A.row_ptr.astype(np.int64) + index_base).tolist())) + " \n")
        f.write(" ".join(map(str, (A.col_idx.astype(np.int64) + index_base).tolist())) + " \n")
        f.write(" ".join("%f" % v for v in A.val.tolist()) + " \n")
