"""Row-range partition across ranks (one process per GPU), SURVEY.md §8e.

The reference has no multi-device code (only a cudaGetDeviceCount print,
cuda-spmv-csrk/cuda/spmv-auto-ampere.cu:200-203); this is new.  Rows are
independent, so the SpMV itself shards with no collective: rank r owns a
contiguous, nnz-balanced row range [splits[r], splits[r+1]) with global column
indices, and needs the whole x.  The two exchange steps of the path are

  * x broadcast from rank 0 (``broadcast_x``), once per new x;
  * y gather into a full-length vector (``gather_y``): an all-gather of the
    shards padded to the longest one, then unpadded.

For iterative use on banded / mesh matrices (C2's Laplacian, C4's band) x is
distributed like y -- rank r owns x[splits[r]:splits[r+1]] -- and the x
broadcast is replaced by a halo exchange (SURVEY.md §8e "banded optional
mode"): each rank keeps only the x window [lo, hi) its rows reference
(``localize``), and receives the parts of it other ranks own by point-to-point
send/recv (``plan_halo`` / ``halo_exchange``; RCCL ncclSend/ncclRecv under
the "nccl" backend).  At C4 that is 2 x 32 entries per neighbour instead of
the 160 MB x.

Both go through ``torch.distributed`` (backend "nccl" = RCCL over xGMI on the
GPU box, "gloo" on the CPU in tests).  Workloads are built per rank from the
seeded generators in :mod:`hspmv.gen`, so no rank ever materialises the global
matrix.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import gen
from .api import CsrMatrix, Csr3Maps, build_csr3_maps, csr3_params, partition_rows


# ------------------------------------------------------------------ workloads

@dataclass
class Shard:
    A: CsrMatrix          # this rank's rows (row_ptr rebased, global columns)
    n_global: int         # length of x
    m_global: int
    nnz_global: int
    splits: np.ndarray    # row ranges of all ranks (world+1)
    rank: int
    world: int
    name: str
    scaling: str          # "weak" (per-rank work fixed) or "strong"
    maps: Optional[Csr3Maps] = None  # CSR-3 maps of this rank's rows (rebased)


# The BASELINE.json configurations a bench / test run can name.
#   c2  configs[1]  CSR fp64, 5-pt Laplacian 1000^2 per rank (weak)
#   c3  configs[2]  CSR-3 fp64, 27-pt 125^3 RCM, (ssrs, srs) = (20, 10) from
#                   the .csr3 writer heuristic (reformat-csr-to-csr3/spmv-auto.cpp:154-173)
#   c3h configs[2]  alt: hugebubbles-00000 stand-in, CSR fp64
#   c4  configs[3]  CSR fp64, banded m = 2e7 split over the ranks (strong)
#   c5  configs[4]  CSR-3 fp32, power-law m = 2e6 (MI355X grouping)
#   c5r configs[4]  the same matrix RCM-permuted (the reference's .rcm.csr
#                   input ordering, helpers/converter.m:8,14)
CONFIGS = ("c2", "c3", "c3h", "c4", "c5", "c5r")


def default_config(world: int) -> str:
    """N = 1: C3, the largest single-GPU configuration (BASELINE.json
    configs[2]); N > 1: C4, the configuration the multi-GPU target is stated
    on (configs[3], row-range partition of one 200 M-nnz matrix)."""
    return "c3" if world == 1 else "c4"


def slice_csr3(A: CsrMatrix, maps: Csr3Maps, splits: np.ndarray, rank: int):
    """Rows [splits[rank], splits[rank+1]) of a CSR-3 matrix whose splits fall
    on super-super-row boundaries (hspmv_partition_rows with maps), with the
    matching slice of the maps rebased to the shard."""
    r0, r1 = int(splits[rank]), int(splits[rank + 1])
    A_loc = A.rows(r0, r1)
    sr_first = maps.inner[maps.outer[:-1]]          # first row of every SSR
    s0 = int(np.searchsorted(sr_first, r0, side="left"))
    s1 = int(np.searchsorted(sr_first, r1, side="left")) if r1 < A.m else maps.n_ssr
    outer = maps.outer[s0:s1 + 1]
    inner = maps.inner[int(outer[0]):int(outer[-1]) + 1] - r0
    return A_loc, Csr3Maps(outer - outer[0], inner)


def _whole_matrix(config: str, dtype):
    if config == "c3":
        A = gen.stencil27(125, dtype=dtype)
        return A, build_csr3_maps(A, *csr3_params(A.nnz / A.m, "volta")), \
            "27-pt stencil 125^3 RCM (fp64 CSR-3, ssrs=20, srs=10)"
    if config == "c3h":
        A = gen.honeycomb(4280, 4280, dtype=dtype)
        return A, None, "hugebubbles-00000 stand-in: honeycomb 4280^2 RCM (fp64 CSR)"
    if config in ("c5", "c5r"):
        rcm = config == "c5r"
        A = gen.powerlaw(2_000_000, seed=1234, dtype=dtype, rcm=rcm)
        return A, build_csr3_maps(A, *csr3_params(A.nnz / A.m, "mi355x")), \
            ("power-law m=2e6, Pareto alpha=1.5, seed 1234" + (", RCM-permuted" if rcm else "")
             + " (fp32 CSR-3)")
    raise ValueError(config)


def config_dtype(config: str):
    return np.float32 if config in ("c5", "c5r") else np.float64


def laplace2d_row_nnz(nx: int, ny: int) -> np.ndarray:
    """Row lengths of the 5-point Laplacian on nx x ny (no columns built)."""
    m = nx * ny
    r = np.arange(m, dtype=np.int64)
    ix = r % nx
    return (1 + (r >= nx) + (ix > 0) + (ix < nx - 1) + (r < m - nx)).astype(np.int64)


def banded_row_nnz(m: int, per_row: int = 10, half: int = 32, seed: int = 11) -> np.ndarray:
    """Row lengths of gen.banded (only the first/last `half` rows lose columns)."""
    cnt = np.full(m, per_row, np.int64)
    edge = min(half, m)
    for r0, r1 in ((0, edge), (max(m - edge, 0), m)):
        if r1 > r0:
            cnt[r0:r1] = np.diff(gen.banded(m, per_row, half, seed, r0=r0, r1=r1).row_ptr)
    return cnt


def splits_from_row_nnz(row_nnz: np.ndarray, world: int) -> np.ndarray:
    rp = np.zeros(row_nnz.shape[0] + 1, np.int64)
    np.cumsum(row_nnz, out=rp[1:])
    if rp[-1] >= 2 ** 31:
        # int32 row_ptr cannot hold it: balance on the int64 prefix sum directly
        targets = rp[-1] * np.arange(world + 1) // world
        s = np.searchsorted(rp, targets, side="left").astype(np.int64)
        s[0], s[-1] = 0, row_nnz.shape[0]
        return s
    return partition_rows(rp.astype(np.int32), world)


def plan_splits(config: str, world: int) -> dict:
    """The row partition a run of `config` on `world` ranks uses, from row
    lengths alone (no matrix, no GPU): what ``bench.py --dry-run`` prints.
    Only the configurations whose row lengths are known in closed form."""
    if config in ("c2", "small"):
        nx = 1000 if config == "c2" else 64
        row_nnz = laplace2d_row_nnz(nx, nx * world)
        scaling = "weak"
    elif config == "c4":
        row_nnz = banded_row_nnz(20_000_000)
        scaling = "strong"
    else:
        raise ValueError(f"no closed-form row lengths for {config!r}")
    s = splits_from_row_nnz(row_nnz, world)
    rp = np.zeros(row_nnz.shape[0] + 1, np.int64)
    np.cumsum(row_nnz, out=rp[1:])
    return {"config": config, "world": world, "scaling": scaling, "m": int(row_nnz.shape[0]),
            "nnz": int(rp[-1]), "splits": [int(v) for v in s],
            "rows_per_rank": [int(v) for v in np.diff(s)],
            "nnz_per_rank": [int(v) for v in rp[s[1:]] - rp[s[:-1]]]}


def build_shard(config: str, rank: int, world: int, dtype=None) -> Shard:
    """c2: 5-pt Laplacian, 1000 x 1000 rows per rank (global grid 1000 x 1000*world,
           weak scaling; world = 1 is BASELINE configs[1] exactly).
       c3 / c3h / c5: one matrix (configs[2], configs[4]) split over the
           ranks, nnz-balanced on super-super-row boundaries when it has
           CSR-3 maps (strong scaling; every rank generates the whole matrix
           and keeps its rows).
       c4: banded m = 2e7 (BASELINE configs[3]) split over the ranks (strong).
       small: 5-pt Laplacian 64 x 64 per rank (tests)."""
    dtype = config_dtype(config) if dtype is None else dtype
    if config in ("c3", "c3h", "c5", "c5r"):
        A, maps, name = _whole_matrix(config, dtype)
        splits = partition_rows(A.row_ptr, world, maps)
        if maps is not None:
            A_loc, m_loc = slice_csr3(A, maps, splits, rank)
        else:
            A_loc, m_loc = A.rows(int(splits[rank]), int(splits[rank + 1])), None
        return Shard(A_loc, A.n, A.m, A.nnz, splits, rank, world, name, "strong", m_loc)
    if config in ("c2", "small"):
        nx = 1000 if config == "c2" else 64
        ny = nx * world
        row_nnz = laplace2d_row_nnz(nx, ny)
        splits = splits_from_row_nnz(row_nnz, world)
        A = gen.laplace2d(nx, ny, int(splits[rank]), int(splits[rank + 1]), dtype=dtype)
        return Shard(A, nx * ny, nx * ny, int(row_nnz.sum()), splits, rank, world,
                     f"5-pt Laplacian {nx}x{ny} (fp64 CSR), {nx}x{nx} rows per GPU", "weak")
    if config == "c4":
        m = 20_000_000
        row_nnz = banded_row_nnz(m)
        splits = splits_from_row_nnz(row_nnz, world)
        A = gen.banded(m, r0=int(splits[rank]), r1=int(splits[rank + 1]), dtype=dtype)
        return Shard(A, m, m, int(row_nnz.sum()), splits, rank, world,
                     "banded m=2e7, 10 nnz/row within +-32 (fp64 CSR)", "strong")
    raise ValueError(f"unknown distributed config {config!r}")


# ------------------------------------------------------------------ exchanges

def _staged(t):
    """gloo moves host tensors only: a device tensor goes through a host copy
    (the one-GPU rehearsal of the multi-rank path); under "nccl" (RCCL) the
    tensor is used as it is."""
    import torch.distributed as dist
    return t.cpu() if (t.is_cuda and dist.get_backend() != "nccl") else t


def broadcast_x(x, src: int = 0) -> None:
    """In-place broadcast of the full x (a torch tensor) from rank src."""
    import torch.distributed as dist
    xs = _staged(x)
    dist.broadcast(xs, src)
    if xs is not x:
        x.copy_(xs)


def gather_y(y_local, splits: np.ndarray):
    """All-gather the row shards into a full-length y on every rank (padded
    all-gather, then unpadded).  y_local: torch tensor of this rank's rows."""
    import torch
    import torch.distributed as dist
    world = len(splits) - 1
    rows = np.diff(splits)
    pad = int(rows.max())
    buf = torch.zeros(pad, dtype=y_local.dtype, device=y_local.device)
    buf[: y_local.shape[0]] = y_local
    buf = _staged(buf)
    out = torch.empty(pad * world, dtype=y_local.dtype, device=buf.device)
    dist.all_gather_into_tensor(out, buf)
    parts = [out[r * pad: r * pad + int(rows[r])] for r in range(world)]
    return torch.cat(parts).to(y_local.device)  # on the caller's device whatever the backend


def chunk_splits(A: CsrMatrix, k: int) -> np.ndarray:
    """k contiguous, nnz-balanced row ranges of this rank's rows (k + 1 bounds)."""
    return partition_rows(A.row_ptr, k).astype(np.int64)


class OverlappedGather:
    """The y all-gather overlapped with the SpMV (SURVEY.md §8e end-to-end
    rate): the rank's rows are computed in K chunks, and chunk k's rows are
    all-gathered (async collective, padded to the longest chunk k over the
    ranks) while chunks k+1.. still compute.  Under "nccl" the collective is
    issued on RCCL's stream after the work already enqueued on the current
    stream, so it starts as soon as chunk k's kernel ends.

    Usage per SpMV: for k: write chunk k's rows into ``buffer(k)[:rows[k]]``
    (bind the chunk's y there), then ``start(k)``; finally ``finish()``
    returns the full-length y (rank order, then chunk order)."""

    def __init__(self, chunk_rows, device="cpu", dtype=None):
        import torch
        import torch.distributed as dist
        self.world = dist.get_world_size()
        self.k = len(chunk_rows)
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        mine = torch.tensor([int(v) for v in chunk_rows], dtype=torch.int64, device=dev)
        allr = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(allr, mine)
        self.rows = np.stack([r.cpu().numpy() for r in allr])       # [world][K]
        self.pad = self.rows.max(axis=0)                             # per chunk
        dtype = dtype or torch.float64
        self.bufs = [torch.zeros(max(int(p), 1), dtype=dtype, device=device) for p in self.pad]
        self.outs = [torch.empty(max(int(p), 1) * self.world, dtype=dtype, device=device)
                     for p in self.pad]
        self.works = [None] * self.k

    def buffer(self, k: int):
        return self.bufs[k]

    def start(self, k: int) -> None:
        import torch.distributed as dist
        src, dst = _staged(self.bufs[k]), _staged(self.outs[k])
        w = dist.all_gather_into_tensor(dst, src, async_op=True)
        self.works[k] = (w, dst)

    def finish(self):
        import torch
        parts = []
        for k in range(self.k):
            w, dst = self.works[k]
            w.wait()
            if dst is not self.outs[k]:
                self.outs[k].copy_(dst)
        p = [max(int(v), 1) for v in self.pad]
        for r in range(self.world):
            for k in range(self.k):
                parts.append(self.outs[k][r * p[k]: r * p[k] + int(self.rows[r][k])])
        return torch.cat(parts)


def checksum_ok(A: CsrMatrix, x: np.ndarray, y: np.ndarray, seed: int = 99) -> tuple[bool, float]:
    """Size-independent identity w.(A x) == (A^T w).x in fp64 -- a property
    check of the GPU y that needs neither the oracle nor a second SpMV path."""
    w = gen.rand_x(A.m, seed)
    lhs = float(np.dot(w, y.astype(np.float64)))
    rows = np.repeat(np.arange(A.m), np.diff(A.row_ptr))
    atw = np.bincount(A.col_idx, weights=A.val.astype(np.float64) * w[rows], minlength=A.n)
    rhs = float(np.dot(atw, x.astype(np.float64)))
    scale = float(np.dot(np.abs(w)[rows], np.abs(A.val.astype(np.float64) * x[A.col_idx]))) + 1e-300
    rel = abs(lhs - rhs) / scale
    tol = 1e-12 if A.val.dtype == np.float64 else 1e-5
    return rel <= tol, rel


# ------------------------------------------------------------------ halo mode

@dataclass
class Halo:
    lo: int               # this rank's x window is x[lo:hi)
    hi: int
    own: tuple            # x[own[0]:own[1]] is owned (computed) by this rank
    recvs: list           # (peer, g0, g1): receive x[g0:g1] from peer
    sends: list           # (peer, g0, g1): send x[g0:g1] to peer


def column_window(A: CsrMatrix, own: tuple) -> tuple:
    """[lo, hi): the smallest x range holding every column of A and the
    rank's own entries."""
    lo, hi = int(own[0]), int(own[1])
    if A.nnz:
        lo = min(lo, int(A.col_idx.min()))
        hi = max(hi, int(A.col_idx.max()) + 1)
    return lo, hi


def localize(A: CsrMatrix, lo: int, hi: int) -> CsrMatrix:
    """A with columns rebased to its x window [lo, hi) (n = hi - lo)."""
    return CsrMatrix(A.m, hi - lo, A.row_ptr, (A.col_idx - lo).astype(np.int32), A.val)


def plan_halo(A: CsrMatrix, splits: np.ndarray, rank: int, world: int) -> Halo:
    """Who sends which part of x to whom.  x is distributed like the rows
    (square matrix); one all-gather of the (lo, hi) windows, then every rank
    intersects the windows with the owned ranges."""
    import torch
    import torch.distributed as dist
    own = (int(splits[rank]), int(splits[rank + 1]))
    lo, hi = column_window(A, own)
    win = torch.tensor([lo, hi], dtype=torch.int64)
    if dist.get_backend() == "nccl":
        win = win.cuda()
    allw = [torch.empty_like(win) for _ in range(world)]
    dist.all_gather(allw, win)
    allw = [tuple(int(v) for v in w.cpu()) for w in allw]
    recvs, sends = [], []
    for q in range(world):
        if q == rank:
            continue
        q0, q1 = int(splits[q]), int(splits[q + 1])
        g0, g1 = max(lo, q0), min(hi, q1)          # of my window, owned by q
        if g1 > g0:
            recvs.append((q, g0, g1))
        w0, w1 = allw[q]
        g0, g1 = max(w0, own[0]), min(w1, own[1])  # of q's window, owned by me
        if g1 > g0:
            sends.append((q, g0, g1))
    return Halo(lo, hi, own, recvs, sends)


def halo_exchange(x_win, halo: Halo) -> None:
    """Fills the non-owned parts of x_win (a torch tensor holding x[lo:hi),
    own part already written) from the ranks that own them."""
    import torch.distributed as dist
    xw = _staged(x_win)
    ops = []
    for q, g0, g1 in halo.sends:
        ops.append(dist.P2POp(dist.isend, xw[g0 - halo.lo:g1 - halo.lo].contiguous(), q))
    for q, g0, g1 in halo.recvs:
        ops.append(dist.P2POp(dist.irecv, xw[g0 - halo.lo:g1 - halo.lo], q))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if xw is not x_win:
        x_win.copy_(xw)


def halo_bytes(halo: Halo, itemsize: int = 8) -> int:
    """Bytes this rank receives per exchange."""
    return sum(g1 - g0 for _, g0, g1 in halo.recvs) * itemsize
