"""Multi-rank row-range partition on the CPU with gloo,
world_size 2, 3, 4 and 8 (the driver's node size): each rank builds only its shard, x is broadcast from rank
0, the per-rank y (computed here by the oracle, the GPU's stand-in on a
CPU-only box) is all-gathered, and the result must equal the oracle on the
global matrix -- the same orchestration bench.py runs over RCCL."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, config, q, use_hip=False):
    sys.path.insert(0, str(REPO / "heterogeneous-spmv_amd"))
    sys.path.insert(0, str(REPO / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from hspmv import dist as hdist
        from hspmv import gen
        sh = hdist.build_shard(config, rank, world)
        x = torch.zeros(sh.n_global, dtype=torch.float64)
        if rank == 0:
            x.copy_(torch.from_numpy(gen.rand_x(sh.n_global, 42)))
        hdist.broadcast_x(x)
        xn = x.numpy()
        if use_hip:  # the rank's shard through the HIP library (C ABI), device 0
            import hspmv
            with hspmv.SpMV(sh.A, device=0) as op:
                y_local = op(xn)
        else:
            y_local = oracle.spmv(sh.A.row_ptr, sh.A.col_idx, sh.A.val, xn)
        ok, rel = hdist.checksum_ok(sh.A, xn, y_local)
        y = hdist.gather_y(torch.from_numpy(y_local), sh.splits).numpy()
        nnz = torch.tensor([sh.A.nnz], dtype=torch.int64)
        dist.all_reduce(nnz)
        q.put((rank, y if rank == 0 else None, ok, int(nnz.item()), sh.splits.tolist(),
               sh.nnz_global, sh.A.m))
    finally:
        dist.destroy_process_group()


def _run_partition(world, use_hip):
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    from hspmv import gen
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, "small", q, use_hip))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    y = res[0][1]
    A = gen.laplace2d(64, 64 * world)
    y_ref = oracle.spmv(A.row_ptr, A.col_idx, A.val, gen.rand_x(A.n, 42))
    assert np.array_equal(y, y_ref)
    assert all(r[2] for r in res)                       # per-rank checksum identity
    assert res[0][3] == A.nnz == res[0][5]              # shards cover every nonzero once
    splits = np.array(res[0][4])
    assert splits[0] == 0 and splits[-1] == A.m and np.all(np.diff(splits) > 0)
    shard_nnz = A.row_ptr[splits[1:]] - A.row_ptr[splits[:-1]]
    assert shard_nnz.max() - shard_nnz.min() <= 10     # nnz-balanced


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_row_range_partition_gloo(world):
    _run_partition(world, use_hip=False)


@pytest.mark.gpu
def test_row_range_partition_gloo_hip_ranks():
    """The same orchestration with every rank's y from the HIP library on
    device 0 (gloo for the exchanges; the oracle only checks): the STREAM
    kernel's y is bit-identical to omp_spmv on these rows, so the gathered y
    equals the oracle exactly."""
    _run_partition(2, use_hip=True)


def test_weak_scaling_shards_have_equal_work():
    from hspmv import dist as hdist
    for world in (1, 2, 4, 8):
        rows = [hdist.build_shard("small", r, world).A.m for r in range(world)]
        assert abs(max(rows) - min(rows)) <= 64
        assert sum(rows) == 64 * 64 * world


def test_c4_split_is_nnz_balanced_without_building_the_matrix():
    from hspmv import dist as hdist
    row_nnz = hdist.banded_row_nnz(20_000_000)
    assert 199_999_000 < row_nnz.sum() <= 200_000_000
    s = hdist.splits_from_row_nnz(row_nnz, 8)
    rp = np.concatenate([[0], np.cumsum(row_nnz)])
    per = rp[s[1:]] - rp[s[:-1]]
    assert per.max() - per.min() <= 20


def _halo_worker(rank, world, port, config, q):
    sys.path.insert(0, str(REPO / "heterogeneous-spmv_amd"))
    sys.path.insert(0, str(REPO / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from hspmv import dist as hdist
        from hspmv import gen
        sh = hdist.build_shard(config, rank, world)
        halo = hdist.plan_halo(sh.A, sh.splits, rank, world)
        xg = gen.rand_x(sh.n_global, 42)  # only the owned part is used below
        xw = torch.zeros(halo.hi - halo.lo, dtype=torch.float64)
        o0, o1 = halo.own
        xw[o0 - halo.lo:o1 - halo.lo] = torch.from_numpy(xg[o0:o1])
        hdist.halo_exchange(xw, halo)
        x_ok = bool(np.array_equal(xw.numpy(), xg[halo.lo:halo.hi]))
        Al = hdist.localize(sh.A, halo.lo, halo.hi)
        y_loc = oracle.spmv(Al.row_ptr, Al.col_idx, Al.val, xw.numpy())
        y_ref = oracle.spmv(sh.A.row_ptr, sh.A.col_idx, sh.A.val, xg)
        q.put((rank, x_ok, bool(np.array_equal(y_loc, y_ref)), hdist.halo_bytes(halo),
               [(p, g0, g1) for p, g0, g1 in halo.recvs]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_halo_exchange_replaces_x_broadcast_gloo(world):
    """Banded optional mode: x distributed like the rows, each
    rank receives only its window's halo from its neighbours by send/recv,
    and the SpMV on the localised shard equals the one with the full x."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, "small", q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, x_ok, y_ok, nbytes, recvs in res:
        assert x_ok and y_ok
        # 5-pt Laplacian on 64 x 64*world: the halo is one grid line per neighbour
        peers = [p for p, _, _ in recvs]
        assert peers == [r for r in (rank - 1, rank + 1) if 0 <= r < world]
        assert nbytes == 64 * 8 * len(peers)


def _overlap_worker(rank, world, port, K, q):
    sys.path.insert(0, str(REPO / "heterogeneous-spmv_amd"))
    sys.path.insert(0, str(REPO / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from hspmv import dist as hdist
        from hspmv import gen
        sh = hdist.build_shard("small", rank, world)
        xg = gen.rand_x(sh.n_global, 42)
        sub = hdist.chunk_splits(sh.A, K)
        og = hdist.OverlappedGather(np.diff(sub))
        for k in range(K):  # chunk k computed (the GPU's stand-in), then its gather starts
            a, b = int(sub[k]), int(sub[k + 1])
            Ak = sh.A.rows(a, b)
            og.buffer(k)[: b - a] = torch.from_numpy(oracle.spmv(Ak.row_ptr, Ak.col_idx, Ak.val, xg))
            og.start(k)
        y = og.finish().numpy()
        q.put((rank, y, [int(v) for v in np.diff(sub)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,K", [(2, 4), (3, 3), (2, 1), (4, 2), (8, 4)])
def test_overlapped_chunked_gather_gloo(world, K):
    """The y all-gather overlapped with the SpMV (bench.py comm
    end_to_end_overlapped_gflops): each rank's rows in K nnz-balanced chunks,
    chunk k gathered (async, padded per chunk) as soon as it is written; the
    assembled y equals the oracle on the global matrix on every rank."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    from hspmv import gen
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = gen.laplace2d(64, 64 * world)
    y_ref = oracle.spmv(A.row_ptr, A.col_idx, A.val, gen.rand_x(A.n, 42))
    for rank, y, rows in res:
        assert len(rows) == K and sum(rows) > 0
        assert np.array_equal(y, y_ref), rank
