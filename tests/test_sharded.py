"""The library's own row-range partition (hspmv_create_sharded /
hspmv_create(num_gpus > 1)): shards split nnz-balanced (on super-super-row
boundaries with CSR-3 maps), x broadcast and the padded y all-gathered and
unpadded by hspmv_get_y.  On a one-GPU box this runs as
  * devices [0]: the sharded branch with an RCCL communicator of one rank
    (ncclCommInitAll / ncclBroadcast / ncclAllGather really execute), and
  * devices [0, 0, (0)]: several shards on one device, exchanged by
    device-to-device copies (the partition, uneven SSR-aligned splits, an
    empty shard and the unpadding all run).
Each y is checked against the oracle; rows of <= 40 nonzeros bitwise."""
import numpy as np
import pytest

import hspmv
import oracle
from conftest import fp64_tol_ok
from hspmv import gen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert hspmv.device_count() >= 1, "no HIP device visible: run on the MI355X box"


def check(A, x, y):
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    assert fp64_tol_ok(y, y64, absrow)
    short = np.diff(A.row_ptr) <= 40
    assert np.array_equal(y[short], y64[short])


def _cases():
    A = gen.laplace2d(200, 150)
    yield "laplace", A, None
    S = gen.stencil27(20)
    yield "stencil-csr3", S, hspmv.build_csr3_maps(S, 20, 10)
    P = gen.powerlaw(30_000, seed=3, dtype=np.float64)
    yield "powerlaw-csr3", P, hspmv.build_csr3_maps(P, 64, 4)


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_sharded_handles_match_oracle(devices):
    for name, A, maps in _cases():
        x1, x2 = gen.rand_x(A.n, 31), gen.rand_x(A.n, 32)
        with hspmv.SpMV(A, maps, devices=devices) as op:
            assert op.info["num_gpus"] == len(devices), name
            check(A, x1, op(x1))
            check(A, x2, op(x2))  # a second x: broadcast again
            b, g = op.exchange()
            assert b >= 0.0 and g >= 0.0
            t = op.run(warmup=2, iters=3)
            assert t["num_gpus"] == len(devices) and t["t_min"] > 0
            check(A, x2, op.get_y())
            with pytest.raises(hspmv.HspmvError):  # y lives in the gather buffer
                op.bind_y_device(1)


def test_sharded_splits_on_ssr_boundaries_with_an_empty_shard():
    A = gen.laplace2d(16, 16)
    maps = hspmv.Csr3Maps(np.array([0, 1, 2], np.int32), np.array([0, 128, 256], np.int32))
    splits = hspmv.partition_rows(A.row_ptr, 3, maps)
    assert list(splits) == [0, 128, 256, 256]  # the third shard is empty
    x = gen.rand_x(A.n, 5)
    for devices in ([0, 0, 0], [0, 0]):
        with hspmv.SpMV(A, maps, devices=devices) as op:
            check(A, x, op(x))


def test_sharded_csort_and_fp32():
    A = gen.powerlaw(60_000, seed=9, dtype=np.float32)
    x = gen.rand_x(A.n, 3).astype(np.float32)
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val.astype(np.float64), x.astype(np.float64))
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    with hspmv.SpMV(A, devices=[0, 0], kernel="csort") as op:
        y = op(x)
        assert op.info["kernel_name"] == "csort"
    # fp32 row partials per column part (part32): an fp32 rounding of y and
    # of each part's sum
    assert np.all(np.abs(y - y64) <= 2.0 ** -24 * (np.abs(y64) + absrow) + 1e-12 * absrow)
    with hspmv.SpMV(A, devices=[0, 0, 0], kernel="stream") as op:
        y = op(x)
    y32 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    short = np.diff(A.row_ptr) <= 40
    assert np.array_equal(y[short].view(np.uint32), y32[short].view(np.uint32))


def test_sharded_reproducible_csort():
    """Row-range shards with deterministic = 2: every shard runs the
    column-sorted kernel with fixed-point sums (each shard's pre-pass reads
    the whole x, so every shard has the same scale); y is the same bits on
    every run and within the fp64 bar plus the fixed-point term."""
    A = gen.powerlaw(60_000, seed=9, dtype=np.float64)
    x = gen.rand_x(A.n, 3)
    with hspmv.SpMV(A, devices=[0, 0, 0], kernel="csort", options={"deterministic": "reproducible"}) as op:
        assert op.info["kernel_name"] == "csort" and op.info["deterministic"] == 1
        y1, y2 = op(x), op(x)
    assert np.array_equal(y1.view(np.uint64), y2.view(np.uint64))
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    lens = np.diff(A.row_ptr)
    vmax = np.zeros(A.m)
    vmax[lens > 0] = np.maximum.reduceat(np.abs(A.val), A.row_ptr[:-1][lens > 0])
    fixed = lens * 2.0 ** -48 * vmax * np.abs(x).max()
    assert np.all(np.abs(y1 - y64) <= 1e-6 * np.abs(y64) + 1e-12 * absrow + fixed)


def test_sharded_rejects_bad_device_lists():
    A = gen.laplace2d(8, 8)
    for devices in ([], [-1], [0, 99]):
        with pytest.raises((hspmv.HspmvError, ValueError)):
            hspmv.SpMV(A, devices=devices)
