"""The AUTO planner on shapes the BASELINE configurations do not cover (its
thresholds were fitted on C2-C5): mid-density banded rows (16-64 nonzeros,
the RCM'd-mesh band), rows whose columns are NOT sorted, and an irregular
matrix with unsorted rows.  Each case asserts the kernel AUTO picks, that
the tables it built agree with that choice, and parity with the oracle:
bit for bit on every row of <= 40 nonzeros (the ordered sums add a row's
products in STORED order, as omp_spmv does, sorted or not), within the fp64
bar elsewhere; the column-sorted kernel (irregular gathers) within its
documented bound.  The same matrices with hspmv_options.deterministic = 1
must keep a bit-reproducible row kernel."""
import numpy as np
import pytest

import hspmv
import oracle
from conftest import fp64_tol_ok
from hspmv import gen

pytestmark = pytest.mark.gpu
SERIAL_MAX = 40


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert hspmv.device_count() >= 1, "no HIP device visible: run on the MI355X box"


def run(A, x, maps=None, **kw):
    with hspmv.SpMV(A, maps, **kw) as op:
        return op(x), op.info


def check(A, x, y, info):
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    assert fp64_tol_ok(y, y64, absrow), np.abs(y - y64).max()
    if info["deterministic"]:
        short = np.diff(A.row_ptr) <= SERIAL_MAX
        assert np.array_equal(y[short].view(np.uint64), y64[short].view(np.uint64))


def shuffle_rows(A, seed):
    """A with every row's (column, value) pairs in a random order."""
    rng = np.random.default_rng(seed)
    key = rng.random(A.nnz) + np.repeat(np.arange(A.m), np.diff(A.row_ptr))
    p = np.argsort(key, kind="stable")
    return hspmv.CsrMatrix(A.m, A.n, A.row_ptr, A.col_idx[p], A.val[p])


@pytest.mark.parametrize("per_row", [16, 32, 48, 64])
def test_mid_density_band(per_row):
    # ~300 MB streamed: HBM-resident, like the reference's >= 10 M-nonzero inputs
    m = 25_000_000 // per_row
    A = gen.banded(m, per_row=per_row, half=per_row + 16, seed=per_row)
    x = gen.rand_x(A.n, 3)
    y, info = run(A, x)
    # banded gathers are regular: an ordered row kernel, never csort
    assert info["kernel_name"] in ("stream", "csr3"), info["kernel_name"]
    assert info["deterministic"] == 1
    # a 64-row group of > 2048 nonzeros is a heavy group: CSR3 wave tasks
    assert (info["kernel_name"] == "csr3") == (64 * per_row > 2048)
    # no maps: the CSR3 kernel runs the cut 64-row groups, reported as such
    assert info["csr3_plan"] == (4 if info["kernel_name"] == "csr3" else 0)
    check(A, x, y, info)
    maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(per_row, "volta"))
    y3, i3 = run(A, x, maps)
    assert i3["kernel_name"] == "csr3" and i3["csr3_plan"] == 1
    check(A, x, y3, i3)
    assert np.array_equal(y3, y) or per_row > SERIAL_MAX


def test_unsorted_columns_banded():
    A = shuffle_rows(gen.banded(3_000_000, per_row=10, half=32, seed=4), 1)
    x = gen.rand_x(A.n, 5)
    y, info = run(A, x)
    assert info["kernel_name"] == "stream" and info["deterministic"] == 1
    check(A, x, y, info)
    # the x slabs need sorted rows: forcing them on unsorted rows is refused
    ys, isl = run(A, x, options={"x_slabs": 4})
    assert isl["x_slabs"] == 0
    assert np.array_equal(ys, y)


def test_unsorted_columns_irregular():
    A = gen.powerlaw(2_000_000, seed=77, dtype=np.float64)
    A = shuffle_rows(A, 2)
    x = gen.rand_x(A.n, 6)
    y, info = run(A, x)
    # irregular gathers from HBM: the column-sorted kernel (it sorts by
    # column itself, so stored order does not matter), not bit-reproducible
    assert info["kernel_name"] == "csort" and info["deterministic"] == 0
    check(A, x, y, info)
    yd, idet = run(A, x, options={"deterministic": 1})
    assert idet["kernel_name"] != "csort" and idet["deterministic"] == 1
    check(A, x, yd, idet)
    yd2, _ = run(A, x, options={"deterministic": 1})
    assert np.array_equal(yd, yd2)


def test_rcm_mesh_stencil_small_and_csr2():
    # an RCM'd 3-D mesh small enough for the Infinity Cache: no x dictionaries
    # (HBM-only), XCD-contiguous order; CSR-3 and CSR-2 maps bit-identical
    A = gen.stencil27(70)
    x = gen.rand_x(A.n, 9)
    y, info = run(A, x)
    assert info["kernel_name"] == "stream" and info["x_dict"] == 0
    check(A, x, y, info)
    for maps in (hspmv.build_csr3_maps(A, 20, 10), hspmv.build_csr2_maps(A, 20)):
        y3, i3 = run(A, x, maps)
        assert i3["kernel_name"] == "csr3"
        assert np.array_equal(y3, y)


@pytest.mark.parametrize("cfg", ["c5", "c5r"])
def test_slab_handles_pick_the_row_kernel_by_group_balance(cfg):
    """A deterministic handle over irregular gathers (csort off, x slabs on)
    with CSR-3 tasks runs STREAM when its 64-row groups are balanced and the
    CSR3 tasks when heavy groups (> 2048 nonzeros) hold >= 1/8 of the
    nonzeros (hspmv_tables.cpp slab_kernel_rule): C5's random rows (6.5 %)
    and c5r's RCM-ordered rows (19.2 %) go opposite ways, as their r04
    timings did.  A rule, so two deterministic handles always agree bit for
    bit; y bitwise against the forced kernel of the same choice, and on rows
    of <= 40 nonzeros against the other kernel and the reference loop."""
    from hspmv import dist as hdist
    sh = hdist.build_shard(cfg, 0, 1)
    A, maps = sh.A, sh.maps
    x = gen.rand_x(A.n, 11).astype(A.val.dtype)
    y, info = run(A, x, maps, options={"deterministic": 1})
    assert info["deterministic"] == 1 and info["x_slabs"] > 0
    want = {"c5": ("stream", 2), "c5r": ("csr3", 1)}[cfg]
    assert (info["kernel_name"], info["slab_kernel_rule"]) == want
    lens = np.diff(A.row_ptr)
    lens_in = np.where(lens > 4096, 0, lens).astype(np.int64)
    g = np.add.reduceat(lens_in, np.arange(0, A.m, 64))
    assert abs(info["heavy_group_frac"] - g[g > 2048].sum() / g.sum()) < 1e-9
    y2, _ = run(A, x, maps, options={"deterministic": 1})
    assert np.array_equal(y2.view(np.uint32), y.view(np.uint32))
    short = lens <= SERIAL_MAX
    for kernel in ("csr3", "stream"):
        yk, ik = run(A, x, maps, kernel=kernel, options={"deterministic": 1})
        assert ik["kernel_name"] == kernel
        if kernel == want[0]:
            assert np.array_equal(yk.view(np.uint32), y.view(np.uint32))
        assert np.array_equal(yk[short].view(np.uint32), y[short].view(np.uint32))
    y32 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    assert np.array_equal(y[short].view(np.uint32), y32[short].view(np.uint32))
