"""The column-sorted row-block kernel (HSPMV_KERNEL_CSORT, csrc/csort.hip)
against the oracle.

csort walks each row block's nonzeros in column order and adds the products
into fp64 LDS row slots with atomics, so its y is NOT omp_spmv's left-to-right
sum bit for bit.  What is checked instead, on the same seeded inputs:

* fp64 data: within the north-star bar |y - y64| <= 1e-6 |y64| + 1e-12 sum|a x|
  (the products are omp_spmv's; only the order of the fp64 additions differs);
* fp32 data: each column part's row sum is the fp64 sum of the exact
  products, stored as an fp32 partial (part32, the default since r06) and
  the parts added in fp64 and rounded to y: within 2^-24 (sum_h |p_h| + |y|)
  (+ the fp64 summation error) of the exact sum -- half an fp32 ulp of y
  with one part -- and within omp_spmv's own fp32 summation error of the
  reference's y;
* run-to-run behaviour: fp32 y equal except at fp32 rounding ties, fp64 y
  within the fp64 rounding of the sum (the atomic order varies), reported as
  hspmv_info.deterministic = 0; hspmv_options.deterministic keeps AUTO off
  csort and refuses an explicit csort;
* long rows cut into slices (first/last/adjacent rows, and with
  HSPMV_FLAG_NO_SPLIT kept whole), empty rows and blocks, 1/2/4 column parts,
  chunk sizes, an Inf in x (padding must not spread it), and the planner's
  auto choice (irregular gathers only).
"""
import numpy as np
import pytest

import hspmv
import oracle
from conftest import GOLDEN, fp64_tol_ok
from hspmv import gen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert hspmv.device_count() >= 1, "no HIP device visible: run on the MI355X box"


def run(A, x, maps=None, **kw):
    with hspmv.SpMV(A, maps, **kw) as op:
        return op(x), op.info


def exact64(A, x):
    return oracle.spmv(A.row_ptr, A.col_idx, A.val.astype(np.float64), x.astype(np.float64))


def fp32_bound(y64, absrow, parts):
    """|y - y64| for fp32 csort: one fp32 rounding of y, plus (two or more
    column parts: fp32 row partials) one of each part's sum p_h, whose
    magnitudes add to at most sum|a x|; plus the fp64 summation error."""
    two = absrow if parts > 1 else 0.0
    # (+ 2^-148: rounding into fp32's subnormal range is absolute, 2^-150 each)
    return 2.0 ** -24 * (np.abs(y64) + two) + 1e-12 * absrow + 2.0 ** -148


def check(A, x, y, parts=2):
    y64 = exact64(A, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    if A.val.dtype == np.float64:
        assert fp64_tol_ok(y, y64, absrow), np.abs(y - y64).max()
    else:
        err = np.abs(y.astype(np.float64) - y64)
        assert np.all(err <= fp32_bound(y64, absrow, parts)), err.max()
        y32 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
        lens = np.diff(A.row_ptr)
        e32 = np.abs(y.astype(np.float64) - y32.astype(np.float64))
        assert np.all(e32 <= (lens + 2) * 2.0 ** -23 * absrow + 1e-30)
    return y64


def _long_rows(seed=3, m=900, n=200_000):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 30, m)
    lens[rng.integers(0, m, 30)] = rng.integers(33, 4000, 30)
    for r, ln in [(0, 90_000), (1, 4097), (63, 5000), (64, 9000), (65, 4096), (400, 30_000),
                  (401, 60_000), (m - 1, 8193)]:
        lens[r] = ln
    rp = np.concatenate([[0], np.cumsum(lens)])
    ci = np.concatenate([np.sort(rng.choice(n, ln, replace=False)) for ln in lens])
    return hspmv.CsrMatrix(m, n, rp, ci, rng.uniform(-1, 1, rp[-1]))


def _matrices():
    yield "powerlaw1500", hspmv.read_csr(GOLDEN / "powerlaw1500.csr", np.float64)
    yield "long_row", hspmv.read_csr(GOLDEN / "long_row.csr", np.float64)
    yield "empty_rows", hspmv.read_csr(GOLDEN / "empty_rows.csr", np.float64)
    yield "single_row", hspmv.read_csr(GOLDEN / "single_row.csr", np.float64)
    yield "lap32", hspmv.read_csr(GOLDEN / "lap32.mtx.rcm.csr", np.float64)
    yield "powerlaw60k", gen.powerlaw(60_000, seed=5, dtype=np.float64)
    yield "long_rows", _long_rows()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("parts", ["1", "2", "4"])
def test_csort_matches_oracle(dtype, parts):
    for name, A in _matrices():
        A = A.astype(dtype)
        x = gen.rand_x(A.n, 17).astype(dtype)
        y, info = run(A, x, kernel="csort", options={"csort_parts": int(parts)})
        assert info["kernel_name"] == "csort", name
        assert info["csort_parts"] == min(int(parts), A.n), name
        assert info["n_split_rows"] == int((np.diff(A.row_ptr) > 4096).sum()), name
        check(A, x, y, info["csort_parts"])


@pytest.mark.parametrize("u", [4, 8, 16])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_csort_chunk_sizes(u, dtype):
    A = gen.powerlaw(50_000, seed=9, dtype=dtype)
    x = gen.rand_x(A.n, 3).astype(dtype)
    y, info = run(A, x, kernel="csort", options={"csort_chunk_u": u})
    assert info["chunk_u"] == u
    check(A, x, y)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_csort_caller_y_at_any_element_offset(dtype):
    """hspmv_bind_y_device takes any element-aligned pointer: the finishing
    pass's 4- and 2-row vector stores are used only when y is aligned for
    them (csort.hip launch_csort_u), so a torch slice at offset 1..3 and an
    m that is not a multiple of 4 give the right y, and the elements on
    either side of the bound range keep their canary."""
    import torch
    for m in (40_000, 40_001, 40_002):
        A = gen.powerlaw(m, seed=4, dtype=dtype)
        x = gen.rand_x(A.n, 6).astype(dtype)
        tdt = torch.float32 if dtype == np.float32 else torch.float64
        xd = torch.from_numpy(x).to("cuda")
        for off in (0, 1, 2, 3):
            buf = torch.full((A.m + 8,), 7.0, dtype=tdt, device="cuda")
            with hspmv.SpMV(A, kernel="csort", options={"csort_parts": 2}) as op:
                assert op.info["kernel_name"] == "csort"
                op.bind_x_device(xd.data_ptr())
                op.bind_y_device(buf.data_ptr() + off * buf.element_size())
                op.spmv()
                torch.cuda.synchronize()
            h = buf.cpu().numpy()
            assert np.all(h[:off] == 7.0) and np.all(h[off + A.m:] == 7.0), (m, off)
            check(A, x, h[off:off + A.m])


def test_csort_long_rows_whole_and_sliced():
    A = _long_rows(seed=8)
    x = gen.rand_x(A.n, 2)
    lens = np.diff(A.row_ptr)
    y1, i1 = run(A, x, kernel="csort")
    assert i1["n_split_rows"] == int((lens > 4096).sum())
    check(A, x, y1)
    y2, i2 = run(A, x, kernel="csort", split_rows=False)  # long rows stay one slot
    assert i2["n_split_rows"] == 0
    check(A, x, y2)


def test_csort_repeatable_fp32():
    A = gen.powerlaw(200_000, seed=4, dtype=np.float32)
    x = gen.rand_x(A.n, 8).astype(np.float32)
    with hspmv.SpMV(A, kernel="csort") as op:
        ys = [op(x) for _ in range(4)]
    # fp64 slot sums rounded to fp32 partials, added in fp64, rounded to y:
    # equal run to run except where an fp64 sum sits within its own rounding
    # of an fp32 tie (partial or y)
    for y in ys[1:]:
        assert np.mean(ys[0] == y) > 0.999
    check(A, x, ys[0])


def test_csort_run_to_run_fp64_and_deterministic_option():
    """fp64: every run is within the fp64 rounding of the sum of the same
    products (only the atomic order of the additions varies), so two runs
    differ by at most a few fp64 ulps of sum|a x| per row -- and the handle
    says so (info.deterministic = 0).  deterministic=1 keeps AUTO on a row
    kernel (bit-identical run to run and to omp_spmv on short rows) and
    refuses an explicit csort."""
    A = gen.powerlaw(2_000_000, seed=12, dtype=np.float64)
    x = gen.rand_x(A.n, 8)
    lens = np.diff(A.row_ptr)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    with hspmv.SpMV(A) as op:
        info = op.info
        ys = [op(x) for _ in range(3)]
    assert info["kernel_name"] == "csort" and info["deterministic"] == 0
    for y in ys[1:]:
        d = np.abs(y - ys[0])
        assert np.all(d <= 2.0 * (lens + 1) * 2.0 ** -53 * absrow)
    check(A, x, ys[0])
    with hspmv.SpMV(A, options={"deterministic": 1}) as op:
        info = op.info
        yd = [op(x) for _ in range(2)]
    assert info["kernel_name"] != "csort" and info["deterministic"] == 1
    assert np.array_equal(yd[0], yd[1])
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    short = lens <= 40
    assert np.array_equal(yd[0][short], y64[short])
    assert fp64_tol_ok(yd[0], y64, absrow)
    with pytest.raises(hspmv.HspmvError):
        hspmv.SpMV(A, kernel="csort", options={"deterministic": 1})
    # the csort option asks for the same kernel: refused together with
    # deterministic too (the tables, once built, would be picked)
    with pytest.raises(hspmv.HspmvError):
        hspmv.SpMV(A, options={"csort": 1, "deterministic": 1})


def _hub_rows(seed=5, m=40_000, n=400_000):
    """Random short rows plus hub rows whose 1000-4000 columns are
    CONTIGUOUS (what an RCM ordering does to a power-law graph's hubs): in
    column order their entries fill whole instructions with one row, so the
    builder stores those chunks slot-sorted and the kernel pre-sums each
    row's lanes (segmented chunks)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 30, m)
    hubs = rng.choice(m, 12, replace=False)
    lens[hubs] = rng.integers(1000, 4000, hubs.size)
    cols = []
    for r, ln in enumerate(lens):
        if r in set(hubs.tolist()):
            c0 = int(rng.integers(0, n - ln))
            cols.append(np.arange(c0, c0 + ln))
        else:
            cols.append(np.sort(rng.choice(n, ln, replace=False)))
    rp = np.concatenate([[0], np.cumsum(lens)])
    return hspmv.CsrMatrix(m, n, rp, np.concatenate(cols), rng.uniform(-1, 1, rp[-1]))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_csort_segmented_chunks_for_contiguous_hub_rows(dtype):
    A = _hub_rows().astype(dtype)
    x = gen.rand_x(A.n, 12).astype(dtype)
    for parts in (1, 2):
        y, info = run(A, x, kernel="csort", options={"csort_parts": parts})
        assert info["kernel_name"] == "csort" and info["csort_row_blocks"] > 0
        # the hub rows' chunks really were stored slot-sorted (the segmented
        # scan ran), and only those: most chunks stay in column order
        assert 0 < info["csort_seg_chunks"] < info["csort_chunks"] // 2, info
        check(A, x, y)
    # short rows over random columns: no instruction crowds one slot, so no
    # chunk is segmented (power-law hubs with thousands of random columns
    # can crowd one: those chunks are segmented by the same rule)
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 30, 40_000)
    rp = np.concatenate([[0], np.cumsum(lens)])
    ci = np.concatenate([np.sort(rng.choice(400_000, ln, replace=False)) for ln in lens])
    B = hspmv.CsrMatrix(40_000, 400_000, rp, ci, rng.uniform(-1, 1, rp[-1]).astype(dtype))
    y, info = run(B, gen.rand_x(B.n, 3).astype(dtype), kernel="csort")
    assert info["csort_chunks"] > 0 and info["csort_seg_chunks"] == 0
    check(B, gen.rand_x(B.n, 3).astype(dtype), y)


def _uniform_with_long_rows(dtype, seed=13, m=600_000, n=1_500_000):
    """Short rows over random columns plus long rows cut into slices,
    first / last / adjacent rows among them."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(2, 16, m)
    for r, ln in [(0, 9000), (1, 4097), (777, 30_000), (778, 5000), (m - 1, 12_000)]:
        lens[r] = ln
    rp = np.concatenate([[0], np.cumsum(lens)])
    # columns sorted within each row (duplicates allowed: summed like any)
    key = np.repeat(np.arange(m, dtype=np.int64), lens) * n + rng.integers(0, n, rp[-1])
    ci = (np.sort(key) % n).astype(np.int32)
    return hspmv.CsrMatrix(m, n, rp, ci, rng.uniform(-1, 1, rp[-1]).astype(dtype))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_csort_long_row_slices_repeated_launches(dtype):
    """Short rows over random columns plus long rows cut into slices (first,
    last, adjacent rows among them): every SpMV of a back-to-back run is
    checked (the LDS atomic order changes from launch to launch), then a new
    x (nothing stale from the last launch)."""
    A = _uniform_with_long_rows(dtype)
    x = gen.rand_x(A.n, 21).astype(dtype)
    lens = np.diff(A.row_ptr)
    with hspmv.SpMV(A, kernel="csort") as op:
        info = op.info
        assert info["csort_parts"] == 2 and info["n_split_rows"] == int((lens > 4096).sum())
        op.set_x(x)
        for _ in range(10):
            op.spmv()
            check(A, x, op.get_y())
        x2 = gen.rand_x(A.n, 22).astype(dtype)
        op.set_x(x2)
        op.spmv()
        check(A, x2, op.get_y())


def test_csort_rcm_powerlaw_matches_oracle():
    A = gen.powerlaw(150_000, seed=21, dtype=np.float32, rcm=True)
    x = gen.rand_x(A.n, 4).astype(np.float32)
    y, info = run(A, x, kernel="csort")
    check(A, x, y)


def test_csort_padding_does_not_spread_inf():
    A = gen.powerlaw(30_000, seed=6, dtype=np.float64)
    x = gen.rand_x(A.n, 5)
    c = int(A.col_idx[A.row_ptr[100]])
    x[c] = np.inf
    y, _ = run(A, x, kernel="csort")
    touched = np.zeros(A.m, bool)
    rows = np.repeat(np.arange(A.m), np.diff(A.row_ptr))
    touched[rows[A.col_idx == c]] = True
    assert not np.any(np.isnan(y[~touched])) and np.all(np.isfinite(y[~touched]))
    xs = x.copy()
    xs[c] = 0.0
    ys = exact64(A, xs)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, xs)
    assert fp64_tol_ok(y[~touched], ys[~touched], absrow[~touched])


def test_csort_empty_and_degenerate():
    # all-empty rows, one column, more row blocks than rows
    for m, n, lens in [(500, 1, np.ones(500, int)), (3, 7, np.array([0, 7, 0])),
                       (2000, 3000, np.zeros(2000, int))]:
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        ci = np.concatenate([np.arange(ln) % n for ln in lens]).astype(np.int32) if rp[-1] else \
            np.zeros(0, np.int32)
        A = hspmv.CsrMatrix(m, n, rp, ci, np.linspace(-1, 1, rp[-1]))
        x = gen.rand_x(n, 1)
        y, info = run(A, x, kernel="csort")
        check(A, x, y)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_csort_reproducible_empty_and_degenerate(dtype):
    """test_csort_empty_and_degenerate's shapes (plus x = 0, whose scale
    floors at 2^-1000) through the fixed-point path: the same bits twice,
    and the CPU restatement's bits."""
    from fixedpoint_model import reproducible_csort_y
    cases = [(500, 1, np.ones(500, int), 1), (3, 7, np.array([0, 7, 0]), 1),
             (2000, 3000, np.zeros(2000, int), 1), (4000, 5000, np.arange(4000) % 9, 0)]
    for m, n, lens, xs in cases:
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        ci = np.concatenate([np.arange(ln) * 37 % n for ln in lens]).astype(np.int32) if rp[-1] else \
            np.zeros(0, np.int32)
        A = hspmv.CsrMatrix(m, n, rp, ci, np.linspace(-1, 1, rp[-1]).astype(dtype))
        x = (gen.rand_x(n, 1) * xs).astype(dtype)
        with hspmv.SpMV(A, kernel="csort", options=REPRO) as op:
            info = op.info
            y1, y2 = op(x), op(x)
        assert np.array_equal(y1.view(np.uint8), y2.view(np.uint8)), (m, n)
        if rp[-1] > 0:
            assert info["kernel_name"] == "csort" and info["csort_fixed_point"] == 1, (m, n, info["kernel_name"])
            pb = info["csort_part_begin"]
            ym = reproducible_csort_y(A.row_ptr, A.col_idx, A.val, x, pb if pb else (0,))
            assert np.array_equal(y1.view(np.uint8), ym.view(np.uint8)), (m, n)
        else:
            assert np.all(y1 == 0), (m, n, info["kernel_name"])


def test_csort_auto_only_for_irregular_gathers():
    # banded / stencil matrices keep the ordered row kernels; a small random
    # matrix (cache-resident) too; csr3 maps do not stop the choice
    _, i1 = run(gen.banded(200_000, seed=2), gen.rand_x(200_000, 1))
    assert i1["kernel_name"] == "stream"
    _, i2 = run(gen.powerlaw(50_000, seed=2, dtype=np.float64), gen.rand_x(50_000, 1))
    assert i2["kernel_name"] == "stream"
    A = gen.powerlaw(2_000_000, seed=12, dtype=np.float32)
    maps = hspmv.build_csr3_maps(A, 64, 4)
    x = gen.rand_x(A.n, 2).astype(np.float32)
    y, i3 = run(A, x, maps)
    assert i3["kernel_name"] == "csort"
    check(A, x, y)
    # an explicit row kernel is honoured
    _, i4 = run(A, x, maps, kernel="csr3")
    assert i4["kernel_name"] == "csr3"


def test_csort_c5_shape_multi_shard():
    # two row-range shards of a power-law matrix, each its own csort handle,
    # assemble the full y (the per-rank layout of bench.py / hspmv.dist)
    A = gen.powerlaw(400_000, seed=7, dtype=np.float32)
    x = gen.rand_x(A.n, 4).astype(np.float32)
    splits = hspmv.partition_rows(A.row_ptr, 2)
    y = np.concatenate([run(A.rows(int(splits[r]), int(splits[r + 1])), x, kernel="csort")[0]
                        for r in range(2)])
    check(A, x, y)


# ---------------------------------------------------------------- reproducible
# hspmv_options.deterministic = 2 ("reproducible"): csort with fixed-point
# (int64) LDS slots.  Each product v x is rounded once to an integer at the
# scale 2^(50 - xexp - rexp[r]) -- |x| < 2^xexp, |v 2^rexp[r]| < 2^-extra
# (extra > 0 only for a row kept whole beyond 4096 nonzeros) -- so y is the
# same bits on every run, and differs from the exact sum by at most
# len * 2^-49 * max_r|v| * max|x| * 2^extra (the rounding of the products)
# plus the roundings of the partials and of y.

def row_absmax(A):
    a = np.abs(A.val.astype(np.float64))
    lens = np.diff(A.row_ptr)
    out = np.zeros(A.m)
    nz = lens > 0
    if a.size:
        out[nz] = np.maximum.reduceat(a, A.row_ptr[:-1][nz])
    return out


def fixed_bound(A, x, split=True):
    lens = np.diff(A.row_ptr).astype(np.float64)
    extra = np.zeros_like(lens) if split else np.maximum(0, np.ceil(np.log2(np.maximum(lens, 1) / 4096)))
    xmax = float(np.abs(x.astype(np.float64)).max()) if x.size else 0.0
    return lens * 2.0 ** (-48 + extra) * row_absmax(A) * xmax


def check_fixed(A, x, y, parts, split=True):
    y64 = exact64(A, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    err = np.abs(y.astype(np.float64) - y64)
    fb = fixed_bound(A, x, split)
    if A.val.dtype == np.float64:
        tol = 2.0 ** -52 * (np.abs(y64) + (absrow if parts > 1 else 0.0)) + fb + 1e-300
        assert np.all(err <= tol), float((err - tol).max())
        assert fp64_tol_ok(y, y64, absrow)
    else:
        tol = fp32_bound(y64, absrow, parts) + fb
        assert np.all(err <= tol), float((err - tol).max())
        y32 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
        lens = np.diff(A.row_ptr)
        e32 = np.abs(y.astype(np.float64) - y32.astype(np.float64))
        assert np.all(e32 <= (lens + 2) * 2.0 ** -23 * absrow + 1e-30)
    return y64


REPRO = {"deterministic": "reproducible"}


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("parts", [1, 2])
def test_csort_reproducible_fixed_point(dtype, parts):
    """deterministic = 2: the column-sorted kernel with fixed-point slots --
    reported as deterministic, y the same bits on every run (LDS atomics in
    any order), within the fixed-point bound of the exact sum."""
    for name, A in _matrices():
        A = A.astype(dtype)
        x = gen.rand_x(A.n, 17).astype(dtype)
        with hspmv.SpMV(A, kernel="csort", options=dict(REPRO, csort_parts=parts)) as op:
            info = op.info
            assert info["kernel_name"] == "csort" and info["csort_fixed_point"] == 1, name
            assert info["deterministic"] == 1, name
            op.set_x(x)
            ys = []
            for _ in range(5):
                op.spmv()
                ys.append(op.get_y())
        for y in ys[1:]:
            assert np.array_equal(y.view(np.uint8), ys[0].view(np.uint8)), name
        check_fixed(A, x, ys[0], info["csort_parts"])


def test_csort_reproducible_auto_and_option_rules():
    """AUTO with deterministic = 2 keeps the column-sorted kernel for
    irregular gathers (fixed-point); deterministic = 1 keeps the row kernels
    and refuses csort; out-of-range values are refused."""
    A = gen.powerlaw(2_000_000, seed=12, dtype=np.float32)
    x = gen.rand_x(A.n, 2).astype(np.float32)
    with hspmv.SpMV(A, options=REPRO) as op:
        assert op.info["kernel_name"] == "csort" and op.info["csort_fixed_point"] == 1
        assert op.info["deterministic"] == 1
        y = op(x)
    check_fixed(A, x, y, 2)
    with hspmv.SpMV(A) as op:  # the default: fp64 slots in atomic order
        assert op.info["csort_fixed_point"] == 0 and op.info["deterministic"] == 0
    with pytest.raises(hspmv.HspmvError):
        hspmv.SpMV(A, kernel="csort", options={"deterministic": "ordered"})
    with pytest.raises(hspmv.HspmvError):
        hspmv.SpMV(A, options={"deterministic": 4})


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_csort_reproducible_scales(dtype):
    """The fixed-point scale follows the data: x of magnitude 1e-30 (the
    per-SpMV x exponent), rows whose values sit at 1e-20 and 1e+20 (the
    per-row value exponents), an all-zero x (y exactly 0), and a new x on the
    same handle."""
    A = gen.powerlaw(60_000, seed=5, dtype=np.float64)
    rows = np.repeat(np.arange(A.m), np.diff(A.row_ptr))
    scale = np.where(rows % 3 == 0, 1e-20, np.where(rows % 3 == 1, 1e20, 1.0))
    lim = 1e30 if dtype == np.float32 else 1e300
    A = hspmv.CsrMatrix(A.m, A.n, A.row_ptr, A.col_idx, np.clip(A.val * scale, -lim, lim)).astype(dtype)
    x = (gen.rand_x(A.n, 3) * 1e-30).astype(dtype)
    with hspmv.SpMV(A, kernel="csort", options=REPRO) as op:
        assert op.info["csort_fixed_point"] == 1
        y = op(x)
        check_fixed(A, x, y, op.info["csort_parts"])
        assert np.all(op(np.zeros(A.n, dtype)) == 0)
        x2 = gen.rand_x(A.n, 4).astype(dtype)
        check_fixed(A, x2, op(x2), op.info["csort_parts"])


def test_csort_reproducible_long_rows_whole_and_sliced():
    A = _long_rows(seed=8)
    x = gen.rand_x(A.n, 2)
    y1, i1 = run(A, x, kernel="csort", options=REPRO)
    assert i1["csort_fixed_point"] == 1 and i1["n_split_rows"] > 0
    check_fixed(A, x, y1, i1["csort_parts"])
    # rows kept whole beyond 4096 nonzeros: their scale leaves 2^extra headroom
    y2, i2 = run(A, x, kernel="csort", split_rows=False, options=REPRO)
    assert i2["n_split_rows"] == 0
    check_fixed(A, x, y2, i2["csort_parts"], split=False)


def test_csort_reproducible_nonfinite_x():
    """An Inf in x: the fixed-point scale is undefined, so that SpMV adds in
    fp64 slots (rows touching the Inf are Inf / NaN as omp_spmv gives them,
    the others within the fp64 tolerance); the next finite x is fixed-point
    again and bit-reproducible."""
    A = gen.powerlaw(30_000, seed=6, dtype=np.float64)
    x = gen.rand_x(A.n, 5)
    c = int(A.col_idx[A.row_ptr[100]])
    x[c] = np.inf
    with hspmv.SpMV(A, kernel="csort", options=REPRO) as op:
        y = op(x)
        touched = np.zeros(A.m, bool)
        rows = np.repeat(np.arange(A.m), np.diff(A.row_ptr))
        touched[rows[A.col_idx == c]] = True
        assert np.all(~np.isfinite(y[touched])) and np.all(np.isfinite(y[~touched]))
        xs = x.copy()
        xs[c] = 0.0
        ys = exact64(A, xs)
        absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, xs)
        assert fp64_tol_ok(y[~touched], ys[~touched], absrow[~touched])
        y1, y2 = op(xs), op(xs)
        assert np.array_equal(y1.view(np.uint64), y2.view(np.uint64))
        check_fixed(A, xs, y1, op.info["csort_parts"])


def test_csort_reproducible_segmented_hub_rows():
    A = _hub_rows().astype(np.float32)
    x = gen.rand_x(A.n, 12).astype(np.float32)
    with hspmv.SpMV(A, kernel="csort", options=dict(REPRO, csort_parts=2)) as op:
        assert op.info["csort_seg_chunks"] > 0 and op.info["csort_fixed_point"] == 1
        y1, y2 = op(x), op(x)
    assert np.array_equal(y1.view(np.uint32), y2.view(np.uint32))
    check_fixed(A, x, y1, 2)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_csort_reproducible_x_at_any_element_offset(dtype):
    """The x-exponent pre-pass reads x with 16-byte loads when x is 16-byte
    aligned and element by element otherwise (a caller's device x at any
    element offset, hspmv_bind_x_device): both give the same exponent, so
    the same y bits; an x length that is not a multiple of the pre-pass
    chunk exercises its tail."""
    import torch
    A = gen.powerlaw(40_001, seed=4, dtype=dtype)
    x = gen.rand_x(A.n, 6).astype(dtype)
    tdt = torch.float32 if dtype == np.float32 else torch.float64
    ys = []
    with hspmv.SpMV(A, kernel="csort", options=REPRO) as op:
        assert op.info["csort_fixed_point"] == 1
        for off in (0, 1, 2, 3):
            buf = torch.zeros(A.n + 8, dtype=tdt, device="cuda")
            buf[off:off + A.n] = torch.from_numpy(x).to("cuda")
            op.bind_x_device(buf.data_ptr() + off * buf.element_size())
            op.spmv()
            ys.append(op.get_y())
    for y in ys[1:]:
        assert np.array_equal(y.view(np.uint8), ys[0].view(np.uint8))
    check_fixed(A, x, ys[0], 2)


def test_csort_reproducible_refused_for_nonfinite_matrix_values():
    """A matrix value that is Inf or NaN has no fixed-point scale (its
    products must stay non-finite): deterministic = 2 then keeps fp64 slots
    and says so (csort_fixed_point = 0, deterministic = 0); the row holding
    it is non-finite, as omp_spmv's, the others within the tolerance."""
    A = gen.powerlaw(30_000, seed=8, dtype=np.float64)
    val = A.val.copy()
    val[A.row_ptr[77]] = np.inf
    B = hspmv.CsrMatrix(A.m, A.n, A.row_ptr, A.col_idx, val)
    x = gen.rand_x(B.n, 3)
    with hspmv.SpMV(B, kernel="csort", options=REPRO) as op:
        assert op.info["csort_fixed_point"] == 0 and op.info["deterministic"] == 0
        y = op(x)
    assert not np.isfinite(y[77])
    ok = np.ones(B.m, bool)
    ok[77] = False
    y64 = exact64(A, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    assert fp64_tol_ok(y[ok], y64[ok], absrow[ok])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("parts", [1, 2])
@pytest.mark.parametrize("which", ["powerlaw60k", "hub_rows", "long_rows", "scaled"])
def test_csort_reproducible_bitwise_vs_cpu_restatement(which, parts, dtype):
    """The fixed-point path's y is an exact function of the inputs and the
    column parts' boundaries -- one half-even rounding of each exact product,
    integer row sums per part, one conversion, one scaling and one rounding
    per part, the parts added in order -- restated on the CPU in
    tests/fixedpoint_model.py (fp64 products exactly, in Python integers):
    the GPU's y equals it bit for bit on every row the kernel does not slice
    (rows of > 4096 nonzeros add their slices in the finishing pass's
    shuffle tree; those are checked against the bound)."""
    from fixedpoint_model import reproducible_csort_y
    if which == "powerlaw60k":
        A = gen.powerlaw(60_000, seed=5, dtype=dtype)
    elif which == "hub_rows":
        A = _hub_rows().astype(dtype)
    elif which == "long_rows":
        A = _long_rows(seed=8).astype(dtype)
    else:  # values and x across many binades
        B = gen.powerlaw(60_000, seed=6, dtype=np.float64)
        rows = np.repeat(np.arange(B.m), np.diff(B.row_ptr))
        A = hspmv.CsrMatrix(B.m, B.n, B.row_ptr, B.col_idx,
                            (B.val * 10.0 ** ((rows % 13) - 6)).astype(dtype))
    x = gen.rand_x(A.n, 31).astype(dtype)
    if which == "scaled":
        x = (x * dtype(1e-20)).astype(dtype)
    with hspmv.SpMV(A, kernel="csort", options=dict(REPRO, csort_parts=parts)) as op:
        info = op.info
        assert info["csort_fixed_point"] == 1 and info["csort_parts"] == parts
        pb = info["csort_part_begin"]
        assert len(pb) == parts and pb[0] == 0 and all(a < b for a, b in zip(pb, pb[1:])) and pb[-1] < A.n
        y = op(x)
    ym = reproducible_csort_y(A.row_ptr, A.col_idx, A.val, x, pb)
    short = np.diff(A.row_ptr) <= 4096
    bad = np.flatnonzero(y[short] != ym[short])
    assert bad.size == 0, (which, int(np.flatnonzero(short)[bad[0]]), y[short][bad[0]], ym[short][bad[0]])
    assert np.array_equal(y[short].view(np.uint8), ym[short].view(np.uint8))  # signed zeros too
    check_fixed(A, x, y, parts)
