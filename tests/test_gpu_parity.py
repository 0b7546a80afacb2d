"""GPU parity: the HIP path (through the C ABI) against the oracle.

Bar (BASELINE.json north star): fp64 y within
    |y - y64| <= 1e-6 |y64| + 1e-12 * sum_k |a_k x_k|
of the spmv-csr restatement.  The STREAM / CSR3 kernels sum each row in the
reference order with the reference rounding, so on rows up to 40 nonzeros
(SERIAL_MAX, hspmv_internal.h kSerialMax; fp32 data: 56, kSerialMaxF32)
they are checked BITWISE: fp32 against the reference binary's own golden
output, fp64 against the restatement.
"""
import numpy as np
import pytest

import hspmv
import oracle
from conftest import GOLDEN, fp64_tol_ok, load_golden
from hspmv import gen

pytestmark = pytest.mark.gpu

KERNELS = [("stream", 0), ("vector", 1), ("vector", 2), ("vector", 4), ("vector", 8),
           ("vector", 16), ("vector", 32), ("vector", 64), ("auto", 0)]
SERIAL_MAX = 40  # rows up to this length go through the ordered (bit-exact) path
SERIAL_MAX_F32 = 56  # fp32 data: up to 56 (hspmv_internal.h kSerialMaxF32)


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    n = hspmv.device_count()
    assert n >= 1, "no HIP device visible: the gpu tests must run on the MI355X box"


def gpu_spmv(A, x, maps=None, **kw):
    with hspmv.SpMV(A, maps, **kw) as op:
        return op(x), op.info


def check_fp64(A, x, y, exact_rows=None):
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val.astype(np.float64), x.astype(np.float64))
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    assert fp64_tol_ok(y, y64, absrow), np.abs(y - y64).max()
    if exact_rows is not None:
        assert np.array_equal(y[exact_rows], y64[exact_rows])
    return y64


def short_rows(A):
    return np.diff(A.row_ptr) <= SERIAL_MAX


def test_golden_fp32_bitwise_vs_reference_binary(golden_names):
    """STREAM / CSR3 in fp32 reproduce the reference's own omp_spmv output
    bit for bit on every row of up to 56 nonzeros (x = 1 and x = rand)."""
    for name in golden_names:
        A = hspmv.read_csr(GOLDEN / f"{name}.csr", np.float32)
        g = load_golden(name)
        ok = np.diff(A.row_ptr) <= SERIAL_MAX_F32
        x = gen.rand_x(A.n, 42).astype(np.float32)
        for kernel in ("stream", "auto"):
            y, _ = gpu_spmv(A, x, kernel=kernel)
            assert np.array_equal(y[ok].view(np.uint32), g["y_ref_f32_rand"][ok].view(np.uint32)), name
            if "y_ref_f32_ones" in g:
                y1, _ = gpu_spmv(A, np.ones(A.n, np.float32), kernel=kernel)
                assert np.array_equal(y1[ok].view(np.uint32), g["y_ref_f32_ones"][ok].view(np.uint32))
            # long rows: within fp32 accumulation error of the reference
            if (~ok).any():
                absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
                nrow = np.diff(A.row_ptr)
                err = np.abs(y.astype(np.float64) - g["y_ref_f32_rand"])
                assert np.all(err <= (nrow + 2) * 2.0 ** -23 * absrow + 1e-30)


@pytest.mark.parametrize("k", [41, 48, 52, 56, 57])
def test_fp32_rows_of_41_to_56_serial(k):
    """fp32 rows of up to kSerialMaxF32 = 56 nonzeros are summed serially
    (omp_spmv's bits), 57 cooperatively (within the reference's own error):
    mid-density banded rows through AUTO / STREAM / CSR3, against the
    oracle's omp_spmv restatement (pinned bitwise to the reference)."""
    rng = np.random.default_rng(k)
    m, n = 60_000, 60_000
    lens = np.full(m, k)
    rp = np.concatenate([[0], np.cumsum(lens)])
    ci = (np.arange(m)[:, None] + np.arange(k)[None, :] * 3) % n
    ci.sort(axis=1)
    A = hspmv.CsrMatrix(m, n, rp, ci.reshape(-1).astype(np.int32), rng.uniform(-1, 1, m * k).astype(np.float32))
    x = gen.rand_x(n, 5).astype(np.float32)
    ref = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    for kernel in ("auto", "stream", "csr3"):
        y, _ = gpu_spmv(A, x, kernel=kernel)
        if k <= SERIAL_MAX_F32:
            assert np.array_equal(y.view(np.uint32), ref.view(np.uint32)), (k, kernel)
        else:
            absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
            assert np.all(np.abs(y.astype(np.float64) - ref) <= (k + 2) * 2.0 ** -23 * absrow + 1e-30)


def test_golden_fp64_all_kernels(golden_names):
    for name in golden_names:
        A = hspmv.read_csr(GOLDEN / f"{name}.csr", np.float64)
        g = load_golden(name)
        x = gen.rand_x(A.n, 42)
        absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
        for kernel, lanes in KERNELS:
            y, info = gpu_spmv(A, x, kernel=kernel, lanes=lanes)
            assert fp64_tol_ok(y, g["y_orc_f64_rand"], absrow), (name, kernel, lanes)
            if kernel in ("stream", "auto"):
                ok = short_rows(A)
                assert np.array_equal(y[ok], g["y_orc_f64_rand"][ok]), (name, kernel)


def test_golden_csr3_fixtures(manifest):
    for name, ent in manifest["fixtures"].items():
        if "csr3" not in ent:
            continue
        for dt in (np.float64, np.float32):
            A, maps = hspmv.read_csr3(GOLDEN / f"{name}.csr3", dt)
            x = gen.rand_x(A.n, 42).astype(dt)
            y, info = gpu_spmv(A, x, maps, kernel="csr3")
            assert info["kernel_name"] == "csr3"
            ok = short_rows(A)
            y_ref = oracle.csr3_spmv(maps.outer, maps.inner, A.row_ptr, A.col_idx, A.val, x)
            assert np.array_equal(y[ok], y_ref[ok]), (name, dt)
            if dt == np.float64:
                check_fp64(A, x, y)


@pytest.mark.parametrize("plan", ["aligned", "packed", "ssr"])
@pytest.mark.parametrize("waves_case", [(7, 8), (20, 10), (64, 4), (1, 1), (400, 2), (2, 100)])
def test_csr3_map_sizes(waves_case, plan):
    """Any map granularity (tiny super-rows, one-row super-rows, huge SSRs
    that need several waves and several 64-row groups, super-rows of more
    than 64 rows) gives the same y, under the three CSR-3 task plans
    (64-row aligned tasks, super-rows packed into tasks, a workgroup per
    super-super-row)."""
    ssrs, srs = waves_case
    # the banded matrix's tasks take the LDS x-window path (span <= 256 columns)
    for A in (gen.laplace2d(300, 200), gen.powerlaw(30000, seed=11, dtype=np.float64),
              gen.banded(20000, per_row=10, half=32, seed=3, dtype=np.float64)):
        maps = hspmv.build_csr3_maps(A, ssrs, srs)
        x = gen.rand_x(A.n, 5)
        y, info = gpu_spmv(A, x, maps, options={"csr3_plan": plan})
        assert info["kernel_name"] == "csr3"
        assert info["csr3_plan"] == hspmv._lib.CSR3_PLANS[plan]
        if plan != "ssr":  # aligned 64-row groups, or whole super-rows per task (<= 64 rows)
            sr_rows = np.diff(maps.inner)
            lower = int(np.ceil(A.m / 64))
            # plus the cuts of tasks over the 2048-nonzero budget (two
            # neighbouring pieces of a cut task always hold > 2048)
            lens = np.diff(A.row_ptr)
            cuts = 2 * int(lens[lens <= 4096].sum()) // 2048 + 1
            assert lower <= info["wave_tasks"] <= len(sr_rows) + int(np.sum(sr_rows // 64)) + 1 + cuts
        else:
            assert info["wave_tasks"] == maps.n_ssr * info["waves_per_block"]
        check_fp64(A, x, y, exact_rows=short_rows(A))


@pytest.mark.parametrize("waves_case", [(20, 10), (7, 8), (64, 4), (400, 2)])
def test_csr3_ssr_plan_with_x_dictionaries(waves_case):
    """The workgroup-per-super-super-row plan (the reference's cuSpMV_3
    mapping) stages a block x dictionary per super-super-row when its W
    waves are 4 or 8 -- one workgroup, one SSR, one dictionary -- and its y
    is bit for bit the aligned plan's (row sums are row-local)."""
    ssrs, srs = waves_case
    A = gen.stencil27(40)
    maps = hspmv.build_csr3_maps(A, ssrs, srs)
    x = gen.rand_x(A.n, 9)
    y0, i0 = gpu_spmv(A, x, maps, options={"csr3_plan": "aligned", "x_dict": -1})
    y1, i1 = gpu_spmv(A, x, maps, options={"csr3_plan": "ssr", "x_dict": 1})
    assert i1["csr3_plan"] == 3 and i1["wave_tasks"] == maps.n_ssr * i1["waves_per_block"]
    assert i1["blocks"] == maps.n_ssr
    # the host planner's view (hspmv_xdict_plan_ex): W of 4 or 8 and every
    # SSR's dictionary within the LDS cap
    planned = hspmv.xdict_plan(A, maps, kernel="csr3", options={"csr3_plan": "ssr", "x_dict": 1})
    assert i1["x_dict"] == (1 if planned is not None else 0), i1
    if planned is not None:
        assert planned[0].size - 1 == maps.n_ssr and i1["waves_per_block"] in (4, 8)
    assert np.array_equal(y0, y1)
    check_fp64(A, x, y1, exact_rows=short_rows(A))


@pytest.mark.parametrize("xwin", ["0", "1"])
def test_x_window_variants_identical(xwin):
    """Global gathers and LDS x windows give the same bits (the windows only
    change where x[col] is read from), for STREAM and for packed CSR-3
    tasks; groups whose columns do not fit a window mix in."""
    opts = {"x_windows": -1} if xwin == "0" else None
    rng = np.random.default_rng(4)
    A0 = gen.banded(40000, per_row=10, half=32, seed=6)
    # every 7th group gets a far column, so some groups do not fit
    ci = A0.col_idx.copy()
    far = np.arange(0, A0.m, 64 * 7)
    ci[A0.row_ptr[far]] = rng.integers(0, A0.n, far.size)
    A = hspmv.CsrMatrix(A0.m, A0.n, A0.row_ptr, ci, A0.val)
    x = gen.rand_x(A.n, 12)
    maps = hspmv.build_csr3_maps(A, 7, 8)
    for mp in (None, maps):
        y, info = gpu_spmv(A, x, mp, options=opts)
        assert info["x_windows"] == int(xwin)
        check_fp64(A, x, y, exact_rows=slice(None))


def test_nontemporal_variants_identical():
    A = gen.stencil27(20)
    x = gen.rand_x(A.n, 8)
    for kernel in ("stream", "vector"):
        y0, _ = gpu_spmv(A, x, kernel=kernel)
        y1, _ = gpu_spmv(A, x, kernel=kernel, nontemporal=True)
        assert np.array_equal(y0, y1)
    maps = hspmv.build_csr3_maps(A, 20, 10)
    y0, _ = gpu_spmv(A, x, maps)
    y1, _ = gpu_spmv(A, x, maps, nontemporal=True)
    assert np.array_equal(y0, y1)


def test_edge_cases():
    # empty matrix rows, all-empty matrix, single row, single column, zero nnz
    cases = []
    cases.append(hspmv.CsrMatrix(5, 7, np.zeros(6, np.int32), np.zeros(0, np.int32),
                                 np.zeros(0, np.float64)))
    cases.append(hspmv.CsrMatrix(1, 1, np.array([0, 1]), np.array([0]), np.array([2.5])))
    cases.append(hspmv.CsrMatrix(3, 1, np.array([0, 1, 1, 2]), np.array([0, 0]),
                                 np.array([1.0, -3.0])))
    rng = np.random.default_rng(1)
    for m in (63, 64, 65, 127, 129, 1000):  # around the 64-row wave tasks
        lens = rng.integers(0, 80, m)
        rp = np.concatenate([[0], np.cumsum(lens)])
        ci = rng.integers(0, 500, rp[-1])
        cases.append(hspmv.CsrMatrix(m, 500, rp, ci, rng.uniform(-1, 1, rp[-1])))
    for A in cases:
        x = gen.rand_x(A.n, 1)
        for kernel, lanes in KERNELS:
            y, _ = gpu_spmv(A, x, kernel=kernel, lanes=lanes)
            check_fp64(A, x, y)
        if A.m > 1:
            maps = hspmv.build_csr3_maps(A, 3, 2)
            y, _ = gpu_spmv(A, x, maps)
            check_fp64(A, x, y, exact_rows=short_rows(A))


def test_repeated_spmv_and_rebinding():
    A = gen.banded(100000, seed=3)
    x1, x2 = gen.rand_x(A.n, 1), gen.rand_x(A.n, 2)
    with hspmv.SpMV(A) as op:
        y1 = op(x1)
        y2 = op(x2)
        for _ in range(10):
            op.spmv()
        op.synchronize()
        assert np.array_equal(op.get_y(), y2)
        t = op.run(warmup=2, iters=5)
        assert t["iters"] == 5 and t["t_min"] > 0 and t["gflops"] > 0
    check_fp64(A, x1, y1)
    # linearity: A(2 x1 - x2) = 2 A x1 - A x2 (fp64 rounding only)
    with hspmv.SpMV(A) as op:
        y3 = op(2 * x1 - x2)
    np.testing.assert_allclose(y3, 2 * y1 - y2, atol=1e-12 * np.abs(A.val).max() * 20)


def test_errors_are_reported_not_crashes():
    A = gen.laplace2d(10, 10)
    with hspmv.SpMV(A) as op:
        with pytest.raises(hspmv.HspmvError, match="E_STATE"):
            op.spmv()  # x not set
        with pytest.raises(ValueError):
            op.set_x(np.zeros(3))
    bad = hspmv.CsrMatrix(2, 2, np.array([0, 1, 2]), np.array([0, 9]), np.array([1.0, 1.0]))
    with pytest.raises(hspmv.HspmvError, match="E_INVALID"):
        hspmv.SpMV(bad)
    with pytest.raises(hspmv.HspmvError, match="E_NODEV"):
        hspmv.SpMV(A, device=999)
    with pytest.raises(hspmv.HspmvError):
        hspmv.SpMV(A, num_gpus=hspmv.device_count() + 1)


# ---------------------------------------------------------------- full size

def test_config_c2_laplacian_1m_fp64():
    """BASELINE configs[1]: CSR fp64 on the 1000x1000 Laplacian, x = 1 and rand."""
    A = gen.laplace2d(1000, 1000)
    assert A.nnz == 4_996_000
    for x in (np.ones(A.n), gen.rand_x(A.n, 42)):
        for kernel in ("auto", "vector"):
            y, info = gpu_spmv(A, x, kernel=kernel)
            check_fp64(A, x, y, exact_rows=slice(None) if kernel == "auto" else None)
            if kernel == "auto":  # Infinity-Cache resident: gathers, no x windows
                assert info["x_windows"] == 0


def test_config_c3_stencil27_csr3_fp64():
    """BASELINE configs[2] stand-in: 27-pt 125^3 RCM, CSR-3 with ssrs=20, srs=10."""
    A = gen.stencil27(125)
    assert A.nnz == 51_895_117
    ssrs, srs = hspmv.csr3_params(A.nnz / A.m, "volta")
    assert (ssrs, srs) == (20, 10)
    maps = hspmv.build_csr3_maps(A, ssrs, srs)
    x = gen.rand_x(A.n, 7)
    y, info = gpu_spmv(A, x, maps)
    check_fp64(A, x, y, exact_rows=slice(None))


def test_config_c3_alt_honeycomb_fp64():
    """BASELINE configs[2]'s SuiteSparse example, hugebubbles-00000
    (helpers/overhead.txt:33-34), has no copy here: its stand-in is an
    RCM-ordered degree-3 honeycomb mesh of the same size (18.3 M rows,
    54.9 M nnz).  Every row is <= 3 nonzeros, so y is bit-identical to the
    oracle, through STREAM and through CSR-3 with the .csr3 writer's
    grouping."""
    A = gen.honeycomb(4280, 4280)
    assert A.m == 18_318_400 and A.nnz == 54_942_360
    x = gen.rand_x(A.n, 13)
    y, info = gpu_spmv(A, x)
    y64 = check_fp64(A, x, y, exact_rows=slice(None))
    maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "volta"))
    y3, i3 = gpu_spmv(A, x, maps)
    assert i3["kernel_name"] == "csr3"
    assert np.array_equal(y3, y64)


def test_config_c4_banded_shard_fp64():
    """BASELINE configs[3]: one rank's row-range shard of the 2e7-row banded
    matrix (P = 8 -> 2.5 M rows), global columns, full-length x."""
    m = 20_000_000
    splits = np.linspace(0, m, 9).astype(np.int64)
    A = gen.banded(m, r0=int(splits[3]), r1=int(splits[4]))
    x = gen.rand_x(m, 11)
    y, info = gpu_spmv(A, x)
    check_fp64(A, x, y, exact_rows=slice(None))
    # the gathers are staged in LDS: one x window of <= 256 columns per
    # group, or (the default for HBM-resident matrices) a block x dictionary
    assert info["x_windows"] == 1 or info["x_dict"] == 1


def test_config_c4_full_matrix_one_gpu():
    """BASELINE configs[3] whole: the 2e7-row, 2e8-nonzero banded matrix on
    ONE GPU (the N = 1 point of the strong-scaling curve, bench.py
    scaling_reference).  Every row has <= 10 nonzeros (<= 40: the ordered
    sums), so y must equal the oracle's omp_spmv restatement bit for bit."""
    from hspmv import dist as hdist
    sh = hdist.build_shard("c4", 0, 1)
    A = sh.A
    assert A.m == 20_000_000 and 199_999_000 < A.nnz <= 200_000_000
    assert int(np.diff(A.row_ptr).max()) <= SERIAL_MAX
    x = gen.rand_x(A.n, 11)
    y, info = gpu_spmv(A, x)
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    assert info["kernel_name"] in ("stream", "csr3") and info["deterministic"] == 1
    assert np.array_equal(y.view(np.uint64), y64.view(np.uint64))
    ok, rel = hdist.checksum_ok(A, x, y)
    assert ok, rel


def test_config_c5_powerlaw_csr3_fp32():
    """BASELINE configs[4]: power-law fp32 with CSR-3 maps.  Its random
    columns make the gathers irregular, so AUTO runs the column-sorted row
    blocks (csort: fp64 row sums, stored per column part as fp32 partials and
    added in fp64): y is checked against the exact (fp64) sums to an fp32
    rounding of y and of each part's sum (sum_h |p_h| <= sum|a x|), and
    against omp_spmv's fp32 sums within their summation error (the parity
    bar).  The x-slab path (options x_slabs) stays
    available and bitwise on short rows -- AUTO streams its passes with
    STREAM (C5's 64-row groups are balanced: slab_kernel_rule), the CSR3
    tasks when forced -- and deterministic=1 keeps the row kernels."""
    A = gen.powerlaw(2_000_000, seed=1234, dtype=np.float32)
    maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "mi355x"))
    x = gen.rand_x(A.n, 9).astype(np.float32)
    y, info = gpu_spmv(A, x, maps)
    lens = np.diff(A.row_ptr)
    assert info["kernel_name"] == "csort" and info["csort_parts"] == 2
    assert info["n_split_rows"] == int((lens > 4096).sum())
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val.astype(np.float64), x.astype(np.float64))
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    y32 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    # every SpMV of a back-to-back run (the LDS atomic order varies from
    # launch to launch)
    with hspmv.SpMV(A, maps, device=0) as op:
        op.set_x(x)
        for it in range(12):
            op.spmv()
            yi = op.get_y() if it else y
            assert np.all(np.abs(yi - y64) <= 2.0 ** -24 * (np.abs(y64) + absrow) + 1e-12 * absrow), it
            err = np.abs(yi.astype(np.float64) - y32.astype(np.float64))
            assert np.all(err <= (lens + 2) * 2.0 ** -23 * absrow + 1e-30), it
    ok = short_rows(A)
    ys, info = gpu_spmv(A, x, maps, options={"x_slabs": 4})
    assert info["kernel_name"] == "stream" and info["x_slabs"] == 4 and info["slab_kernel_rule"] == 2
    assert np.array_equal(ys[ok].view(np.uint32), y32[ok].view(np.uint32))
    ys, info = gpu_spmv(A, x, maps, kernel="csr3", options={"x_slabs": 4})
    assert info["kernel_name"] == "csr3" and info["x_slabs"] == 4
    assert np.array_equal(ys[ok].view(np.uint32), y32[ok].view(np.uint32))


@pytest.mark.parametrize("rcm", [False, True])
def test_config_c5_reproducible_fixed_point(rcm):
    """BASELINE configs[4] (and its RCM ordering) with hspmv_options
    deterministic = 2: the column-sorted kernel with fixed-point (int64) row
    sums.  Twelve back-to-back SpMVs give the same y bits; y stays within
    omp_spmv's own fp32 summation error (the parity bar above) and within the
    fixed-point bound of the exact sum (len 2^-49 max_r|v| max|x| + the
    partials' and y's fp32 roundings)."""
    A = gen.powerlaw(2_000_000, seed=1234, dtype=np.float32, rcm=rcm)
    maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "mi355x"))
    x = gen.rand_x(A.n, 9).astype(np.float32)
    lens = np.diff(A.row_ptr)
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val.astype(np.float64), x.astype(np.float64))
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    y32 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    vmax = np.zeros(A.m)
    nz = lens > 0
    vmax[nz] = np.maximum.reduceat(np.abs(A.val.astype(np.float64)), A.row_ptr[:-1][nz])
    fixed = lens * 2.0 ** -48 * vmax * float(np.abs(x).max())
    with hspmv.SpMV(A, maps, device=0, options={"deterministic": "reproducible"}) as op:
        info = op.info
        assert info["kernel_name"] == "csort" and info["csort_fixed_point"] == 1
        assert info["deterministic"] == 1
        op.set_x(x)
        ys = []
        for _ in range(12):
            op.spmv()
            ys.append(op.get_y())
    for y in ys[1:]:
        assert np.array_equal(y.view(np.uint32), ys[0].view(np.uint32))
    y = ys[0]
    err = np.abs(y.astype(np.float64) - y32.astype(np.float64))
    assert np.all(err <= (lens + 2) * 2.0 ** -23 * absrow + 1e-30)
    assert np.all(np.abs(y - y64) <= 2.0 ** -24 * (np.abs(y64) + absrow) + fixed + 2.0 ** -148)
    # and bit for bit the CPU restatement at the handle's own column parts
    # (tests/fixedpoint_model.py) on every row the kernel does not slice
    from fixedpoint_model import reproducible_csort_y
    ym = reproducible_csort_y(A.row_ptr, A.col_idx, A.val, x, info["csort_part_begin"])
    short = lens <= 4096
    bad = np.flatnonzero(y[short].view(np.uint32) != ym[short].view(np.uint32))
    assert bad.size == 0, (info["csort_part_begin"], int(np.flatnonzero(short)[bad[0]]))


def test_config_c5r_powerlaw_rcm_csr3_fp32():
    """C5's matrix in the reference's input ordering: RCM-permuted
    (helpers/converter.m:8,14, symrcm -> .mtx.rcm.csr).  RCM leaves a
    random graph's columns scattered, so AUTO still takes the column-sorted
    kernel (per-part row partitions keep its column parts balanced; hub
    rows' contiguous columns go to segmented chunks); checked like C5."""
    A = gen.powerlaw(2_000_000, seed=1234, dtype=np.float32, rcm=True)
    maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "mi355x"))
    x = gen.rand_x(A.n, 9).astype(np.float32)
    y, info = gpu_spmv(A, x, maps)
    lens = np.diff(A.row_ptr)
    assert info["kernel_name"] == "csort"
    assert info["n_split_rows"] == int((lens > 4096).sum())
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val.astype(np.float64), x.astype(np.float64))
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    assert np.all(np.abs(y - y64) <= 2.0 ** -24 * (np.abs(y64) + absrow) + 1e-12 * absrow)
    y32 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    err = np.abs(y.astype(np.float64) - y32.astype(np.float64))
    assert np.all(err <= (lens + 2) * 2.0 ** -23 * absrow + 1e-30)
    # deterministic row kernels on the same matrix: bitwise on short rows
    yd, idet = gpu_spmv(A, x, maps, options={"deterministic": 1})
    assert idet["kernel_name"] == "csr3"
    ok = short_rows(A)
    assert np.array_equal(yd[ok].view(np.uint32), y32[ok].view(np.uint32))


def _split_row_matrix(seed=3):
    """Rows of 5e3 .. 1.2e5 nonzeros (split rows) beside short and medium rows,
    including split rows first, last, adjacent, and at 64-row group edges."""
    rng = np.random.default_rng(seed)
    m, n = 700, 150_000
    lens = rng.integers(0, 40, m)
    lens[rng.integers(0, m, 40)] = rng.integers(33, 4000, 40)     # medium rows
    for r, ln in [(0, 120_000), (1, 4097), (63, 5000), (64, 9000), (65, 4096), (300, 30_000),
                  (301, 70_000), (699, 8193)]:
        lens[r] = ln
    rp = np.concatenate([[0], np.cumsum(lens)])
    ci = np.concatenate([np.sort(rng.choice(n, ln, replace=False)) for ln in lens])
    return hspmv.CsrMatrix(m, n, rp, ci, rng.uniform(-1, 1, rp[-1]))


def test_split_rows_all_kernels():
    A = _split_row_matrix()
    x = gen.rand_x(A.n, 4)
    lens = np.diff(A.row_ptr)
    maps = hspmv.build_csr3_maps(A, 20, 4)
    for kw, mp in [(dict(kernel="stream"), None), (dict(kernel="auto"), maps),
                   (dict(kernel="stream", split_rows=False), None),
                   (dict(kernel="csr3", split_rows=False), maps),
                   (dict(kernel="stream", xcd_remap=False), None),
                   (dict(kernel="vector", lanes=64), None)]:
        y, info = gpu_spmv(A, x, mp, **kw)
        split = kw.get("split_rows", True) and kw["kernel"] != "vector"
        assert info["n_split_rows"] == (int((lens > 4096).sum()) if split else 0), kw
        check_fp64(A, x, y, exact_rows=short_rows(A) if kw["kernel"] != "vector" else None)


def test_chunk_u_and_remap_variants():
    for A in (gen.stencil27(24), gen.powerlaw(40000, seed=21, dtype=np.float64)):
        x = gen.rand_x(A.n, 6)
        ys = []
        maps = hspmv.build_csr3_maps(A, 20, 10)
        for u in (2, 3, 4, 5, 6, 8, 16):
            for remap, pf in ((True, False), (False, True), (True, True)):
                y, info = gpu_spmv(A, x, kernel="stream", chunk_u=u, xcd_remap=remap, prefetch=pf)
                assert info["chunk_u"] == u and (info["xcd_remap"] > 1) == remap
                ys.append(y)
                y3, _ = gpu_spmv(A, x, maps, chunk_u=u, xcd_remap=remap, prefetch=pf)
                ys.append(y3)
        for g in (2, 4, 16):  # several 64-row groups per wave, rp prefetched
            for pf in (False, True):
                y, info = gpu_spmv(A, x, kernel="stream", groups_per_wave=g, prefetch=pf)
                assert info["groups_per_wave"] == g
                ys.append(y)
        for xc in (2, 4, 16):  # chunked XCD orders (tail blocks keep their index)
            y, info = gpu_spmv(A, x, kernel="stream", xcd_chunk=xc)
            assert info["xcd_remap"] == xc
            ys.append(y)
            y3, _ = gpu_spmv(A, x, maps, xcd_chunk=xc)
            ys.append(y3)
        ok = short_rows(A)
        y64 = check_fp64(A, x, ys[0], exact_rows=ok)
        absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
        for y in ys[1:]:
            assert np.array_equal(y[ok], ys[0][ok])
            assert fp64_tol_ok(y, y64, absrow)


def test_borrowed_device_arrays():
    """HSPMV_FLAG_DEVICE_PTRS: the handle reads caller-owned device arrays
    (torch tensors here) and caller-bound x / y; the host tables (x slabs
    included: the values are read back for the slab-major copy) are built
    from device reads."""
    import torch
    A = gen.stencil27(30)
    maps = hspmv.build_csr3_maps(A, 20, 10)
    x = gen.rand_x(A.n, 13)
    rp, ci, val = (torch.from_numpy(a).cuda() for a in (A.row_ptr, A.col_idx, A.val))
    xd = torch.from_numpy(x).cuda()
    yd = torch.zeros(A.m, dtype=torch.float64, device="cuda")
    o, i = torch.from_numpy(maps.outer).cuda(), torch.from_numpy(maps.inner).cuda()
    cs = hspmv._lib.Csr(A.m, A.n, A.nnz, rp.data_ptr(), ci.data_ptr(), val.data_ptr(), 1)
    ms = hspmv._lib.Csr3Maps(maps.n_ssr, maps.n_sr, o.data_ptr(), i.data_ptr())
    for mdev, kernel in ((None, "stream"), (ms, "csr3"), (None, "vector")):
        op = hspmv.SpMV.from_device(cs, mdev, A, device=0, kernel=kernel)
        op.bind_x_device(xd.data_ptr())
        op.bind_y_device(yd.data_ptr())
        op.spmv()
        op.synchronize()
        check_fp64(A, x, yd.cpu().numpy(), exact_rows=short_rows(A) if kernel != "vector" else None)
        op.close()
    for mdev, kernel in ((None, "stream"), (ms, "csr3")):
        yd.zero_()
        op = hspmv.SpMV.from_device(cs, mdev, A, device=0, kernel=kernel, options={"x_slabs": 3})
        assert op.info["x_slabs"] == 3
        op.bind_x_device(xd.data_ptr())
        op.bind_y_device(yd.data_ptr())
        op.spmv()
        op.synchronize()
        check_fp64(A, x, yd.cpu().numpy(), exact_rows=short_rows(A))
        op.close()
    bad = hspmv._lib.Csr(A.m, A.n, A.nnz, rp.data_ptr(), 0, val.data_ptr(), 1)
    with pytest.raises(hspmv.HspmvError, match="E_INVALID"):
        hspmv.SpMV.from_device(bad, None, A, device=0)


def _wide_random(m, n, per_row, seed):
    rng = np.random.default_rng(seed)
    cols = np.sort(rng.choice(n, size=(m, per_row), replace=True), axis=1)
    rp = np.arange(0, m * per_row + 1, per_row, dtype=np.int32)
    val = rng.uniform(-1, 1, m * per_row)
    return hspmv.CsrMatrix(m, n, rp, cols.reshape(-1).astype(np.int32), val)


def _band_random(m, per_row, half, seed):
    """Rows with per_row sorted columns within +-half of the diagonal."""
    rng = np.random.default_rng(seed)
    cols = np.arange(m)[:, None] + rng.integers(-half, half + 1, size=(m, per_row))
    cols = np.sort(np.clip(cols, 0, m - 1), axis=1)
    rp = np.arange(0, m * per_row + 1, per_row, dtype=np.int32)
    return hspmv.CsrMatrix(m, m, rp, cols.reshape(-1).astype(np.int32),
                           rng.uniform(-1, 1, m * per_row))


def test_col16_offsets_bitwise_and_fallback():
    """16-bit column offsets give the same y bit for bit as 32-bit columns,
    through STREAM, CSR3, prefetch and split rows, in both encodings:
    per-256-nonzero block bases + p high-bit planes (forced here with
    options col16_group=-1, p <= 8; p grows with a block's column span and a matrix
    needing more than 8 planes keeps 32-bit columns), and one base per
    64-row STREAM group or packed CSR3 task (col16_group=1) when every
    group spans < 65536.
    By default these small (Infinity-Cache-resident) matrices use the group
    bases where they fit and 32-bit columns otherwise."""
    cases = [(gen.laplace2d(300, 200), 1, True),                  # spans < 65536
             (gen.stencil27(20), 1, True),
             (gen.banded(30000, per_row=10, half=32, seed=5), 1, True),
             (_band_random(150000, 10, 50000, 6), 2, False),          # 1 plane
             (gen.powerlaw(200000, seed=3, dtype=np.float64), 3, False),  # 2 planes
             (_split_row_matrix(), None, False),
             (_wide_random(2000, 1 << 25, 40, 4), 0, False)]            # 10 planes: off
    for A, want, group_fits in cases:
        x = gen.rand_x(A.n, 9)
        maps = hspmv.build_csr3_maps(A, 20, 10)
        for kw, mp in [(dict(kernel="stream"), None), (dict(kernel="stream", prefetch=True), None),
                       (dict(kernel="csr3"), maps), (dict(kernel="stream", chunk_u=2), None)]:
            y16, i16 = gpu_spmv(A, x, mp, col16=True, options={"col16_group": -1}, **kw)
            y16g, i16g = gpu_spmv(A, x, mp, col16=True, options={"col16_group": 1}, **kw)
            y32, i32 = gpu_spmv(A, x, mp, col16=False, **kw)
            assert i32["col16"] == 0 and i32["format_bytes"] == i32["alg_bytes"]
            assert i16["col16_group"] == 0
            if want is not None:
                assert i16["col16"] == want, (kw, i16["col16"], want)
            if i16["col16"]:
                assert i16["format_bytes"] < i16["alg_bytes"]
            g = group_fits  # STREAM's 64-row groups or CSR3's packed tasks
            assert i16g["col16_group"] == int(g), (kw, i16g["col16_group"])
            if g:
                assert i16g["col16"] == 1 and i16g["format_bytes"] < i16g["alg_bytes"]
            assert np.array_equal(y16, y32), kw
            assert np.array_equal(y16g, y32), kw
        check_fp64(A, x, y16, exact_rows=short_rows(A))
        _, idef = gpu_spmv(A, x)
        assert idef["col16_group"] == int(group_fits)
        assert idef["col16"] == int(group_fits)  # small: block offsets only when forced
    # the vector kernel always reads 32-bit columns
    A = gen.laplace2d(100, 100)
    _, iv = gpu_spmv(A, gen.rand_x(A.n, 1), kernel="vector", col16=True)
    assert iv["col16"] == 0


def _few_random(m, n, per_row, seed, dtype=np.float64):
    """per_row random (sorted) columns per row: hundreds of column runs per
    256-row block, so the dictionary builder must bridge gaps."""
    rng = np.random.default_rng(seed)
    cols = np.sort(rng.choice(n, size=(m, per_row), replace=True), axis=1)
    rp = np.arange(0, m * per_row + 1, per_row, dtype=np.int32)
    return hspmv.CsrMatrix(m, n, rp, cols.reshape(-1).astype(np.int32),
                           rng.uniform(-1, 1, m * per_row).astype(dtype))


def test_xdict_bitwise_and_fallback():
    """Block x dictionaries (options x_dict=1 forces them on these small
    matrices): each workgroup stages the x runs its rows reference in LDS
    and gathers from there through 16-bit positions.  y is bit-identical to
    the 32-bit-column path through STREAM, CSR3 (packed tasks), prefetch,
    nontemporal loads, U = 2 and split rows, in fp64 and fp32; a matrix whose
    blocks exceed the LDS cap falls back (x_dict = 0) with the same y."""
    big = 64 * 1024  # LDS bytes per block (default cap: 20 KiB)
    cases = [(gen.laplace2d(300, 200), True, None),
             (gen.stencil27(20), True, None),
             (gen.banded(30000, per_row=10, half=32, seed=5), True, None),
             (_split_row_matrix(), None, big),
             (gen.laplace2d(1, 1), True, None),
             (gen.powerlaw(200000, seed=3, dtype=np.float64), False, None),   # > cap: off
             (_few_random(3000, 8000, 2, 4), None, big)]                    # gap bridging
    for A, want, cap in cases:
        for dt in (np.float64, np.float32):
            Ad = A.astype(dt)
            x = gen.rand_x(A.n, 9).astype(dt)
            maps = hspmv.build_csr3_maps(Ad, 20, 10)
            for kw, mp in [(dict(kernel="stream"), None), (dict(kernel="stream", prefetch=True), None),
                           (dict(kernel="csr3"), maps), (dict(kernel="stream", chunk_u=2), None),
                           (dict(kernel="csr3", nontemporal=True), maps),
                           (dict(kernel="csr3", prefetch=True), maps)]:
                yd, idd = gpu_spmv(Ad, x, mp, options={"x_dict": 1, "x_dict_cap": cap or 0}, **kw)
                y0, i0 = gpu_spmv(Ad, x, mp, col16=False, options={"x_dict": -1}, **kw)
                assert i0["x_dict"] == 0 and i0["x_dict_entries"] == 0
                if want is not None and not (want is False and dt == np.float32):
                    assert idd["x_dict"] == int(want), (kw, dt, idd["x_dict"])
                if idd["x_dict"]:
                    assert idd["x_dict_entries"] > 0 and idd["col16"] == 1
                assert np.array_equal(yd.view(np.uint8), y0.view(np.uint8)), (kw, dt)
            if dt == np.float64:
                check_fp64(Ad, x, yd, exact_rows=short_rows(Ad))
    # default on these small (Infinity-Cache-resident) matrices: no dictionary
    A = gen.stencil27(20)
    _, idef = gpu_spmv(A, gen.rand_x(A.n, 1))
    assert idef["x_dict"] == 0


def _slab_exact_rows(A, slabs):
    """Rows whose every x-slab segment has <= SERIAL_MAX nonzeros: the slab
    passes sum them left to right from 0, i.e. bit-identical to omp_spmv."""
    w = -(-A.n // slabs)
    rows = np.repeat(np.arange(A.m), np.diff(A.row_ptr))
    seg = np.zeros((A.m, slabs), np.int64)
    np.add.at(seg, (rows, A.col_idx.astype(np.int64) // w), 1)
    lens = np.diff(A.row_ptr)
    return (seg.max(axis=1, initial=0) <= SERIAL_MAX) & (lens <= 4096)


def test_xslabs_bitwise_rows_and_fallback():
    """x slabs (options x_slabs=B forces B column slabs): the row kernel runs
    once per slab over a slab-major copy, each pass continuing the rows
    from y.  Rows whose slab segments are all <= 40 nonzeros are
    bit-identical to the oracle (fp64 restatement, fp32 reference loop),
    the rest within the fp64 bar; split rows, empty rows, CSR3 tasks,
    prefetch and U = 2 included.  Unsorted rows fall back (x_slabs = 0)."""
    cases = [_wide_random(3000, 1 << 20, 40, 4), gen.powerlaw(100000, seed=3, dtype=np.float64),
             _split_row_matrix(), gen.laplace2d(1, 1), gen.laplace2d(300, 200)]
    for A in cases:
        for slabs in (2, 5):
            exact = _slab_exact_rows(A, min(slabs, A.n))
            for dt in (np.float64, np.float32):
                Ad = A.astype(dt)
                x = gen.rand_x(A.n, 9).astype(dt)
                maps = hspmv.build_csr3_maps(Ad, 20, 10)
                ref = oracle.spmv(Ad.row_ptr, Ad.col_idx, Ad.val, x)
                for kw, mp in [(dict(kernel="stream"), None), (dict(kernel="csr3"), maps),
                               (dict(kernel="stream", prefetch=True), None),
                               (dict(kernel="stream", chunk_u=2, nontemporal=True), None)]:
                    ys, info = gpu_spmv(Ad, x, mp, options={"x_slabs": slabs}, **kw)
                    want = min(slabs, A.n) if min(slabs, A.n) >= 2 else 0
                    assert info["x_slabs"] == want, (kw, info["x_slabs"])
                    assert np.array_equal(ys[exact].view(np.uint8), ref[exact].view(np.uint8)), kw
                    if dt == np.float64:
                        check_fp64(Ad, x, ys)
                    else:
                        absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x.astype(np.float64))
                        nrow = np.diff(A.row_ptr)
                        err = np.abs(ys.astype(np.float64) - ref.astype(np.float64))
                        assert np.all(err <= (nrow + 2) * 2.0 ** -23 * absrow + 1e-30), kw
    # a row whose columns go back to an earlier slab: the slab passes would
    # reorder its sum -> off (unsorted columns inside one slab are fine)
    A = gen.laplace2d(50, 50)
    ci = A.col_idx.copy()
    ci[A.row_ptr[10]] = 2400  # row 10: [2400, 10, 11, 60] -> slabs 2, 0, 0, 0
    Au = hspmv.CsrMatrix(A.m, A.n, A.row_ptr, ci, A.val)
    x = gen.rand_x(A.n, 2)
    yu, iu = gpu_spmv(Au, x, options={"x_slabs": 3})
    assert iu["x_slabs"] == 0
    check_fp64(Au, x, yu, exact_rows=short_rows(Au))
    # the vector kernel never uses slabs; default on small matrices: none
    _, iv = gpu_spmv(A, x, kernel="vector", options={"x_slabs": 3})
    assert iv["x_slabs"] == 0
    _, idef = gpu_spmv(gen.powerlaw(100000, seed=3, dtype=np.float64), gen.rand_x(100000, 1))
    assert idef["x_slabs"] == 0


@pytest.mark.parametrize("cfg", ["c2", "c3", "c3h", "c4", "c5"])
def test_full_size_fp32_bitwise_vs_reference_omp_spmv(cfg):
    """BASELINE's configs at full size in fp32 -- the reference's only dtype --
    against the reference's OWN omp_spmv (spmv-csr/spmv.c, built unmodified
    into oracle/_ref): C2-C4 have no row over 32 nonzeros, so the GPU's y must
    be bit-identical everywhere (C3 through its CSR-3 maps); C5 (power-law,
    irregular gathers: the column-sorted kernel, fp64 row sums) within the
    reference's fp32 summation error, and with deterministic = 1 bitwise on
    every row of <= SERIAL_MAX nonzeros."""
    if not oracle.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference where build() ran)")
    from hspmv import dist as hdist
    if cfg == "c2":
        A, maps = gen.laplace2d(1000, 1000), None
    elif cfg == "c3":
        A = gen.stencil27(125)
        maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "volta"))
    elif cfg == "c3h":
        A, maps = gen.honeycomb(4280, 4280), None
    elif cfg == "c4":
        A, maps = hdist.build_shard("c4", 3, 8).A, None
    else:
        A = gen.powerlaw(2_000_000, seed=1234, dtype=np.float32)
        maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "mi355x"))
    A = A.astype(np.float32)
    x = gen.rand_x(A.n, 21).astype(np.float32)
    y_ref = oracle.ref_spmv(A.row_ptr, A.col_idx, A.val, x)
    y, info = gpu_spmv(A, x, maps)
    if cfg != "c5":
        assert info["kernel_name"] == ("csr3" if maps is not None else "stream")
        assert np.diff(A.row_ptr).max() <= SERIAL_MAX
        assert np.array_equal(y.view(np.uint32), y_ref.view(np.uint32))
        return
    # C5: the column-sorted kernel's fp64 sums (not omp_spmv's fp32 running
    # sums): within the reference's own fp32 summation error of its y
    assert info["kernel_name"] == "csort"
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x.astype(np.float64))
    err = np.abs(y.astype(np.float64) - y_ref.astype(np.float64))
    assert np.all(err <= (np.diff(A.row_ptr) + 2) * 2.0 ** -23 * absrow + 1e-30)
    # deterministic = 1 (the ordered row kernels): omp_spmv's own fp32 sum,
    # bit for bit, on every row the kernels add serially (<= SERIAL_MAX)
    yd, idet = gpu_spmv(A, x, maps, options={"deterministic": 1})
    assert idet["kernel_name"] != "csort" and idet["deterministic"] == 1
    short = np.diff(A.row_ptr) <= SERIAL_MAX
    assert np.array_equal(yd[short].view(np.uint32), y_ref[short].view(np.uint32))
    err = np.abs(yd.astype(np.float64) - y_ref.astype(np.float64))
    assert np.all(err <= (np.diff(A.row_ptr) + 2) * 2.0 ** -23 * absrow + 1e-30)


def test_stream_workgroup_sizes_identical():
    """STREAM with 1, 2 and 4 waves per workgroup (options stream_waves; the
    planner picks 1 for cache-resident matrices, 2 for HBM-resident ones,
    4 with x dictionaries): bit-identical y, including x windows, several
    groups per wave, split rows and a row count that is not a multiple of
    64."""
    rng = np.random.default_rng(4)
    lens = rng.integers(0, 40, 3001)
    lens[:70] = 0
    lens[-90:] = 0
    rp = np.concatenate([[0], np.cumsum(lens)])
    ragged = hspmv.CsrMatrix(3001, 5000, rp, np.concatenate(
        [np.sort(rng.choice(5000, n, replace=False)) for n in lens]).astype(np.int32),
        rng.uniform(-1, 1, rp[-1]))
    cases = [gen.laplace2d(300, 200), gen.banded(30000, per_row=10, half=32, seed=5),
             _split_row_matrix(), ragged]
    for A in cases:
        x = gen.rand_x(A.n, 3)
        for kw in (dict(kernel="stream"), dict(kernel="stream", groups_per_wave=2),
                   dict(kernel="stream", col16=True)):
            ys = []
            for w in ("1", "2", "4"):
                y, info = gpu_spmv(A, x, options={"stream_waves": int(w)}, **kw)
                assert info["waves_per_block"] == int(w), (kw, w, info["waves_per_block"])
                ys.append(y)
            assert all(np.array_equal(ys[0].view(np.uint8), v.view(np.uint8)) for v in ys[1:]), kw
        check_fp64(A, x, ys[0], exact_rows=short_rows(A))
    _, info = gpu_spmv(gen.laplace2d(300, 200), gen.rand_x(60000, 1))
    assert info["waves_per_block"] == 1  # cache-resident: one wave per workgroup
