"""hspmv_options.deterministic = 3 (HSPMV_DETERMINISTIC_SERIAL): every row
summed left to right from 0 by one lane, as omp_spmv does
(spmv-csr/spmv.c:92-114) -- so y equals the reference's BIT FOR BIT on every
row, not only on the rows of <= 40 nonzeros the default ordered sums cover.

Checked on the GPU, through the C ABI:
* the golden fixtures in fp32 against the reference binary's own output
  (tests/golden, made by oracle/_ref), long rows included;
* fp64 against the oracle's omp_spmv restatement (pinned bitwise to the
  reference in tests/test_oracle.py) on matrices with rows of 41 .. 90 000
  nonzeros (those over 4096 added in order by one workgroup each,
  hspmv_long_serial, or with HSPMV_FLAG_NO_SPLIT by their lane in the row
  kernels), through every row kernel and CSR-3 plan, x slabs, x
  dictionaries, 32-bit columns and a two-shard handle;
* BASELINE configs[4] (C5, 2 M rows, power-law) in fp32 at full size against
  the reference's own omp_spmv (oracle/_ref) when it was built;
* the mode's refusals and reports (VECTOR / CSORT refused, hspmv_info
  .serial_order), and spmv-csr --serial ("Bitwise: 0 rows differ").
"""
import subprocess

import numpy as np
import pytest

import hspmv
import oracle
from conftest import GOLDEN, REPO, load_golden
from hspmv import gen
from hspmv._lib import HspmvError

pytestmark = pytest.mark.gpu

SERIAL = {"deterministic": "serial"}


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    assert hspmv.device_count() >= 1, "no HIP device visible: run on the MI355X box"


def run(A, x, maps=None, options=None, **kw):
    opts = dict(SERIAL, **(options or {}))
    with hspmv.SpMV(A, maps, options=opts, **kw) as op:
        return op(x), op.info


def long_rows(seed=3, m=900, n=200_000, dtype=np.float64):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 30, m)
    lens[rng.integers(0, m, 30)] = rng.integers(41, 4000, 30)
    for r, ln in [(0, 90_000), (1, 4097), (63, 5000), (64, 9000), (65, 4096), (400, 30_000), (m - 1, 8193)]:
        lens[r] = ln
    rp = np.concatenate([[0], np.cumsum(lens)])
    ci = np.concatenate([np.sort(rng.choice(n, ln, replace=False)) for ln in lens])
    return hspmv.CsrMatrix(m, n, rp, ci, rng.uniform(-1, 1, rp[-1]).astype(dtype))


def bits_equal(y, ref):
    return np.array_equal(np.ascontiguousarray(y).view(np.uint8), np.ascontiguousarray(ref).view(np.uint8))


def test_serial_golden_fp32_bitwise_vs_reference_binary_every_row(golden_names):
    for name in golden_names:
        A = hspmv.read_csr(GOLDEN / f"{name}.csr", np.float32)
        g = load_golden(name)
        x = gen.rand_x(A.n, 42).astype(np.float32)
        for kernel in ("auto", "stream"):
            y, info = run(A, x, kernel=kernel)
            assert info["serial_order"] == 1 and info["deterministic"] == 1
            assert bits_equal(y, g["y_ref_f32_rand"]), (name, kernel)
            if "y_ref_f32_ones" in g:
                y1, _ = run(A, np.ones(A.n, np.float32), kernel=kernel)
                assert bits_equal(y1, g["y_ref_f32_ones"]), (name, kernel)


def test_serial_golden_csr3_fixtures_every_plan(manifest):
    """The golden .csr3 files (their maps as written) under each CSR3 plan,
    fp64 and fp32: the CSR-3 CPU loop's bits (oracle csr3_spmv, csrk.cpp:
    247-285, equal to omp_spmv row by row) on every row."""
    for name, ent in manifest["fixtures"].items():
        if "csr3" not in ent:
            continue
        for dt in (np.float64, np.float32):
            A, maps = hspmv.read_csr3(GOLDEN / f"{name}.csr3", dt)
            x = gen.rand_x(A.n, 42).astype(dt)
            ref = oracle.csr3_spmv(maps.outer, maps.inner, A.row_ptr, A.col_idx, A.val, x)
            for plan in ("aligned", "packed", "ssr"):
                y, info = run(A, x, maps, {"csr3_plan": plan}, kernel="csr3")
                assert info["kernel_name"] == "csr3" and info["serial_order"] == 1
                assert bits_equal(y, ref), (name, dt, plan)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_serial_long_rows_every_kernel_and_plan(dtype):
    """Rows of 41 .. 90 000 nonzeros (default handles split those over 4096
    and tree-sum those over 40): serial order through STREAM, the CSR3 plans
    over CSR-3 maps, x slabs and 32-bit columns."""
    A = long_rows(dtype=dtype)
    x = gen.rand_x(A.n, 7).astype(dtype)
    ref = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    maps = hspmv.build_csr3_maps(A, 4, 8)
    cases = [(None, "stream", {}), (None, "auto", {}), (None, "stream", {"x_slabs": 3}),
             (maps, "csr3", {"csr3_plan": "aligned"}), (maps, "csr3", {"csr3_plan": "packed"}),
             (maps, "csr3", {"csr3_plan": "ssr"}), (maps, "csr3", {"x_slabs": 2})]
    n_long = int((np.diff(A.row_ptr) > 4096).sum())
    for mp, kernel, opts in cases:
        y, info = run(A, x, mp, opts, kernel=kernel)
        # rows over 4096 nonzeros: one workgroup each (hspmv_long_serial)
        assert info["serial_order"] == 1 and info["n_split_rows"] == n_long, (kernel, opts)
        assert bits_equal(y, ref), (kernel, opts, int(np.flatnonzero(y != ref)[0]))
    y, _ = run(A, x, col16=False)
    assert bits_equal(y, ref)
    # HSPMV_FLAG_NO_SPLIT: the long rows stay in the row kernels' lanes
    for mp, kernel in ((None, "stream"), (maps, "csr3")):
        y, info = run(A, x, mp, kernel=kernel, split_rows=False)
        assert info["serial_order"] == 1 and info["n_split_rows"] == 0
        assert bits_equal(y, ref), kernel


def test_serial_dictionaries_stencil_and_mid_density():
    """The dictionary kernels (C3's shape, small) and 33..100-nonzero rows,
    which the default CSR3 kernel sums four rows at a time in DPP trees."""
    S = gen.stencil27(40, seed=7)
    maps = hspmv.build_csr3_maps(S, *hspmv.csr3_params(S.nnz / S.m, "volta"))
    x = gen.rand_x(S.n, 3)
    for opts in ({}, {"x_dict": 1}, {"csr3_plan": "ssr", "x_dict": 1}):
        y, info = run(S, x, maps, opts)
        assert bits_equal(y, oracle.spmv(S.row_ptr, S.col_idx, S.val, x)), opts
    rng = np.random.default_rng(11)
    m, n = 20_000, 50_000
    lens = rng.integers(33, 101, m)
    rp = np.concatenate([[0], np.cumsum(lens)])
    ci = np.concatenate([np.sort(rng.choice(n, ln, replace=False)) for ln in lens])
    D = hspmv.CsrMatrix(m, n, rp, ci, rng.uniform(-1, 1, rp[-1]))
    xd = gen.rand_x(n, 4)
    ref = oracle.spmv(D.row_ptr, D.col_idx, D.val, xd)
    for kernel in ("auto", "stream", "csr3"):
        y, info = run(D, xd, kernel=kernel)
        assert bits_equal(y, ref), (kernel, info["kernel_name"])
    # the default (ordered) handle differs from omp_spmv on such rows
    with hspmv.SpMV(D, options={"deterministic": "ordered"}) as op:
        yo = op(xd)
        assert op.info["serial_order"] == 0
    assert not bits_equal(yo, ref)


def test_serial_two_shards_and_repeat():
    A = gen.powerlaw(60_000, seed=5, dtype=np.float64)
    x = gen.rand_x(A.n, 9)
    ref = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    y, info = run(A, x, devices=[0, 0])
    assert info["serial_order"] == 1 and info["num_gpus"] == 2
    assert bits_equal(y, ref)
    with hspmv.SpMV(A, options=SERIAL) as op:
        op.set_x(x)
        ys = []
        for _ in range(3):
            op.spmv()
            ys.append(op.get_y())
    assert all(bits_equal(v, ref) for v in ys)


def test_serial_refusals():
    A = gen.powerlaw(5000, seed=1, dtype=np.float64)
    for kernel in ("vector", "csort"):
        with pytest.raises(HspmvError):
            hspmv.SpMV(A, kernel=kernel, options=SERIAL)


@pytest.mark.parametrize("rcm", [False, True])
def test_config_c5_serial_fp32_bitwise_vs_reference_omp_spmv(rcm):
    """BASELINE configs[4] at full size in fp32, and its RCM ordering (the
    reference's input convention): y bit-identical to the reference's own
    omp_spmv (oracle/_ref, spmv-csr/spmv.c built unmodified) on all 2 M
    rows, long hub rows included; and again on a second SpMV (the forked
    long-row stream leaves no state behind)."""
    A = gen.powerlaw(2_000_000, seed=1234, dtype=np.float32, rcm=rcm)
    maps = hspmv.build_csr3_maps(A, *hspmv.csr3_params(A.nnz / A.m, "mi355x"))
    x = gen.rand_x(A.n, 21).astype(np.float32)
    y_ref = oracle.ref_spmv(A.row_ptr, A.col_idx, A.val, x) if oracle.ref_available() else \
        oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    assert np.diff(A.row_ptr).max() > 4096  # the hub rows a default handle splits
    with hspmv.SpMV(A, maps, options=SERIAL) as op:
        info = op.info
        assert info["kernel_name"] in ("stream", "csr3") and info["serial_order"] == 1
        for _ in range(2):
            y = op(x)
            bad = np.flatnonzero(y.view(np.uint32) != y_ref.view(np.uint32))
            assert bad.size == 0, (bad.size, int(bad[0]))


def test_cli_serial_reports_bitwise():
    cli = REPO / "heterogeneous-spmv_amd" / "build" / "spmv-csr"
    out = subprocess.run([str(cli), str(GOLDEN / "long_row.csr"), "3", "--x", "rand:5", "--serial"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "Bitwise: 0 rows differ" in out.stdout and "Check: PASS" in out.stdout
    for dt in ("f32", "f64"):
        out = subprocess.run([str(cli), str(GOLDEN / "powerlaw1500.csr"), "2", "--dtype", dt, "--serial"],
                             capture_output=True, text=True, timeout=120)
        assert out.returncode == 0 and "Bitwise: 0 rows differ" in out.stdout, (dt, out.stdout[-400:])
