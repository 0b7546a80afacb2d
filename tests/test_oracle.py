"""The oracle (CPU restatement) pinned against the reference's own outputs.

The golden y vectors were produced by the reference's spmv-csr/spmv.c compiled
unmodified (tests/golden/make_golden.py); the restatement must reproduce them
bit for bit in fp32.  When the reference build is present (this container),
the restatement is also re-checked against it live on fresh inputs.
"""
import numpy as np
import pytest

import oracle
from conftest import GOLDEN, load_golden
from hspmv import gen


def test_oracle_matches_reference_golden_fp32_bitwise(golden_names):
    for name in golden_names:
        m, n, rp, ci, v32, v64, base = oracle.read_csr(GOLDEN / f"{name}.csr")
        g = load_golden(name)
        x32 = gen.rand_x(n, 42).astype(np.float32)
        y = oracle.spmv(rp, ci, v32, x32)
        assert np.array_equal(y.view(np.uint32), g["y_ref_f32_rand"].view(np.uint32)), name
        if "y_ref_f32_ones" in g:
            y1 = oracle.spmv(rp, ci, v32, np.ones(n, np.float32))
            assert np.array_equal(y1.view(np.uint32), g["y_ref_f32_ones"].view(np.uint32)), name


def test_oracle_fp64_golden_and_serial_equals_parallel(golden_names):
    for name in golden_names:
        m, n, rp, ci, v32, v64, base = oracle.read_csr(GOLDEN / f"{name}.csr")
        x = gen.rand_x(n, 42)
        y = oracle.spmv(rp, ci, v64, x)
        ys = oracle.spmv(rp, ci, v64, x, serial=True)
        assert np.array_equal(y, ys)
        assert np.array_equal(y, load_golden(name)["y_orc_f64_rand"]), name


def test_oracle_fp64_close_to_fp32_reference(golden_names):
    # the fp64 restatement agrees with the fp32 reference at fp32 accuracy
    for name in golden_names:
        m, n, rp, ci, v32, v64, base = oracle.read_csr(GOLDEN / f"{name}.csr")
        x = gen.rand_x(n, 42)
        g = load_golden(name)
        absrow = oracle.abs_rowsum(rp, ci, v64, x)
        nrow = np.diff(rp).astype(np.float64)
        err = np.abs(g["y_ref_f32_rand"].astype(np.float64) - g["y_orc_f64_rand"])
        assert np.all(err <= (nrow + 2) * 2.0 ** -23 * absrow + 1e-6), name


def test_oracle_matches_scipy():
    A = gen.laplace2d(50, 40)
    x = gen.rand_x(A.n, 3)
    y = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    np.testing.assert_allclose(y, A.to_scipy() @ x, rtol=1e-14, atol=1e-14)


def test_one_based_file_reads_identically():
    a = oracle.read_csr(GOLDEN / "lap32.mtx.rcm.csr")
    b = oracle.read_csr(GOLDEN / "lap32.onebased.csr")
    assert b[6] == 1 and a[6] == 0
    for u, v in zip(a[:6], b[:6]):
        assert np.array_equal(u, v)


def test_csr3_fixture_maps_and_spmv(manifest):
    for name, ent in manifest["fixtures"].items():
        if "csr3" not in ent:
            continue
        outer, inner, m, n, rp, ci, v32, v64 = oracle.read_csr3(GOLDEN / f"{name}.csr3")
        maps = np.load(GOLDEN / f"{name}.maps.npz")
        assert np.array_equal(outer, maps["outer"]) and np.array_equal(inner, maps["inner"])
        # A13 invariants: maps monotone and complete
        assert outer[0] == 0 and outer[-1] == len(inner) - 1
        assert inner[0] == 0 and inner[-1] == m
        assert np.all(np.diff(outer) >= 0) and np.all(np.diff(inner) >= 0)
        x = gen.rand_x(n, 42)
        y3 = oracle.csr3_spmv(outer, inner, rp, ci, v64, x)
        assert np.array_equal(y3, load_golden(name)["y_orc_f64_rand"])
        # rebuilding the maps reproduces the fixture
        o2, i2 = oracle.build_maps(rp, ci, ent["csr3"]["ssrs"], ent["csr3"]["srs"])
        assert np.array_equal(o2, outer) and np.array_equal(i2, inner)


def test_hand_coarsen_grouping_rule():
    # every super-row but the last holds >= threshold nnz and drops below it
    # without its last row (csrk.cu:1450-1484)
    A = gen.powerlaw(3000, seed=5, dtype=np.float64)
    ssrs, srs = 7, 8
    outer, inner = oracle.build_maps(A.row_ptr, A.col_idx, ssrs, srs)
    thr = ssrs * A.nnz // A.m
    for s in range(len(inner) - 2):
        a, b = inner[s], inner[s + 1]
        assert A.row_ptr[b] - A.row_ptr[a] >= thr
        assert A.row_ptr[b - 1] - A.row_ptr[a] < thr


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build not present (GPU box)")
def test_oracle_matches_live_reference_fp32(tmp_path):
    for seed, A in enumerate([gen.powerlaw(4000, seed=9, dtype=np.float64),
                              gen.banded(5000, seed=3), gen.laplace2d(40, 60)]):
        p = tmp_path / f"m{seed}.csr"
        gen.write_csr_text(str(p), A)
        m, n, rp, ci, v32, v64, base = oracle.read_csr(p)
        x = gen.rand_x(n, 100 + seed).astype(np.float32)
        y_ref = oracle.ref_spmv_file(p, x)
        y_ser = oracle.ref_spmv_file(p, x, serial=True)
        y = oracle.spmv(rp, ci, v32, x)
        assert np.array_equal(y.view(np.uint32), y_ref.view(np.uint32))
        assert np.array_equal(y_ser.view(np.uint32), y_ref.view(np.uint32))


def test_fixedpoint_model_is_within_its_bound():
    """tests/fixedpoint_model.py (the CPU restatement the reproducible csort
    is checked against bitwise on the GPU): its y stays within the
    fixed-point bound of the exact sum -- len 2^-49 max_r|v| max|x| plus an
    fp32 rounding of y -- and is exactly 0 for x = 0."""
    import numpy as np
    from fixedpoint_model import reproducible_csort_y
    from hspmv import gen
    A = gen.powerlaw(20_000, seed=3, dtype=np.float32)
    x = gen.rand_x(A.n, 5).astype(np.float32)
    y = reproducible_csort_y(A.row_ptr, A.col_idx, A.val, x)
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val.astype(np.float64), x.astype(np.float64))
    lens = np.diff(A.row_ptr)
    vmax = np.zeros(A.m)
    vmax[lens > 0] = np.maximum.reduceat(np.abs(A.val.astype(np.float64)), A.row_ptr[:-1][lens > 0])
    bound = lens * 2.0 ** -49 * vmax * np.abs(x).max() + 2.0 ** -24 * np.abs(y64) + 2.0 ** -148
    ok = lens <= 4096
    assert np.all(np.abs(y[ok].astype(np.float64) - y64[ok]) <= bound[ok])
    assert np.all(reproducible_csort_y(A.row_ptr, A.col_idx, A.val, np.zeros(A.n, np.float32))[ok] == 0)


def test_fixedpoint_model_fp64_is_within_its_bound():
    """The fp64 branch of the model (exact products in Python integers,
    fixedpoint_model.exact_q): within the fixed-point bound plus the fp64
    roundings of the oracle's own sum."""
    import numpy as np
    from fixedpoint_model import reproducible_csort_y
    from hspmv import gen
    A = gen.powerlaw(8_000, seed=4, dtype=np.float64)
    x = gen.rand_x(A.n, 6)
    y = reproducible_csort_y(A.row_ptr, A.col_idx, A.val, x, (0, A.n // 3))
    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    lens = np.diff(A.row_ptr)
    vmax = np.zeros(A.m)
    vmax[lens > 0] = np.maximum.reduceat(np.abs(A.val), A.row_ptr[:-1][lens > 0])
    bound = lens * 2.0 ** -49 * vmax * np.abs(x).max() + (lens + 3) * 2.0 ** -53 * absrow + 1e-300
    ok = lens <= 4096
    assert np.all(np.abs(y[ok] - y64[ok]) <= bound[ok])


def test_fixedpoint_model_exact_q_is_half_even_of_the_exact_product():
    """fixedpoint_model.exact_q (the fp64 branch's product rounding) against
    Python's exact rationals: rint(v x 2^E), ties to even, on values spread
    over 60 binades, zeros, signs, and exact ties."""
    from fractions import Fraction

    import numpy as np
    from fixedpoint_model import FIX_BITS, exact_q, xexp_of
    rng = np.random.default_rng(1)
    v = rng.uniform(-1, 1, 3000) * np.exp2(-rng.integers(0, 60, 3000))
    x = rng.standard_normal(3000) * 3
    v[::7] = 0.0
    E = FIX_BITS - xexp_of(x)
    # exact ties: (5/8 or 7/8) * 4 * 2^-E -> 2.5 / 3.5 units (to 2 and 4)
    v[1::22], v[12::22] = 0.625, -0.875
    x[1::11] = np.ldexp(4.0, -E)
    assert xexp_of(x) == FIX_BITS - E
    q = exact_q(v, x, E)
    assert set(q[1::22].tolist()) == {2} and set(q[12::22].tolist()) == {-4}
    for a, b, qq in zip(v, x, q):
        assert int(qq) == round(Fraction(float(a)) * Fraction(float(b)) * 2 ** E), (a, b)


def test_fixedpoint_model_parts_small_exact():
    """reproducible_csort_y on a tiny matrix against a direct restatement in
    rationals: per column part, the integer sum of the rounded scaled
    products, converted and scaled, rounded to fp32; the parts added in
    order in fp64 and rounded (the kernel's finishing pass)."""
    from fractions import Fraction

    import numpy as np
    from fixedpoint_model import FIX_BITS, reproducible_csort_y, row_scales, xexp_of
    rng = np.random.default_rng(4)
    m, n = 40, 30
    lens = rng.integers(0, 12, m)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ci = np.concatenate([np.sort(rng.choice(n, ln, replace=False)) for ln in lens]).astype(np.int64)
    val = (rng.standard_normal(rp[-1]) * np.exp2(rng.integers(-8, 8, rp[-1]))).astype(np.float32)
    x = rng.standard_normal(n).astype(np.float32)
    pb = (0, 11, 23)
    y = reproducible_csort_y(rp, ci, val, x, pb)
    E = FIX_BITS - xexp_of(x)
    rexp = row_scales(rp, val)
    for r in range(m):
        acc = 0.0
        for h in range(len(pb)):
            lo, hi = pb[h], (pb[h + 1] if h + 1 < len(pb) else n)
            s = 0
            for k in range(rp[r], rp[r + 1]):
                if lo <= ci[k] < hi:
                    vs = Fraction(float(np.float32(np.ldexp(val[k], int(rexp[r])))))
                    s += round(vs * Fraction(float(x[ci[k]])) * 2 ** E)
            p = np.float32(np.ldexp(float(s), int(-E - rexp[r])))
            acc = acc + float(p)
        assert np.float32(acc).tobytes() == y[r].tobytes(), r
