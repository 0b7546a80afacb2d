"""Product host code that needs no GPU: readers, writers, binary cache, CSR-3
map builder, launch heuristics, partitioner -- checked against the oracle."""
import numpy as np
import pytest

import hspmv
import oracle
from conftest import GOLDEN
from hspmv import gen


def test_product_reader_matches_oracle_reader(golden_names):
    for name in golden_names:
        p = GOLDEN / f"{name}.csr"
        m, n, rp, ci, v32, v64, base = oracle.read_csr(p)
        A64 = hspmv.read_csr(p, np.float64)
        A32 = hspmv.read_csr(p, np.float32)
        for A in (A64, A32):
            assert (A.m, A.n, A.nnz, A.index_base) == (m, n, len(ci), 0)
            assert np.array_equal(A.row_ptr, rp) and np.array_equal(A.col_idx, ci)
        # correctly rounded parse: identical to strtod / strtof (fscanf "%f")
        assert np.array_equal(A64.val, v64)
        assert np.array_equal(A32.val.view(np.uint32), v32.view(np.uint32))


def test_one_based_detection():
    a = hspmv.read_csr(GOLDEN / "lap32.mtx.rcm.csr")
    b = hspmv.read_csr(GOLDEN / "lap32.onebased.csr")
    assert b.index_base == 1 and a.index_base == 0
    assert np.array_equal(a.row_ptr, b.row_ptr) and np.array_equal(a.col_idx, b.col_idx)
    assert np.array_equal(a.val, b.val)


def test_csr3_reader_matches_oracle(manifest):
    for name, ent in manifest["fixtures"].items():
        if "csr3" not in ent:
            continue
        p = GOLDEN / f"{name}.csr3"
        outer, inner, m, n, rp, ci, v32, v64 = oracle.read_csr3(p)
        A, maps = hspmv.read_csr3(p, np.float64)
        assert np.array_equal(maps.outer, outer) and np.array_equal(maps.inner, inner)
        assert np.array_equal(A.row_ptr, rp) and np.array_equal(A.col_idx, ci)
        assert np.array_equal(A.val, v64)


def test_map_builder_matches_oracle(manifest):
    cases = [(GOLDEN / f"{n}.csr", e["csr3"]["ssrs"], e["csr3"]["srs"])
             for n, e in manifest["fixtures"].items() if "csr3" in e]
    for p, ssrs, srs in cases:
        A = hspmv.read_csr(p)
        maps = hspmv.build_csr3_maps(A, ssrs, srs)
        o, i = oracle.build_maps(A.row_ptr, A.col_idx, ssrs, srs)
        assert np.array_equal(maps.outer, o) and np.array_equal(maps.inner, i)
    for A, ssrs, srs in [(gen.laplace2d(100, 100), 7, 8), (gen.stencil27(12), 20, 10),
                         (gen.powerlaw(5000, seed=2, dtype=np.float64), 64, 4),
                         (gen.banded(7000, seed=4), 1, 1)]:
        maps = hspmv.build_csr3_maps(A, ssrs, srs)
        o, i = oracle.build_maps(A.row_ptr, A.col_idx, ssrs, srs)
        assert np.array_equal(maps.outer, o) and np.array_equal(maps.inner, i)


def test_lap100_csr3_shape_matches_survey():
    # the reference reformatter on lap100 gives
    # "174 1411 10000 10000 49600" -- that run includes RCM per coarse level;
    # file-order grouping must give the same level-1 count on a natural-order
    # Laplacian (rows are uniform, so RCM does not change the row grouping).
    A = gen.laplace2d(100, 100)
    ssrs, srs = hspmv.csr3_params(A.nnz / A.m, "volta")
    assert (ssrs, srs) == (7, 8)
    maps = hspmv.build_csr3_maps(A, ssrs, srs)
    assert maps.n_sr == 1411


def test_csr3_params_reference_values():
    # d=4.96 -> (7, 8); d=23.2 -> (20, 10)
    assert hspmv.csr3_params(4.96, "volta") == (7, 8)
    assert hspmv.csr3_params(23.2, "volta") == (20, 10)
    # MI100 driver formula (hip/spmv-auto-mi100.cu:130-158) at d = 4.96
    import math
    ssrs = math.floor(0.5 + (8.489 - 1.15 * math.log(4.96)))
    srs = math.floor(0.5 + (10.711 - 1.607 * math.log(4.96)))
    assert hspmv.csr3_params(4.96, "mi100") == (ssrs, srs)


def test_writer_roundtrip(tmp_path):
    A = gen.powerlaw(800, seed=3, dtype=np.float64)
    A.val = np.round(A.val, 6)
    p = tmp_path / "a.csr"
    hspmv.write_csr(p, A)
    B = hspmv.read_csr(p)
    assert np.array_equal(A.row_ptr, B.row_ptr) and np.array_equal(A.col_idx, B.col_idx)
    np.testing.assert_allclose(B.val, A.val, atol=5e-7)
    # oracle can read the product's text too (reference layout)
    m, n, rp, ci, v32, v64, base = oracle.read_csr(p)
    assert np.array_equal(rp, A.row_ptr) and np.array_equal(v64, B.val)
    maps = hspmv.build_csr3_maps(A, 5, 6)
    p3 = tmp_path / "a.csr3"
    hspmv.write_csr3(p3, A, maps)
    C, maps2 = hspmv.read_csr3(p3)
    assert np.array_equal(maps.outer, maps2.outer) and np.array_equal(maps.inner, maps2.inner)
    assert np.array_equal(C.col_idx, A.col_idx)


def test_bin_cache_roundtrip(tmp_path):
    for dt in (np.float32, np.float64):
        A = gen.banded(4000, seed=5, dtype=dt)
        maps = hspmv.build_csr3_maps(A, 20, 10)
        p = tmp_path / f"a{np.dtype(dt).itemsize}.bin"
        hspmv.save_bin(p, A, maps)
        B, m2 = hspmv.load_bin(p)
        assert B.val.dtype == dt
        assert np.array_equal(A.row_ptr, B.row_ptr) and np.array_equal(A.col_idx, B.col_idx)
        assert np.array_equal(A.val, B.val)
        assert np.array_equal(maps.outer, m2.outer) and np.array_equal(maps.inner, m2.inner)
        p2 = tmp_path / "nomaps.bin"
        hspmv.save_bin(p2, A)
        B2, m3 = hspmv.load_bin(p2)
        assert m3 is None and np.array_equal(B2.val, A.val)


@pytest.mark.parametrize("text,err", [
    ("", "E_IO"), ("3 3", "E_IO"), ("2 2 2\n0 1 2\n0 1\n1.0", "E_IO"),
    ("2 2 2\n0 1 3\n0 1\n1.0 2.0", "E_INVALID"),      # row_ptr[m] != nnz
    ("2 2 2\n0 2 1\n0 1\n1.0 2.0", "E_INVALID"),      # decreasing row_ptr
    ("2 2 2\n0 1 2\n0 5\n1.0 2.0", "E_INVALID"),      # column out of range
    ("2 2 2\n2 3 4\n0 1\n1.0 2.0", "E_IO"),           # base neither 0 nor 1
    ("2 2 2\n0 1 2\n0 x\n1.0 2.0", "E_IO"),           # malformed token
])
def test_reader_rejects_malformed(tmp_path, text, err):
    p = tmp_path / "bad.csr"
    p.write_text(text)
    with pytest.raises(hspmv.HspmvError, match=err):
        hspmv.read_csr(p)


def test_missing_file_raises():
    with pytest.raises(hspmv.HspmvError, match="E_IO"):
        hspmv.read_csr("/nonexistent/file.csr")


def test_partition_rows_balanced():
    A = gen.powerlaw(20000, seed=8, dtype=np.float64)
    for parts in (1, 2, 3, 4, 8):
        s = hspmv.partition_rows(A.row_ptr, parts)
        assert s[0] == 0 and s[-1] == A.m and np.all(np.diff(s) >= 0)
        nnz = A.row_ptr[s[1:]] - A.row_ptr[s[:-1]]
        assert nnz.sum() == A.nnz
        assert nnz.max() <= A.nnz / parts + np.diff(A.row_ptr).max()
    maps = hspmv.build_csr3_maps(A, 20, 10)
    ssr_starts = set(maps.inner[maps.outer].tolist())
    s = hspmv.partition_rows(A.row_ptr, 4, maps)
    assert all(int(v) in ssr_starts for v in s)


def test_alg_bytes_formula():
    # C1/C2 fp64 = 79.95 MB
    b = hspmv.alg_bytes(1_000_000, 1_000_000, 4_996_000, np.float64)
    assert b == 4_996_000 * 12 + 1_000_001 * 4 + 2 * 8_000_000
    assert abs(b / 1e6 - 79.95) < 0.01
    assert hspmv.alg_bytes(10, 10, 30, np.float32, 2, 5) == 30 * 8 + 11 * 4 + 80 + 9 * 4


def test_csr2_maps_are_the_first_level_of_the_csr3_grouping():
    # CSR-2 (one level, spmv-csrk/spmv.cpp:28 CSRK_LEVEL 2): inner = the
    # oracle's level-1 handCoarsen grouping at threshold srs*NNZ/N, outer = identity
    for A, srs in [(gen.laplace2d(100, 100), 8), (gen.stencil27(12), 10),
                   (gen.powerlaw(5000, seed=2, dtype=np.float64), 4),
                   (hspmv.read_csr(GOLDEN / "empty_rows.csr"), 2)]:
        maps = hspmv.build_csr2_maps(A, srs)
        _, inner = oracle.build_maps(A.row_ptr, A.col_idx, srs, 1)
        assert np.array_equal(maps.inner, inner)
        assert np.array_equal(maps.outer, np.arange(maps.n_sr + 1))
    with pytest.raises(hspmv.HspmvError):
        hspmv.build_csr2_maps(gen.laplace2d(4, 4), 0)


def test_writers_match_printf_formatting(tmp_path):
    """The parallel writers print what the reference's fprintf calls print:
    "%d " indices and "%f " (.csr) / "%.6f " (.csr3) values -- checked
    against Python's %-formatting (correctly rounded, as glibc's printf) on
    values that stress the rounding: tiny, huge, negative zero, halfway
    cases."""
    rng = np.random.default_rng(11)
    m = 2000
    lens = rng.integers(0, 9, m)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    ci = rng.integers(0, m, rp[-1]).astype(np.int32)
    v = rng.uniform(-1, 1, rp[-1]) * 10.0 ** rng.integers(-9, 12, rp[-1])
    v[:8] = [-0.0, 0.0, 1e20, -1e-7, 5e-7, 0.0000025, 123456.0000005, -2.5e-6]
    A = hspmv.CsrMatrix(m, m, rp, ci, v)
    maps = hspmv.build_csr3_maps(A, 7, 8)
    hspmv.write_csr(tmp_path / "a.csr", A)
    hspmv.write_csr3(tmp_path / "a.csr3", A, maps)
    ints = lambda a: "".join(f"{int(t)} " for t in a)  # noqa: E731
    want = (f"{m} {m} {A.nnz}\n" + ints(rp) + "\n" + ints(ci) + "\n"
            + "".join("%f " % t for t in v) + "\n")
    assert (tmp_path / "a.csr").read_text() == want
    want3 = (f"{maps.n_ssr} {maps.n_sr} {m} {m} {A.nnz} \n" + ints(maps.outer) + ints(maps.inner)
             + ints(rp) + ints(ci) + "".join("%.6f " % t for t in v))
    assert (tmp_path / "a.csr3").read_text() == want3
    # fp32 values print their float's exact decimal
    hspmv.write_csr(tmp_path / "b.csr", A.astype(np.float32))
    vals = (tmp_path / "b.csr").read_text().split("\n")[3].split()
    assert vals == ["%f" % t for t in v.astype(np.float32).astype(np.float64)]
