"""The band-k CSR-3 build (hspmv_build_csr3_bandk, restating BAND_k::
preprocessingForSpMV, cuda-spmv-csrk/hip/csrk.cu:1035-1262, and reorderA
:722-870).  The reference's CSR-k library needs Boost.Graph and cannot be built
here, so the build is pinned by (a) the reference reformatter's
recorded lap100 output header "174 1411 10000 10000 49600" (SURVEY.md §8a A13),
(b) the invariants SURVEY.md §8f rank 2 names: a symmetric permutation, maps
monotone and complete, columns sorted, y parity after un-permuting."""
import numpy as np
import pytest
import scipy.sparse as sp

import hspmv
import oracle
from conftest import GOLDEN
from hspmv import gen


def _csr(A):
    return sp.csr_matrix((A.val, A.col_idx, A.row_ptr), shape=(A.m, A.n))


def _shuffled(A, seed):
    q = np.random.default_rng(seed).permutation(A.m)
    R = _csr(A)[q][:, q].tocsr()
    R.sort_indices()
    return hspmv.CsrMatrix(A.m, A.n, R.indptr.astype(np.int32), R.indices.astype(np.int32), R.data)


def check_bandk(A, ssrs, srs):
    Ap, maps, perm = hspmv.build_csr3_bandk(A, ssrs, srs)
    m = A.m
    # a permutation, and A_perm = P A P^T exactly (values moved, not changed)
    assert np.array_equal(np.sort(perm), np.arange(m))
    M, Mp = _csr(A), _csr(Ap)
    assert (abs(M[perm][:, perm] - Mp)).nnz == 0
    assert Ap.nnz == A.nnz
    # columns sorted (strictly) per row
    for r in range(0, m, max(1, m // 500)):
        c = Ap.col_idx[Ap.row_ptr[r]:Ap.row_ptr[r + 1]]
        assert np.all(np.diff(c) > 0)
    # maps monotone and complete
    o, i = maps.outer, maps.inner
    assert o[0] == 0 and o[-1] == maps.n_sr and np.all(np.diff(o) > 0)
    assert i[0] == 0 and i[-1] == m and np.all(np.diff(i) > 0)
    # level-1 grouping runs in file order: same super-row count as the
    # file-order builder, the super-row sizes permuted
    fo = hspmv.build_csr3_maps(A, ssrs, srs)
    assert fo.n_sr == maps.n_sr
    assert np.array_equal(np.sort(np.diff(fo.inner)), np.sort(np.diff(i)))
    # y parity: A_perm @ x[perm] == (A @ x)[perm] (oracle, fp64, same order of sums per row
    # up to the column re-sort, so compared within tolerance)
    x = gen.rand_x(A.n, 5)
    y = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    yp = oracle.spmv(Ap.row_ptr, Ap.col_idx, Ap.val, x[perm])
    assert np.allclose(yp, y[perm], rtol=1e-12, atol=1e-12)
    return Ap, maps, perm


def test_lap100_matches_reference_header():
    A = gen.laplace2d(100, 100)
    ssrs, srs = hspmv.csr3_params(A.nnz / A.m, "volta")
    Ap, maps, perm = check_bandk(A, ssrs, srs)
    assert (maps.n_ssr, maps.n_sr, Ap.m, Ap.n, Ap.nnz) == (174, 1411, 10000, 10000, 49600)


@pytest.mark.parametrize("name,ssrs,srs", [("lap32.mtx.rcm", 7, 8), ("powerlaw1500", 20, 10),
                                           ("banded3000", 7, 8), ("empty_rows", 3, 2)])
def test_invariants_on_fixtures(name, ssrs, srs):
    A = hspmv.read_csr(GOLDEN / f"{name}.csr", np.float64)
    check_bandk(A, ssrs, srs)


def test_invariants_on_generators():
    for A, p in [(gen.stencil27(16), (20, 10)), (_shuffled(gen.laplace2d(60, 50), 3), (7, 8)),
                 (gen.powerlaw(4000, seed=8, dtype=np.float64), (64, 4))]:
        check_bandk(A, *p)


def test_deterministic_and_fp32():
    A = gen.stencil27(12)
    a = hspmv.build_csr3_bandk(A, 20, 10)
    b = hspmv.build_csr3_bandk(A, 20, 10)
    assert np.array_equal(a[2], b[2]) and np.array_equal(a[1].inner, b[1].inner)
    A32 = hspmv.CsrMatrix(A.m, A.n, A.row_ptr, A.col_idx, A.val.astype(np.float32))
    Ap32, maps32, perm32 = hspmv.build_csr3_bandk(A32, 20, 10)
    assert np.array_equal(perm32, a[2]) and Ap32.val.dtype == np.float32


def test_rejects_rectangular():
    A = hspmv.CsrMatrix(2, 3, np.array([0, 1, 2], np.int32), np.array([0, 2], np.int32),
                        np.ones(2))
    with pytest.raises(hspmv.HspmvError):
        hspmv.build_csr3_bandk(A, 2, 2)


def check_bandk2(A, srs):
    """CSR-2 (k = 2): one coarsening + RCM (csrk.cu:1072-1096 with k = 2)."""
    Ap, maps, perm = hspmv.build_csr2_bandk(A, srs)
    m = A.m
    assert np.array_equal(np.sort(perm), np.arange(m))
    assert (abs(_csr(A)[perm][:, perm] - _csr(Ap))).nnz == 0
    o, i = maps.outer, maps.inner
    assert maps.n_ssr == maps.n_sr and np.array_equal(o, np.arange(maps.n_sr + 1))
    assert i[0] == 0 and i[-1] == m and np.all(np.diff(i) > 0)
    fo = hspmv.build_csr2_maps(A, srs)
    assert fo.n_sr == maps.n_sr
    assert np.array_equal(np.sort(np.diff(fo.inner)), np.sort(np.diff(i)))
    # the super-rows are whole groups of the file order, moved as blocks
    for s in range(0, maps.n_sr, max(1, maps.n_sr // 200)):
        rows = perm[i[s]:i[s + 1]]
        assert np.all(np.diff(rows) == 1)
    x = gen.rand_x(A.n, 5)
    y = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    yp = oracle.spmv(Ap.row_ptr, Ap.col_idx, Ap.val, x[perm])
    assert np.allclose(yp, y[perm], rtol=1e-12, atol=1e-12)
    return Ap, maps, perm


@pytest.mark.parametrize("name,srs", [("lap32.mtx.rcm", 8), ("powerlaw1500", 10),
                                      ("banded3000", 4), ("empty_rows", 2)])
def test_csr2_invariants_on_fixtures(name, srs):
    A = hspmv.read_csr(GOLDEN / f"{name}.csr", np.float64)
    check_bandk2(A, srs)


def test_csr2_on_generators_and_shuffled_order_is_recovered():
    check_bandk2(gen.stencil27(14), 10)
    # a shuffled Laplacian: the RCM of the super-row graph brings the band back
    A = _shuffled(gen.laplace2d(40, 40), 11)
    Ap, maps, perm = check_bandk2(A, 1)
    rows = np.repeat(np.arange(Ap.m), np.diff(Ap.row_ptr))
    bw = np.abs(Ap.col_idx - rows).max()
    rows0 = np.repeat(np.arange(A.m), np.diff(A.row_ptr))
    assert bw < np.abs(A.col_idx - rows0).max() / 4
