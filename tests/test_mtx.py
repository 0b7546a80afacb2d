"""Matrix Market input (hspmv_read_mtx, the mtx2csr CLI and
hspmv_rcm_reorder): the reference's Octave converter (helpers/converter.m
with helpers/mmread.m, helpers/sparse2csr.m) is the contract, Octave is
absent, so the reader is pinned against scipy.io.mmread (the same
MatrixMarket semantics: symmetric files expanded, duplicates summed) and
against the .csr files of the golden fixtures; the RCM order against its
invariants (a symmetric permutation that narrows the band of a shuffled
mesh).  The exact symrcm order is parity-unpinned (Octave's tie-breaking).
Host only."""
import subprocess

import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp

import hspmv
import oracle
from conftest import GOLDEN, REPO
from hspmv import gen

BUILD = REPO / "heterogeneous-spmv_amd" / "build"


def run(*args, check=True):
    p = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=300)
    if check and p.returncode != 0:
        raise AssertionError(f"{args} -> {p.returncode}\n{p.stdout}\n{p.stderr}")
    return p


def expected(path):
    S = sp.csr_matrix(scipy.io.mmread(str(path)))
    if "skew-symmetric" in open(path).readline().lower():
        # mmread.m forms A - A.' (helpers/mmread.m:214-216): a stored diagonal
        # entry cancels; scipy keeps it
        S = S - sp.diags(S.diagonal())
    S.sum_duplicates()
    S.eliminate_zeros()
    S.sort_indices()
    return S


def same(A, S):
    assert (A.m, A.n, A.nnz) == (S.shape[0], S.shape[1], S.nnz)
    assert np.array_equal(A.row_ptr, S.indptr) and np.array_equal(A.col_idx, S.indices)
    assert np.array_equal(A.val, S.data.astype(A.val.dtype))


MTX = {
    "general_real": """%%MatrixMarket matrix coordinate real general
% a comment
4 5 7
1 1 1.5
2 3 -2.25e-1
4 5 3
1 4 7.125
3 2 0.5
2 3 1.0
4 1 0
""",
    "symmetric_real": """%%MatrixMarket matrix coordinate real symmetric
4 4 6
1 1 2.0
2 1 -1.0
3 2 -1.0
4 3 -1.0
4 4 2.0
4 1 0.25
""",
    "pattern_symmetric": """%%MatrixMarket matrix coordinate pattern symmetric
%
5 5 5
2 1
3 1
5 2
4 4
5 3
""",
    "skew_integer": """%%MatrixMarket matrix coordinate integer skew-symmetric
3 3 3
2 1 3
3 1 -4
2 2 5
""",
}


@pytest.mark.parametrize("name", sorted(MTX))
def test_read_mtx_matches_scipy(tmp_path, name):
    f = tmp_path / f"{name}.mtx"
    f.write_text(MTX[name])  # general_real: a duplicate (2, 3) and an explicit zero
    same(hspmv.read_mtx(f, np.float64), expected(f))


def test_read_mtx_errors(tmp_path):
    bad = {
        "array.mtx": "%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n",
        "complex.mtx": "%%MatrixMarket matrix coordinate complex general\n1 1 1\n1 1 1 0\n",
        "short.mtx": "%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1\n2 2 1\n",
        "range.mtx": "%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1\n",
        # 2^32 + 1 would wrap to row 1 if narrowed to int32 before the check
        "wrap.mtx": "%%MatrixMarket matrix coordinate real general\n2 2 1\n4294967297 1 1\n",
        "zero_index.mtx": "%%MatrixMarket matrix coordinate real general\n2 2 1\n1 0 1\n",
        "nonsquare_sym.mtx": "%%MatrixMarket matrix coordinate real symmetric\n2 3 1\n1 1 1\n",
        "noheader.mtx": "2 2 1\n1 1 1\n",
    }
    for fname, text in bad.items():
        f = tmp_path / fname
        f.write_text(text)
        with pytest.raises(hspmv.HspmvError):
            hspmv.read_mtx(f)
    with pytest.raises(hspmv.HspmvError):
        hspmv.read_mtx(tmp_path / "missing.mtx")


def test_read_mtx_out_of_range_values(tmp_path):
    """Values beyond the double range read as mmread's fscanf reads them:
    1e400 -> +Inf, -1e400 -> -Inf, 1e-400 -> 0 (then dropped as an explicit
    zero), never as the parser's initial 1.0."""
    f = tmp_path / "huge.mtx"
    f.write_text("%%MatrixMarket matrix coordinate real general\n3 3 4\n"
                 "1 1 1e400\n2 2 -1e400\n3 3 1e-400\n1 3 2.5\n")
    A = hspmv.read_mtx(f, np.float64)
    d = {(r, int(c)): v for r in range(A.m)
         for c, v in zip(A.col_idx[A.row_ptr[r]:A.row_ptr[r + 1]], A.val[A.row_ptr[r]:A.row_ptr[r + 1]])}
    assert d[(0, 0)] == np.inf and d[(1, 1)] == -np.inf and d[(0, 2)] == 2.5
    assert (2, 2) not in d and A.nnz == 3


def test_read_mtx_long_overflowing_token(tmp_path):
    """A 400-digit literal with no exponent overflows to +Inf (the whole
    token is parsed, not its first 127 characters), and a tiny literal
    written with 400 leading zeros underflows to a dropped zero."""
    big = "9" * 400
    tiny = "0." + "0" * 400 + "1"
    f = tmp_path / "long.mtx"
    f.write_text("%%MatrixMarket matrix coordinate real general\n2 2 3\n"
                 f"1 1 {big}\n2 2 -{big}.5\n1 2 {tiny}\n")
    A = hspmv.read_mtx(f, np.float64)
    assert A.nnz == 2
    assert A.val[0] == np.inf and A.val[1] == -np.inf


def test_read_mtx_large_parallel(tmp_path):
    # enough lines that every parse thread gets a share, CRLF line ends
    A = gen.powerlaw(20000, seed=3, dtype=np.float64)
    S = sp.csr_matrix((A.val, A.col_idx, A.row_ptr), shape=(A.m, A.n))
    f = tmp_path / "pl.mtx"
    scipy.io.mmwrite(str(f), sp.tril(S), symmetry="symmetric")
    f.write_bytes(f.read_bytes().replace(b"\n", b"\r\n"))
    same(hspmv.read_mtx(f, np.float64), expected(f))


def test_mtx2csr_writes_converter_files(tmp_path):
    """mtx2csr in.mtx out.csr out.rcm.csr: what converter.m writes per file
    (the .csr read back equals the .mtx; values printed "%f")."""
    f = tmp_path / "sym.mtx"
    f.write_text(MTX["symmetric_real"])
    out, rcm = tmp_path / "sym.mtx.csr", tmp_path / "sym.mtx.rcm.csr"
    p = run(BUILD / "mtx2csr", f, out, rcm)
    assert p.stdout.startswith("Converting matrix sym.mtx...") and p.stdout.rstrip().endswith("done")
    S = expected(f)
    head = out.read_text().split("\n")[0].split()
    assert head == [str(S.shape[0]), str(S.shape[1]), str(S.nnz)]
    B = hspmv.read_csr(out, np.float64)
    assert np.array_equal(B.row_ptr, S.indptr) and np.array_equal(B.col_idx, S.indices)
    assert np.allclose(B.val, S.data, atol=5e-7)
    R = hspmv.read_csr(rcm, np.float64)
    assert R.nnz == S.nnz and sorted(np.diff(R.row_ptr)) == sorted(np.diff(S.indptr))
    assert run(BUILD / "mtx2csr").stdout.startswith("Syntax:")
    assert run(BUILD / "mtx2csr", tmp_path / "missing.mtx", out, check=False).returncode == 1


def test_golden_fixture_round_trip(tmp_path):
    """A golden .csr written as .mtx and converted back gives the same CSR."""
    A = hspmv.read_csr(GOLDEN / "lap32.mtx.rcm.csr", np.float64)
    S = sp.csr_matrix((A.val, A.col_idx, A.row_ptr), shape=(A.m, A.n))
    f = tmp_path / "lap32.mtx"
    scipy.io.mmwrite(str(f), S, precision=17)
    B = hspmv.read_mtx(f, np.float64)
    assert np.array_equal(B.row_ptr, A.row_ptr) and np.array_equal(B.col_idx, A.col_idx)
    assert np.array_equal(B.val, A.val)


def _bandwidth(A):
    rows = np.repeat(np.arange(A.m), np.diff(A.row_ptr))
    return int(np.abs(A.col_idx - rows).max()) if A.nnz else 0


def test_rcm_reorder_is_a_symmetric_permutation_that_narrows_the_band():
    L = gen.laplace2d(60, 40)
    q = np.random.default_rng(5).permutation(L.m)
    S = sp.csr_matrix((L.val, L.col_idx, L.row_ptr), shape=(L.m, L.n))[q][:, q].tocsr()
    S.sort_indices()
    A = hspmv.CsrMatrix(L.m, L.n, S.indptr, S.indices, S.data)
    R, perm = hspmv.rcm_reorder(A)
    assert np.array_equal(np.sort(perm), np.arange(A.m))
    P = sp.csr_matrix((R.val, R.col_idx, R.row_ptr), shape=(A.m, A.n))
    assert abs(S[perm][:, perm] - P).nnz == 0
    assert _bandwidth(R) <= 2 * 40 and _bandwidth(A) > 10 * _bandwidth(R)
    x = gen.rand_x(A.n, 2)
    assert np.allclose(oracle.spmv(R.row_ptr, R.col_idx, R.val, x[perm]),
                       oracle.spmv(A.row_ptr, A.col_idx, A.val, x)[perm], rtol=0, atol=1e-12)
    # disconnected pieces, an isolated vertex, a non-symmetric pattern
    B = hspmv.CsrMatrix(5, 5, np.array([0, 1, 2, 2, 3, 4]), np.array([3, 0, 1, 4]), np.ones(4))
    R2, p2 = hspmv.rcm_reorder(B)
    assert np.array_equal(np.sort(p2), np.arange(5)) and R2.nnz == 4
    with pytest.raises(hspmv.HspmvError):
        hspmv.rcm_reorder(hspmv.CsrMatrix(2, 3, np.array([0, 1, 1]), np.array([2]), np.ones(1)))


def test_mtx2csr_binary_outputs(tmp_path):
    f = tmp_path / "sym.mtx"
    f.write_text(MTX["symmetric_real"])
    run(BUILD / "mtx2csr", f, tmp_path / "s.bin", tmp_path / "s.rcm.bin")
    A, maps = hspmv.load_bin(tmp_path / "s.bin")
    S = expected(f)
    assert maps is None and np.array_equal(A.row_ptr, S.indptr) and np.array_equal(A.val, S.data)
    R, _ = hspmv.load_bin(tmp_path / "s.rcm.bin")
    assert R.nnz == S.nnz
