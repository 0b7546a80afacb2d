"""The offline converters reformat-auto / reformat (cli/reformat.cpp), the
reference's reformat-csr-to-csr3 tools (spmv-auto.cpp:132-200, spmv.cpp:
132-190).  Host only: they run here without a GPU.

Pinned by the reference reformatter's recorded lap100 output header
"174 1411 10000 10000 49600" (SURVEY.md §8a A13), and by the library's
band-k build (tests/test_bandk.py holds its invariants): the files hold
exactly hspmv_build_csr3_bandk's matrix and maps, values as "%.6f" of the
float the reference parses."""
import subprocess

import numpy as np
import pytest

import hspmv
from conftest import GOLDEN, REPO
from hspmv import gen

BUILD = REPO / "heterogeneous-spmv_amd" / "build"


def run(*args, check=True):
    p = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=300)
    if check and p.returncode != 0:
        raise AssertionError(f"{args} -> {p.returncode}\n{p.stdout}\n{p.stderr}")
    return p


def six(v):
    """Values as the converters print them: %.6f of the fp32 value."""
    return np.array([float(f"{x:.6f}") for x in np.asarray(v, np.float32).astype(np.float64)])


def expected(path, ssrs, srs):
    A = hspmv.read_csr(path, np.float32)
    return hspmv.build_csr3_bandk(A, ssrs, srs)


def test_usage_and_errors(tmp_path):
    for tool in ("reformat-auto", "reformat"):
        p = run(BUILD / tool)
        assert "Syntax:" in p.stdout and p.returncode == 0
    rect = hspmv.CsrMatrix(3, 5, np.array([0, 1, 2, 3]), np.array([0, 4, 2]), np.ones(3))
    gen.write_csr_text(str(tmp_path / "rect.csr"), rect)
    p = run(BUILD / "reformat-auto", tmp_path / "rect.csr", tmp_path / "o.csr3", check=False)
    assert p.returncode == 1 and "square" in p.stderr
    p = run(BUILD / "reformat-auto", tmp_path / "missing.csr", tmp_path / "o.csr3", check=False)
    assert p.returncode == 1
    p = run(BUILD / "reformat-auto", tmp_path / "rect.csr", tmp_path / "o.csr3", "--ssrs", "3",
            check=False)
    assert p.returncode == 1


def test_lap100_header_matches_reference(tmp_path):
    src = tmp_path / "lap100.csr"
    gen.write_csr_text(str(src), gen.laplace2d(100, 100))
    out = tmp_path / "lap100.csr3"
    p = run(BUILD / "reformat-auto", src, out)
    # the reference's banner lines (spmv-auto.cpp:171-192)
    assert "using ssrs 7, srs 8" in p.stdout
    assert "SpMV\nHAND\n3\n78\n" in p.stdout and "In CSR-k format." in p.stdout
    assert "reordered in" in p.stdout
    assert out.read_text().split("\n", 1)[0].split() == ["174", "1411", "10000", "10000", "49600"]


@pytest.mark.parametrize("name", ["lap32.mtx.rcm", "powerlaw1500", "banded3000", "empty_rows"])
def test_csr3_file_is_the_bandk_build(tmp_path, name):
    src = GOLDEN / f"{name}.csr"
    A = hspmv.read_csr(src, np.float32)
    ssrs, srs = hspmv.csr3_params(A.nnz / A.m, "volta")
    Ap, maps, _ = expected(src, ssrs, srs)
    out = tmp_path / "o.csr3"
    run(BUILD / "reformat-auto", src, out)
    B, bm = hspmv.read_csr3(out, np.float64)
    assert (bm.n_ssr, bm.n_sr) == (maps.n_ssr, maps.n_sr)
    assert np.array_equal(bm.outer, maps.outer) and np.array_equal(bm.inner, maps.inner)
    assert np.array_equal(B.row_ptr, Ap.row_ptr) and np.array_equal(B.col_idx, Ap.col_idx)
    assert np.array_equal(B.val, six(Ap.val))


def test_plain_reformat_and_overrides(tmp_path):
    src = GOLDEN / "powerlaw1500.csr"
    Ap, _, _ = expected(src, 5, 3)
    out = tmp_path / "o.csr2"
    p = run(BUILD / "reformat", src, out, "96", "--ssrs", "5", "--srs", "3")
    assert "using ssrs 5, srs 3" in p.stdout
    B = hspmv.read_csr(out, np.float64)
    assert np.array_equal(B.row_ptr, Ap.row_ptr) and np.array_equal(B.col_idx, Ap.col_idx)
    assert np.array_equal(B.val, six(Ap.val))
    # the .csr3 of the same sizes feeds spmv-csrk's .csr3 path unchanged
    out3 = tmp_path / "o.csr3"
    run(BUILD / "reformat-auto", src, out3, "--ssrs", "5", "--srs", "3")
    B3, m3 = hspmv.read_csr3(out3, np.float64)
    assert np.array_equal(B3.col_idx, B.col_idx) and m3.inner[-1] == B3.m


REF_STATS = REPO / "oracle" / "_ref" / "stats"


@pytest.mark.parametrize("name", ["lap32.mtx.rcm", "powerlaw1500", "banded3000"])
def test_csr_stats_matches_reference_tool(tmp_path, name):
    """csr-stats prints what the reference's spmv-csr/stats.c prints (its
    binary, built from the reference's sources by `make -C oracle ref`, is
    the checker; fixtures without empty rows, where stats.c reads outside
    the row)."""
    if not REF_STATS.exists():
        pytest.skip("oracle/_ref/stats not built (needs /root/reference)")
    src = GOLDEN / f"{name}.csr"
    ours = run(BUILD / "csr-stats", src).stdout
    ref = run(REF_STATS, src).stdout
    assert ours == ref
    # the .csr3 form: the same statistics of its embedded CSR, plus the maps
    A = hspmv.read_csr(src, np.float32)
    out = tmp_path / "o.csr3"
    run(BUILD / "reformat-auto", src, out)
    B, maps = hspmv.read_csr3(out, np.float64)
    s3 = run(BUILD / "csr-stats", out).stdout
    assert f"Total NNZ: {A.nnz}\n" in s3 and f"Dim: {A.m}x{A.n}\n" in s3
    assert f"Super-super-rows: {maps.n_ssr} Super-rows: {maps.n_sr}" in s3


def test_csr_stats_empty_rows_and_usage():
    p = run(BUILD / "csr-stats")
    assert "inputfile" in p.stdout
    s = run(BUILD / "csr-stats", GOLDEN / "empty_rows.csr").stdout
    A = hspmv.read_csr(GOLDEN / "empty_rows.csr", np.float64)
    lens = np.diff(A.row_ptr)
    assert f"NNZ Min: {lens.min()}  " in s and f"NNZ Max: {lens.max()}  " in s
    assert f"NNZ Var: {np.var(lens):f} " in s
