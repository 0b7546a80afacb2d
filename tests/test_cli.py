"""The spmv-csr / spmv-csrk executables keep the reference's command line and
stdout contract (TimeMin/TimeMax/TimeAvg in seconds, Number Wrong), parsed the
way run_scripts/run_norm.py:94-107 parses it."""
import re
import subprocess

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, REPO
from hspmv import gen

BUILD = REPO / "heterogeneous-spmv_amd" / "build"


def run(*args, check=True):
    p = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=300)
    if check and p.returncode != 0:
        raise AssertionError(f"{args} -> {p.returncode}\n{p.stdout}\n{p.stderr}")
    return p


def harness_parse(out: str):
    # run_norm.py:94-107: find("TimeMin:") + 8 chars to end of line
    vals = []
    for key in ("TimeMin:", "TimeMax:", "TimeAvg:"):
        i = out.find(key)
        j = out.find("\n", i)
        vals.append(float(out[i + 8:j]))
    return vals


def test_usage_without_gpu():
    # argc < 3 prints the usage line and exits 0 (spmv-csr/spmv.c:118-121)
    p = run(BUILD / "spmv-csr")
    assert "num_runs" in p.stdout
    p = run(BUILD / "spmv-csrk")
    assert "num_runs" in p.stdout


@pytest.mark.gpu
def test_spmv_csr_contract_and_check(tmp_path):
    for name in ("lap32.mtx.rcm", "powerlaw1500", "long_row", "empty_rows"):
        for dtype in ("f64", "f32"):
            p = run(BUILD / "spmv-csr", GOLDEN / f"{name}.csr", 7, "--dtype", dtype, "--x", "rand:42")
            tmin, tmax, tavg = harness_parse(p.stdout)
            assert 0 < tmin <= tavg <= tmax
            assert "Number Wrong: 0" in p.stdout
            assert "Check: PASS" in p.stdout
            assert "TEAST" in p.stdout


@pytest.mark.gpu
def test_spmv_csr_dump_y_is_reference_bitwise_fp32(tmp_path):
    out = tmp_path / "y.bin"
    run(BUILD / "spmv-csr", GOLDEN / "lap32.mtx.rcm.csr", 3, "--dtype", "f32", "--dump-y", out)
    y = np.fromfile(out, np.float32)
    g = np.load(GOLDEN / "lap32.mtx.rcm.npz")
    assert np.array_equal(y.view(np.uint32), g["y_ref_f32_ones"].view(np.uint32))
    run(BUILD / "spmv-csr", GOLDEN / "lap32.mtx.rcm.csr", 3, "--x", "rand:42", "--dump-y", out)
    y = np.fromfile(out, np.float64)
    assert np.array_equal(y, g["y_orc_f64_rand"])


@pytest.mark.gpu
def test_spmv_csr_kernels_and_onebased():
    for extra in (["--kernel", "vector:8"], ["--kernel", "vector"], ["--kernel", "stream", "--nt"]):
        p = run(BUILD / "spmv-csr", GOLDEN / "lap32.onebased.csr", 4, "--x", "rand:1", *extra)
        assert "index_base 1" in p.stdout and "Check: PASS" in p.stdout


@pytest.mark.gpu
def test_spmv_csrk_modes(tmp_path):
    f = GOLDEN / "powerlaw1500.csr"
    # manual sizes (hip/spmv.cu:112-132)
    p = run(BUILD / "spmv-csrk", f, 5, 7, 8, "--x", "rand:3")
    assert "using ssrs 7, srs 8" in p.stdout and "Check: PASS" in p.stdout
    harness_parse(p.stdout)
    # auto sizes (hip/spmv-auto-mi100.cu:130-158)
    for params in ("mi100", "volta", "mi355x"):
        p = run(BUILD / "spmv-csrk", f, 5, "--params", params)
        assert "using ssrs" in p.stdout and "Number Wrong: 0" in p.stdout
    # .csr3 input carries its own maps
    p = run(BUILD / "spmv-csrk", GOLDEN / "powerlaw1500.csr3", 5, "--x", "rand:3")
    assert "using ssrs" not in p.stdout and "Check: PASS" in p.stdout
    assert "Kernel: csr3" in p.stdout


@pytest.mark.gpu
def test_cli_bad_input_fails_loudly(tmp_path):
    bad = tmp_path / "bad.csr"
    bad.write_text("2 2 2\n0 1 2\n0 7\n1.0 2.0\n")
    p = run(BUILD / "spmv-csr", bad, 3, check=False)
    assert p.returncode != 0 and "out of" in p.stderr


@pytest.mark.gpu
def test_bin_cache_through_cli(tmp_path):
    import hspmv
    A = gen.stencil27(30)
    maps = hspmv.build_csr3_maps(A, 20, 10)
    f = tmp_path / "s.bin"
    hspmv.save_bin(f, A, maps)
    p = run(BUILD / "spmv-csrk", f, 5, "--x", "rand:9")
    assert "Check: PASS" in p.stdout and "Kernel: csr3" in p.stdout
    p = run(BUILD / "spmv-csr", f, 5, "--x", "rand:9")
    assert "Check: PASS" in p.stdout and "Kernel: stream" in p.stdout


@pytest.mark.gpu
def test_spmv_csrk_bandk_reorders_and_restores_file_order(tmp_path):
    # a .csr input goes through the band-k build (CSRk_Graph::putInCSRkFormat);
    # x is permuted with the matrix and --dump-y writes y in the file's order
    import hspmv
    A = hspmv.read_csr(GOLDEN / "powerlaw1500.csr", np.float64)
    x = gen.rand_x(A.n, 7)
    y_ref = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    for extra in ([], ["--file-order"]):
        out = tmp_path / "y.bin"
        p = run(BUILD / "spmv-csrk", GOLDEN / "powerlaw1500.csr", 5, 20, 10, "--x", "rand:7",
                "--dump-y", out, *extra)
        assert "Check: PASS" in p.stdout and "reordered in" in p.stdout
        y = np.fromfile(out, np.float64)
        assert np.all(np.abs(y - y_ref) <= 1e-6 * np.abs(y_ref) + 1e-12 * absrow)


def harness_value(out: str, key: str) -> float:
    i = out.find(key)
    j = out.find("\n", i)
    return float(out[i + len(key):j])


@pytest.mark.gpu
def test_spmv_csrk_csr2_three_argument_form(tmp_path):
    # spmv-csrk <file> <num_runs> <super_row_size>: CSR-2, one map level
    # (spmv-csrk/spmv.cpp:97-128, CSRK_LEVEL 2); band-k (default) and file
    # order, y back in file order checked against the oracle
    import hspmv
    A = hspmv.read_csr(GOLDEN / "powerlaw1500.csr", np.float64)
    x = gen.rand_x(A.n, 5)
    y_ref = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
    for extra in ([], ["--file-order"]):
        out = tmp_path / "y.bin"
        p = run(BUILD / "spmv-csrk", GOLDEN / "powerlaw1500.csr", 5, 8, "--x", "rand:5",
                "--dump-y", out, *extra)
        assert "SpMV\nHAND\n2\n8\n" in p.stdout, p.stdout
        assert "Check: PASS" in p.stdout and "Number Wrong: 0" in p.stdout
        m = re.search(r"super-super-rows (\d+) super-rows (\d+)", p.stdout)
        assert m and m.group(1) == m.group(2)  # one super-row per super-super-row
        y = np.fromfile(out, np.float64)
        assert np.all(np.abs(y - y_ref) <= 1e-6 * np.abs(y_ref) + 1e-12 * absrow)
        harness_parse(p.stdout)
    # a bad size fails loudly
    p = run(BUILD / "spmv-csrk", GOLDEN / "powerlaw1500.csr", 5, 0, check=False)
    assert p.returncode != 0


@pytest.mark.gpu
def test_cli_gflops_printed_from_timemin():
    # GFLOPs / GBps are computed from TimeMin (what run_norm.py records), the
    # event-timed rates are KernelGFLOPs / KernelGBps
    import hspmv
    A = hspmv.read_csr(GOLDEN / "lap32.mtx.rcm.csr", np.float64)
    p = run(BUILD / "spmv-csr", GOLDEN / "lap32.mtx.rcm.csr", 9)
    tmin = harness_value(p.stdout, "TimeMin:")
    g = harness_value(p.stdout, "GFLOPs:")
    assert abs(g - 2.0 * A.nnz / tmin * 1e-9) <= 1e-5 * g
    kmin = harness_value(p.stdout, "KernelMin:")
    kg = harness_value(p.stdout, "KernelGFLOPs:")
    assert abs(kg - 2.0 * A.nnz / kmin * 1e-9) <= 1e-5 * kg
    assert "KernelGBps:" in p.stdout and "GBps:" in p.stdout


@pytest.mark.gpu
def test_reference_pipeline_mtx_to_spmv(tmp_path):
    """The reference's whole input pipeline with this framework's tools:
    .mtx -> (mtx2csr, converter.m's role) .csr + .rcm.csr -> (reformat-auto)
    .csr3 -> spmv-csr / spmv-csrk, each run's y checked by the driver."""
    import scipy.io
    import scipy.sparse as sp
    import hspmv
    A = gen.stencil27(20, rcm=False)
    S = sp.csr_matrix((A.val, A.col_idx, A.row_ptr), shape=(A.m, A.n))
    mtx = tmp_path / "s27.mtx"
    scipy.io.mmwrite(str(mtx), sp.tril(S), symmetry="symmetric")
    csr, rcm, csr3 = tmp_path / "s27.mtx.csr", tmp_path / "s27.mtx.rcm.csr", tmp_path / "s27.mtx.rcm.csr3"
    run(BUILD / "mtx2csr", mtx, csr, rcm)
    run(BUILD / "reformat-auto", rcm, csr3)
    for tool, f in (("spmv-csr", csr), ("spmv-csr", rcm), ("spmv-csrk", rcm), ("spmv-csrk", csr3)):
        p = run(BUILD / tool, f, 5, "--x", "rand:4")
        assert "Number Wrong: 0" in p.stdout and "Check: PASS" in p.stdout, (tool, f, p.stdout)
        harness_parse(p.stdout)
    assert hspmv.read_csr(rcm).nnz == A.nnz


@pytest.mark.gpu
def test_spmv_csr_reproducible_and_deterministic_flags(tmp_path):
    """--reproducible (hspmv_options.deterministic = 2) runs the column-sorted
    kernel with fixed-point sums: two runs dump the same y bits and the
    serial check passes; --deterministic (1) refuses an explicit csort."""
    f = GOLDEN / "powerlaw1500.csr"
    ys = []
    for i in range(2):
        out = tmp_path / f"y{i}.bin"
        p = run(BUILD / "spmv-csr", f, 5, "--kernel", "csort", "--reproducible", "--x", "rand:1",
                "--dump-y", out)
        assert "Kernel: csort" in p.stdout and "deterministic=1" in p.stdout
        assert "Check: PASS" in p.stdout
        ys.append(np.fromfile(out, np.float64))
    assert np.array_equal(ys[0].view(np.uint64), ys[1].view(np.uint64))
    p = run(BUILD / "spmv-csr", f, 3, "--kernel", "csort", "--deterministic", check=False)
    assert p.returncode != 0
