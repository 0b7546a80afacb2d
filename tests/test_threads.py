"""The ABI's threading contract (include/hspmv.h): a handle is
not re-entrant, distinct handles may be used from different threads at the
same time, and hspmv_last_error() is per thread.  ctypes drops the GIL around
every foreign call, so the threads below really run the library
concurrently."""
import ctypes as C
import threading

import numpy as np
import pytest

import hspmv
import oracle
from conftest import fp64_tol_ok
from hspmv import gen


def test_last_error_is_per_thread(tmp_path):
    lib = hspmv.lib()
    lib.hspmv_last_error.restype = C.c_char_p
    seen = {}

    def fail():
        buf = hspmv._lib.CsrBuf()
        rc = lib.hspmv_read_csr(str(tmp_path / "missing.csr").encode(), 1, C.byref(buf))
        seen["rc"], seen["msg"] = rc, lib.hspmv_last_error().decode()

    ok = hspmv.read_csr  # a successful call in this thread clears its message
    A = gen.laplace2d(10, 10)
    hspmv.write_csr(tmp_path / "a.csr", A)
    ok(tmp_path / "a.csr")
    t = threading.Thread(target=fail)
    t.start()
    t.join()
    assert seen["rc"] != 0 and "missing.csr" in seen["msg"]
    assert lib.hspmv_last_error().decode() == ""


def test_host_builders_in_parallel_threads():
    """Readers / map builders / band-k from several threads at once give the
    same results as one thread."""
    mats = [gen.laplace2d(60 + 7 * i, 50) for i in range(6)]
    want = [hspmv.build_csr3_bandk(A, 7, 8) for A in mats]
    got = [None] * len(mats)

    def work(i):
        got[i] = hspmv.build_csr3_bandk(mats[i], 7, 8)

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(mats))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for (a, am, ap), (b, bm, bp) in zip(want, got):
        assert np.array_equal(a.col_idx, b.col_idx) and np.array_equal(ap, bp)
        assert np.array_equal(am.inner, bm.inner) and np.array_equal(am.outer, bm.outer)


@pytest.mark.gpu
def test_distinct_handles_from_concurrent_threads():
    """Four threads, each with its own handle on its own matrix (STREAM,
    CSR-3 with maps, column-sorted, vector), run 25 SpMVs with fresh x each
    time, at the same time; every y is checked against the oracle."""
    assert hspmv.device_count() >= 1
    cases = [(gen.banded(200000, seed=1), None, "auto"),
             (gen.stencil27(40), "maps", "auto"),
             (gen.powerlaw(120000, seed=5, dtype=np.float64), None, "csort"),
             (gen.laplace2d(300, 300), None, "vector")]
    errors = []

    def work(k):
        try:
            A, mp, kernel = cases[k]
            maps = hspmv.build_csr3_maps(A, 20, 10) if mp else None
            rng = np.random.default_rng(k)
            with hspmv.SpMV(A, maps, device=0, kernel=kernel) as op:
                for it in range(25):
                    x = rng.uniform(-1, 1, A.n)
                    y = op(x)
                    y64 = oracle.spmv(A.row_ptr, A.col_idx, A.val, x)
                    absrow = oracle.abs_rowsum(A.row_ptr, A.col_idx, A.val, x)
                    if not fp64_tol_ok(y, y64, absrow):
                        errors.append((k, it, float(np.abs(y - y64).max())))
                        return
        except Exception as e:  # reported below, in the test's thread
            errors.append((k, repr(e)))

    th = [threading.Thread(target=work, args=(k,)) for k in range(len(cases))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th)
    assert not errors, errors
