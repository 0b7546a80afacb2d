"""oracle.py -- TEST INFRASTRUCTURE ONLY.

numpy front end of the CPU restatement in spmv_oracle.c (liboracle.so) and of
the reference's own spmv-csr/spmv.c compiled by ``make -C oracle ref`` into
oracle/_ref/libref_spmvcsr.so.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product never does.

Functions mirror the reference symbols they restate (file:line in
spmv_oracle.c):
    read_csr      -> my_read_csr          spmv-csr/spmv.c:11-57
    spmv          -> omp_spmv             spmv-csr/spmv.c:92-114
    spmv_serial   -> test_spmv            spmv-csr/spmv.c:68-90
    csr3_spmv     -> CSRk_Graph::SpMV k=3 spmv-csrk/csrk.cpp:247-285
    build_maps    -> handCoarsen grouping cuda-spmv-csrk/hip/csrk.cu:1438-1484
    time_spmv     -> timed loop           spmv-csr/spmv.c:164-185
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
REF_LIB = HERE / "_ref" / "libref_spmvcsr.so"

_i64 = C.c_int64
_p = C.c_void_p
_pp = C.POINTER(C.c_void_p)
_lib = None
_ref = None
_SCHED = {"static": 1, "dynamic": 2, "guided": 3, "auto": 4}


def build(ref: bool = False) -> None:
    subprocess.run(["make", "-C", str(HERE), "-s"] + (["ref"] if ref else []), check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        for nm in ("orc_omp_spmv_f32", "orc_test_spmv_f32"):
            getattr(L, nm).argtypes = [_i64, _p, _p, _p, _p, _p]
        for nm in ("orc_omp_spmv_f64", "orc_test_spmv_f64", "orc_abs_rowsum_f64"):
            getattr(L, nm).argtypes = [_i64, _p, _p, _p, _p, _p]
        L.orc_csr3_spmv_f64.argtypes = [_i64, _p, _p, _p, _p, _p, _p, _p]
        L.orc_csr3_spmv_f32.argtypes = [_i64, _p, _p, _p, _p, _p, _p, _p]
        L.orc_read_csr.argtypes = [C.c_char_p, C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64),
                                   _pp, _pp, _pp, _pp, C.POINTER(C.c_int)]
        L.orc_read_csr3.argtypes = [C.c_char_p] + [C.POINTER(_i64)] * 5 + [_pp] * 6
        L.orc_build_csr3_maps.argtypes = [_i64, _p, _p, _i64, _i64, C.POINTER(_i64),
                                          C.POINTER(_i64), _pp, _pp]
        L.orc_time_omp_spmv_f64.argtypes = [_i64, _p, _p, _p, _p, _p, C.c_int, C.c_int,
                                            C.POINTER(C.c_double), C.POINTER(C.c_double),
                                            C.POINTER(C.c_double)]
        L.orc_time_omp_spmv_f32.argtypes = L.orc_time_omp_spmv_f64.argtypes
        L.orc_free.argtypes = [_p]
        L.orc_max_threads.restype = C.c_int
        L.orc_set_schedule.argtypes = [C.c_int, C.c_int]
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_set_schedule(_SCHED[os.environ.get("OMP_SCHEDULE", "static").split(",")[0]], 0)
        _lib = L
    return _lib


def _c(a):
    return a.ctypes.data


def _arr(ptr, n, ctype, dtype):
    if n == 0:
        lib().orc_free(ptr)
        return np.zeros(0, dtype)
    a = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ctype)), (n,)).copy()
    lib().orc_free(ptr)
    return a


def read_csr(path):
    """-> (m, n, row_ptr, col_idx, val32, val64, base)."""
    m, n, z = _i64(), _i64(), _i64()
    rp, ci, v32, v64 = _p(), _p(), _p(), _p()
    base = C.c_int()
    rc = lib().orc_read_csr(str(path).encode(), C.byref(m), C.byref(n), C.byref(z), C.byref(rp),
                            C.byref(ci), C.byref(v32), C.byref(v64), C.byref(base))
    if rc != 0:
        raise IOError(f"orc_read_csr({path}) = {rc}")
    M, Z = m.value, z.value
    return (M, n.value, _arr(rp, M + 1, C.c_int32, np.int32), _arr(ci, Z, C.c_int32, np.int32),
            _arr(v32, Z, C.c_float, np.float32), _arr(v64, Z, C.c_double, np.float64), base.value)


def read_csr3(path):
    """-> (outer, inner, m, n, row_ptr, col_idx, val32, val64)."""
    h = [_i64() for _ in range(5)]
    ps = [_p() for _ in range(6)]
    rc = lib().orc_read_csr3(str(path).encode(), *[C.byref(x) for x in h],
                             *[C.byref(x) for x in ps])
    if rc != 0:
        raise IOError(f"orc_read_csr3({path}) = {rc}")
    nssr, nsr, m, n, z = (x.value for x in h)
    return (_arr(ps[0], nssr + 1, C.c_int32, np.int32), _arr(ps[1], nsr + 1, C.c_int32, np.int32),
            m, n, _arr(ps[2], m + 1, C.c_int32, np.int32), _arr(ps[3], z, C.c_int32, np.int32),
            _arr(ps[4], z, C.c_float, np.float32), _arr(ps[5], z, C.c_double, np.float64))


def _prep(row_ptr, col_idx, val, x):
    rp = np.ascontiguousarray(row_ptr, np.int32)
    ci = np.ascontiguousarray(col_idx, np.int32)
    val = np.ascontiguousarray(val)
    x = np.ascontiguousarray(x, val.dtype)
    return rp, ci, val, x


def spmv(row_ptr, col_idx, val, x, serial: bool = False) -> np.ndarray:
    """omp_spmv (or test_spmv when serial) in the dtype of val."""
    rp, ci, val, x = _prep(row_ptr, col_idx, val, x)
    m = rp.shape[0] - 1
    y = np.zeros(m, val.dtype)
    L = lib()
    if val.dtype == np.float64:
        fn = L.orc_test_spmv_f64 if serial else L.orc_omp_spmv_f64
    elif val.dtype == np.float32:
        fn = L.orc_test_spmv_f32 if serial else L.orc_omp_spmv_f32
    else:
        raise TypeError(val.dtype)
    fn(m, _c(rp), _c(ci), _c(val), _c(x), _c(y))
    return y


def abs_rowsum(row_ptr, col_idx, val, x) -> np.ndarray:
    """sum_k |val[k] * x[col[k]]| per row, in fp64 (tolerance floor)."""
    rp, ci, _, _ = _prep(row_ptr, col_idx, val, x)
    v = np.ascontiguousarray(val, np.float64)
    xx = np.ascontiguousarray(x, np.float64)
    s = np.zeros(rp.shape[0] - 1, np.float64)
    lib().orc_abs_rowsum_f64(rp.shape[0] - 1, _c(rp), _c(ci), _c(v), _c(xx), _c(s))
    return s


def csr3_spmv(outer, inner, row_ptr, col_idx, val, x) -> np.ndarray:
    rp, ci, val, x = _prep(row_ptr, col_idx, val, x)
    o = np.ascontiguousarray(outer, np.int32)
    i = np.ascontiguousarray(inner, np.int32)
    y = np.full(rp.shape[0] - 1, np.nan, val.dtype)
    fn = lib().orc_csr3_spmv_f64 if val.dtype == np.float64 else lib().orc_csr3_spmv_f32
    fn(o.shape[0] - 1, _c(o), _c(i), _c(rp), _c(ci), _c(val), _c(x), _c(y))
    return y


def build_maps(row_ptr, col_idx, ssrs: int, srs: int):
    rp = np.ascontiguousarray(row_ptr, np.int32)
    ci = np.ascontiguousarray(col_idx, np.int32)
    nssr, nsr = _i64(), _i64()
    po, pi = _p(), _p()
    lib().orc_build_csr3_maps(rp.shape[0] - 1, _c(rp), _c(ci), ssrs, srs, C.byref(nssr),
                              C.byref(nsr), C.byref(po), C.byref(pi))
    return (_arr(po, nssr.value + 1, C.c_int32, np.int32),
            _arr(pi, nsr.value + 1, C.c_int32, np.int32))


def set_schedule(kind: str = "static", threads: int = 0) -> None:
    lib().orc_set_schedule(_SCHED[kind], 0)
    lib().orc_set_threads(int(threads))


def time_spmv_samples(row_ptr, col_idx, val, x, warmup: int = 5, runs: int = 20) -> np.ndarray:
    """The same protocol, every run's seconds (for the median)."""
    rp, ci, val, x = _prep(row_ptr, col_idx, val, x)
    y = np.zeros(rp.shape[0] - 1, val.dtype)
    out = np.zeros(int(runs), np.float64)
    L = lib()
    fn = L.orc_time_omp_spmv_samples_f64 if val.dtype == np.float64 else L.orc_time_omp_spmv_samples_f32
    fn.argtypes = [_i64, _p, _p, _p, _p, _p, C.c_int, C.c_int, _p]
    fn(rp.shape[0] - 1, _c(rp), _c(ci), _c(val), _c(x), _c(y), int(warmup), int(runs), _c(out))
    return out


def bind_threads(nthreads: int, places: list) -> int:
    """Team thread t -> CPU set places[t % len(places)] (orc_bind_threads);
    returns the threads bound."""
    off = np.zeros(len(places) + 1, np.int32)
    off[1:] = np.cumsum([len(p) for p in places])
    cpus = np.array([c for p in places for c in p] or [0], np.int32)
    L = lib()
    L.orc_bind_threads.argtypes = [C.c_int, C.c_int, _p, _p]
    return int(L.orc_bind_threads(int(nthreads), len(places), _c(off), _c(cpus)))


def localize(row_ptr, col_idx, val):
    """First-touch copies of a CSR in omp_spmv's static row partition
    (orc_localize_csr): each team thread's rows on its own NUMA node."""
    rp = np.ascontiguousarray(row_ptr, np.int32)
    ci = np.ascontiguousarray(col_idx, np.int32)
    val = np.ascontiguousarray(val)
    rp2, ci2, v2 = np.empty_like(rp), np.empty_like(ci), np.empty_like(val)  # untouched pages
    L = lib()
    L.orc_localize_csr.argtypes = [_i64, _p, _p, _p, C.c_int, _p, _p, _p]
    L.orc_localize_csr(rp.shape[0] - 1, _c(rp), _c(ci), _c(val), val.itemsize, _c(rp2), _c(ci2),
                       _c(v2))
    return rp2, ci2, v2


def time_spmv(row_ptr, col_idx, val, x, warmup: int = 5, runs: int = 20):
    """OpenMP omp_spmv timed like spmv-csr/spmv.c:164-185 -> (tmin, tmax, tavg, threads)."""
    rp, ci, val, x = _prep(row_ptr, col_idx, val, x)
    y = np.zeros(rp.shape[0] - 1, val.dtype)
    a, b, c = C.c_double(), C.c_double(), C.c_double()
    fn = lib().orc_time_omp_spmv_f64 if val.dtype == np.float64 else lib().orc_time_omp_spmv_f32
    fn(rp.shape[0] - 1, _c(rp), _c(ci), _c(val), _c(x), _c(y), warmup, runs, C.byref(a),
       C.byref(b), C.byref(c))
    return a.value, b.value, c.value, lib().orc_max_threads()


# ------------------------------------------------------------------ reference

def ref_available() -> bool:
    return REF_LIB.exists()


def ref() -> C.CDLL:
    """The reference's own spmv-csr/spmv.c (built from /root/reference)."""
    global _ref
    if _ref is None:
        if not REF_LIB.exists():
            build(ref=True)
        R = C.CDLL(str(REF_LIB))
        R.my_read_csr.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                  C.POINTER(C.c_int), _pp, _pp, _pp]
        R.omp_spmv.argtypes = [C.c_int, C.c_int, C.c_int, _p, _p, _p, _p, _p]
        R.test_spmv.argtypes = R.omp_spmv.argtypes
        _ref = R
    return _ref


def ref_spmv(row_ptr, col_idx, val, x) -> np.ndarray:
    """The reference's own omp_spmv (spmv-csr/spmv.c:92-114) on in-memory fp32
    arrays (its reader is pinned separately by the golden fixtures)."""
    R = ref()
    rp, ci, v, xx = _prep(row_ptr, col_idx, np.asarray(val, np.float32), x)
    y = np.zeros(rp.shape[0] - 1, np.float32)
    R.omp_spmv(rp.shape[0] - 1, xx.shape[0], ci.shape[0], _c(rp), _c(ci), _c(v), _c(xx), _c(y))
    return y


def ref_spmv_file(path, x: np.ndarray | None = None, serial: bool = False) -> np.ndarray:
    """Runs the reference reader + omp_spmv (or test_spmv) on a .csr file.
    x defaults to all-ones (spmv-csr/spmv.c:133); otherwise float32(x)."""
    R = ref()
    m, n, z = C.c_int(), C.c_int(), C.c_int()
    rp, ci, val = _p(), _p(), _p()
    R.my_read_csr(str(path).encode(), C.byref(m), C.byref(n), C.byref(z), C.byref(rp),
                  C.byref(ci), C.byref(val))
    xx = np.ones(max(m.value, n.value), np.float32) if x is None else np.ascontiguousarray(x, np.float32)
    y = np.zeros(m.value, np.float32)
    fn = R.test_spmv if serial else R.omp_spmv
    fn(m.value, n.value, z.value, rp, ci, val, _c(xx), _c(y))
    for p in (rp, ci, val):
        lib().orc_free(p)
    return y

