"""Python host mirror of the reference's CSR / CSR-3 SpMV interface, on top of
the libhspmv C ABI (include/hspmv.h).

Reference interface it mirrors:

* ``CSRk_Graph(nRows, nCols, nnz, rVec, cVec, val, ..., k, supRowSizes)`` +
  ``putInCSRkFormat()`` / ``setX()`` / ``setY()`` / ``getY()``
  (cuda-spmv-csrk/hip/csrk.cuh:321-353)  ->  :class:`SpMV` (+ :func:`build_csr3_maps`)
* ``my_read_csr`` (spmv-csr/spmv.c:11-57), ``my_read_csr3``
  (reformat-csr-to-csr3/stats.c:10-79)  ->  :func:`read_csr`, :func:`read_csr3`
* the timed loop + ``TimeMin/TimeMax/TimeAvg`` (spmv-csr/spmv.c:164-185)
  ->  :meth:`SpMV.run`

Every call goes to the GPU through libhspmv; errors raise :class:`HspmvError`.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _lib
from ._lib import (F32, F64, KERNEL_AUTO, KERNEL_CSORT, KERNEL_CSR3, KERNEL_STREAM, KERNEL_VECTOR,
                   FLAG_DEVICE_PTRS, FLAG_NONTEMPORAL, HspmvError, check, lanes_flag, lib,
                   remap_flag)

_KERNELS = {"auto": KERNEL_AUTO, "vector": KERNEL_VECTOR, "stream": KERNEL_STREAM,
            "csr3": KERNEL_CSR3, "csort": KERNEL_CSORT}
KERNEL_NAMES = {v: k for k, v in _KERNELS.items()}


def dtype_code(dtype) -> int:
    dt = np.dtype(dtype)
    if dt == np.float64:
        return F64
    if dt == np.float32:
        return F32
    raise ValueError(f"unsupported dtype {dt} (float32 / float64)")


def np_dtype(code: int):
    return np.float64 if code == F64 else np.float32


def _ptr(a: Optional[np.ndarray]) -> Optional[int]:
    return None if a is None else a.ctypes.data


@dataclass
class CsrMatrix:
    """Host CSR matrix (0-based int32 indices, float32/float64 values)."""
    m: int
    n: int
    row_ptr: np.ndarray
    col_idx: np.ndarray
    val: np.ndarray
    index_base: int = 0

    def __post_init__(self):
        self.row_ptr = np.ascontiguousarray(self.row_ptr, dtype=np.int32)
        self.col_idx = np.ascontiguousarray(self.col_idx, dtype=np.int32)
        self.val = np.ascontiguousarray(self.val)
        if self.val.dtype not in (np.float32, np.float64):
            self.val = self.val.astype(np.float64)

    @property
    def nnz(self) -> int:
        return int(self.col_idx.shape[0])

    @property
    def dtype(self):
        return self.val.dtype

    def astype(self, dtype) -> "CsrMatrix":
        return CsrMatrix(self.m, self.n, self.row_ptr, self.col_idx,
                         self.val.astype(dtype), self.index_base)

    def c_struct(self) -> _lib.Csr:
        return _lib.Csr(self.m, self.n, self.nnz, _ptr(self.row_ptr), _ptr(self.col_idx),
                        _ptr(self.val), dtype_code(self.val.dtype))

    @classmethod
    def from_scipy(cls, S, dtype=np.float64) -> "CsrMatrix":
        S = S.tocsr()
        S.sort_indices()
        return cls(S.shape[0], S.shape[1], S.indptr, S.indices, S.data.astype(dtype))

    def to_scipy(self):
        import scipy.sparse as sp
        return sp.csr_matrix((self.val, self.col_idx, self.row_ptr), shape=(self.m, self.n))

    def rows(self, r0: int, r1: int) -> "CsrMatrix":
        """Rows [r0, r1) with row_ptr rebased to 0 (global columns kept)."""
        k0, k1 = int(self.row_ptr[r0]), int(self.row_ptr[r1])
        return CsrMatrix(r1 - r0, self.n, self.row_ptr[r0:r1 + 1] - k0,
                         self.col_idx[k0:k1], self.val[k0:k1])


@dataclass
class Csr3Maps:
    """CSR-3 multilevel maps: outer (n_ssr+1) -> super-rows, inner (n_sr+1) -> rows."""
    outer: np.ndarray
    inner: np.ndarray

    def __post_init__(self):
        self.outer = np.ascontiguousarray(self.outer, dtype=np.int32)
        self.inner = np.ascontiguousarray(self.inner, dtype=np.int32)

    @property
    def n_ssr(self) -> int:
        return int(self.outer.shape[0] - 1)

    @property
    def n_sr(self) -> int:
        return int(self.inner.shape[0] - 1)

    def c_struct(self) -> _lib.Csr3Maps:
        return _lib.Csr3Maps(self.n_ssr, self.n_sr, _ptr(self.outer), _ptr(self.inner))


# ------------------------------------------------------------------ formats

def _take_csr(buf: _lib.CsrBuf) -> CsrMatrix:
    m, nnz = int(buf.m), int(buf.nnz)
    dt = np_dtype(buf.dtype)
    rp = np.ctypeslib.as_array(C.cast(buf.row_ptr, C.POINTER(C.c_int32)), (m + 1,)).copy()
    if nnz:
        ci = np.ctypeslib.as_array(C.cast(buf.col_idx, C.POINTER(C.c_int32)), (nnz,)).copy()
        ctype = C.c_double if dt == np.float64 else C.c_float
        val = np.ctypeslib.as_array(C.cast(buf.val, C.POINTER(ctype)), (nnz,)).copy()
    else:
        ci = np.zeros(0, np.int32)
        val = np.zeros(0, dt)
    A = CsrMatrix(m, int(buf.n), rp, ci, val, int(buf.index_base))
    lib().hspmv_free_csr(C.byref(buf))
    return A


def _take_maps(buf: _lib.Csr3Buf) -> Optional[Csr3Maps]:
    if buf.n_ssr <= 0:
        lib().hspmv_free_csr3(C.byref(buf))
        return None
    o = np.ctypeslib.as_array(C.cast(buf.outer, C.POINTER(C.c_int32)), (int(buf.n_ssr) + 1,)).copy()
    i = np.ctypeslib.as_array(C.cast(buf.inner, C.POINTER(C.c_int32)), (int(buf.n_sr) + 1,)).copy()
    lib().hspmv_free_csr3(C.byref(buf))
    return Csr3Maps(o, i)


def read_csr(path: str, dtype=np.float64) -> CsrMatrix:
    buf = _lib.CsrBuf()
    check(lib().hspmv_read_csr(str(path).encode(), dtype_code(dtype), C.byref(buf)), "read_csr")
    return _take_csr(buf)


def read_mtx(path: str, dtype=np.float64) -> CsrMatrix:
    """Matrix Market coordinate file as mmread.m + sparse2csr.m read it
    (hspmv_read_mtx: symmetric files expanded, duplicates summed, zeros
    dropped, columns sorted)."""
    buf = _lib.CsrBuf()
    check(lib().hspmv_read_mtx(str(path).encode(), dtype_code(dtype), C.byref(buf)), "read_mtx")
    return _take_csr(buf)


def rcm_reorder(A: CsrMatrix):
    """Reverse Cuthill-McKee of A's symmetrised pattern (hspmv_rcm_reorder):
    (A_perm, perm) with row i of A_perm = row perm[i] of A."""
    cs, buf = A.c_struct(), _lib.CsrBuf()
    perm = np.empty(A.m, np.int32)
    check(lib().hspmv_rcm_reorder(C.byref(cs), C.byref(buf), _ptr(perm)), "rcm_reorder")
    return _take_csr(buf), perm


def read_csr3(path: str, dtype=np.float64):
    buf, mbuf = _lib.CsrBuf(), _lib.Csr3Buf()
    check(lib().hspmv_read_csr3(str(path).encode(), dtype_code(dtype), C.byref(buf),
                                C.byref(mbuf)), "read_csr3")
    return _take_csr(buf), _take_maps(mbuf)


def write_csr(path: str, A: CsrMatrix) -> None:
    cs = A.c_struct()
    check(lib().hspmv_write_csr(str(path).encode(), C.byref(cs)), "write_csr")


def write_csr3(path: str, A: CsrMatrix, maps: Csr3Maps) -> None:
    cs, ms = A.c_struct(), maps.c_struct()
    check(lib().hspmv_write_csr3(str(path).encode(), C.byref(cs), C.byref(ms)), "write_csr3")


def save_bin(path: str, A: CsrMatrix, maps: Optional[Csr3Maps] = None) -> None:
    cs = A.c_struct()
    ms = maps.c_struct() if maps is not None else None
    check(lib().hspmv_save_bin(str(path).encode(), C.byref(cs),
                               C.byref(ms) if ms is not None else None), "save_bin")


def load_bin(path: str):
    buf, mbuf = _lib.CsrBuf(), _lib.Csr3Buf()
    check(lib().hspmv_load_bin(str(path).encode(), C.byref(buf), C.byref(mbuf)), "load_bin")
    return _take_csr(buf), _take_maps(mbuf)


def build_csr3_maps(A: CsrMatrix, ssrs: int, srs: int) -> Csr3Maps:
    cs, mbuf = A.c_struct(), _lib.Csr3Buf()
    check(lib().hspmv_build_csr3_maps(C.byref(cs), int(ssrs), int(srs), C.byref(mbuf)),
          "build_csr3_maps")
    maps = _take_maps(mbuf)
    if maps is None:  # empty matrix: one empty super-super-row is not needed
        maps = Csr3Maps(np.zeros(1, np.int32), np.zeros(1, np.int32))
    return maps


def build_csr3_bandk(A: CsrMatrix, ssrs: int, srs: int):
    """The reference's band-k CSR-3 build (hspmv_build_csr3_bandk): returns
    (A_perm, maps, perm) with A_perm = P A P^T, row i of A_perm = row perm[i]
    of A; so A_perm @ x[perm] = (A @ x)[perm]."""
    cs, buf, mbuf = A.c_struct(), _lib.CsrBuf(), _lib.Csr3Buf()
    perm = np.empty(A.m, np.int32)
    check(lib().hspmv_build_csr3_bandk(C.byref(cs), int(ssrs), int(srs), C.byref(buf),
                                       C.byref(mbuf), _ptr(perm)), "build_csr3_bandk")
    Ap = _take_csr(buf)
    maps = _take_maps(mbuf)
    if maps is None:
        maps = Csr3Maps(np.zeros(1, np.int32), np.zeros(1, np.int32))
    return Ap, maps, perm


def build_csr2_maps(A: CsrMatrix, super_row_size: int) -> Csr3Maps:
    """CSR-2 maps (one level; outer = identity): hspmv_build_csr2_maps."""
    cs, mbuf = A.c_struct(), _lib.Csr3Buf()
    check(lib().hspmv_build_csr2_maps(C.byref(cs), int(super_row_size), C.byref(mbuf)),
          "build_csr2_maps")
    maps = _take_maps(mbuf)
    if maps is None:
        maps = Csr3Maps(np.zeros(1, np.int32), np.zeros(1, np.int32))
    return maps


def build_csr2_bandk(A: CsrMatrix, super_row_size: int):
    """The k = 2 band-k build (hspmv_build_csr2_bandk): (A_perm, maps, perm)
    as build_csr3_bandk, maps with one super-row per super-super-row."""
    cs, buf, mbuf = A.c_struct(), _lib.CsrBuf(), _lib.Csr3Buf()
    perm = np.empty(A.m, np.int32)
    check(lib().hspmv_build_csr2_bandk(C.byref(cs), int(super_row_size), C.byref(buf),
                                       C.byref(mbuf), _ptr(perm)), "build_csr2_bandk")
    Ap = _take_csr(buf)
    maps = _take_maps(mbuf)
    if maps is None:
        maps = Csr3Maps(np.zeros(1, np.int32), np.zeros(1, np.int32))
    return Ap, maps, perm


_FLAVOURS = {"volta": 0, "csr3-writer": 0, "mi100": 1, "mi355x": 2}


def csr3_params(nnz_per_row: float, flavour: str = "mi355x"):
    a, b = C.c_int(), C.c_int()
    check(lib().hspmv_csr3_params(float(nnz_per_row), _FLAVOURS[flavour], C.byref(a), C.byref(b)),
          "csr3_params")
    return a.value, b.value


def partition_rows(row_ptr: np.ndarray, parts: int, maps: Optional[Csr3Maps] = None) -> np.ndarray:
    rp = np.ascontiguousarray(row_ptr, dtype=np.int32)
    out = np.zeros(parts + 1, np.int64)
    ms = maps.c_struct() if maps is not None else None
    check(lib().hspmv_partition_rows(rp.shape[0] - 1, _ptr(rp),
                                     C.byref(ms) if ms is not None else None, int(parts),
                                     _ptr(out)), "partition_rows")
    return out


def xdict_plan(A: CsrMatrix, maps: Optional[Csr3Maps] = None, *, kernel: str = "auto",
               cap_entries: int = 0, split: bool = True, options: Optional[dict] = None):
    """Block x dictionaries the library would build for A (hspmv_xdict_plan_ex):
    (blk, runs, pos) with runs as an (n_records, 2) array of {x_start,
    lds_off}, or None when some workgroup exceeds cap_entries (0 = the
    library's LDS cap for A's dtype)."""
    cs = A.c_struct()
    ms = maps.c_struct() if maps is not None else None
    flags = _KERNELS[kernel] | (0 if split else _lib.FLAG_NO_SPLIT)
    opt = _lib.make_options(flags, options)
    nb, nr = C.c_int64(), C.c_int64()
    L = lib()
    args = (C.byref(cs), C.byref(ms) if ms is not None else None, C.byref(opt), int(cap_entries))
    check(L.hspmv_xdict_plan_ex(*args, C.byref(nb), C.byref(nr), None, None, None), "xdict_plan")
    if nb.value == 0:
        return None
    blk = np.empty(nb.value + 1, np.int32)
    runs = np.empty((nr.value, 2), np.int32)
    pos = np.zeros(max(A.nnz, 1), np.uint16)
    check(L.hspmv_xdict_plan_ex(*args, C.byref(nb), C.byref(nr), _ptr(blk), _ptr(runs), _ptr(pos)),
          "xdict_plan")
    return blk, runs, pos[:A.nnz]


def alg_bytes(m: int, n: int, nnz: int, dtype, n_ssr: int = 0, n_sr: int = 0) -> float:
    return float(lib().hspmv_alg_bytes(m, n, nnz, dtype_code(dtype), n_ssr, n_sr))


def device_count() -> int:
    c = C.c_int()
    rc = lib().hspmv_device_count(C.byref(c))
    return c.value if rc == 0 else 0


def version() -> str:
    return lib().hspmv_version().decode()


# ------------------------------------------------------------------ handle

class SpMV:
    """One SpMV operator y = A x on one or more GPUs (a libhspmv handle).

    ``kernel``: "auto" | "stream" | "vector" | "csr3" | "csort";  ``lanes``: lanes per row
    for "vector" (0 = auto).  ``device``/``stream``: single-device handle on that
    HIP device / hipStream_t (as an int); ``devices``: row-range shards on that
    device list (hspmv_create_sharded; devices may repeat); otherwise
    ``num_gpus`` GPUs with the row-range partition.  ``options``: explicit
    planner choices (hspmv_options fields by name, e.g. ``{"csr3_plan": "ssr",
    "deterministic": "ordered"}`` -- deterministic 1 / "ordered": the ordered
    row kernels; 2 / "reproducible": bit-identical run to run, csort with
    fixed-point row sums allowed; 3 / "serial": every row summed in
    omp_spmv's order, y bit-identical to it; handle created with
    hspmv_create_ex).
    """

    def __init__(self, A: CsrMatrix, maps: Optional[Csr3Maps] = None, *, num_gpus: int = 1,
                 kernel: str = "auto", lanes: int = 0, nontemporal: bool = False,
                 device: Optional[int] = None, stream: Optional[int] = None,
                 xcd_remap: Optional[bool] = None, split_rows: bool = True, chunk_u: int = 0,
                 prefetch: Optional[bool] = None, xcd_chunk: int = 0, groups_per_wave: int = 0,
                 col16: Optional[bool] = None, devices: Optional[list] = None,
                 options: Optional[dict] = None):
        self.A = A
        self.maps = maps
        self.dtype = A.val.dtype
        flags = _KERNELS[kernel] | lanes_flag(lanes) | (FLAG_NONTEMPORAL if nontemporal else 0)
        flags |= remap_flag(xcd_remap, xcd_chunk) | _lib.groups_flag(groups_per_wave)
        flags |= _lib.col16_flag(col16)
        flags |= (0 if split_rows else _lib.FLAG_NO_SPLIT)
        if chunk_u:
            if chunk_u not in (2, 3, 4, 5, 6, 8, 16):
                raise ValueError("chunk_u must be one of 2, 3, 4, 5, 6, 8, 16")
            flags |= chunk_u << _lib.U_SHIFT
        if prefetch:
            flags |= _lib.FLAG_PREFETCH
        cs = A.c_struct()
        ms = maps.c_struct() if maps is not None else None
        h = C.c_void_p()
        if options:  # explicit planner choices: hspmv_create_ex
            if num_gpus != 1 and devices is None:
                # num_gpus <= 0 means every visible GPU, as in hspmv_create
                n = num_gpus if num_gpus > 0 else device_count()
                if n < 1:
                    raise HspmvError("hspmv_create_ex", -6, "no HIP device visible")
                devices = list(range(n))
            opt = _lib.make_options(flags, options, device=0 if device is None else device,
                                    stream=stream, devices=devices)
            rc = lib().hspmv_create_ex(C.byref(h), C.byref(cs),
                                       C.byref(ms) if ms is not None else None, C.byref(opt))
        elif devices is not None:  # row-range shards on an explicit device list
            dl = (C.c_int * len(devices))(*[int(d) for d in devices])
            rc = lib().hspmv_create_sharded(C.byref(h), C.byref(cs),
                                            C.byref(ms) if ms is not None else None, dl,
                                            len(devices), flags)
        elif device is not None:
            rc = lib().hspmv_create_on_device(C.byref(h), C.byref(cs),
                                              C.byref(ms) if ms is not None else None,
                                              int(device), stream, flags)
        else:
            rc = lib().hspmv_create(C.byref(h), C.byref(cs),
                                    C.byref(ms) if ms is not None else None, int(num_gpus), flags)
        check(rc, "hspmv_create")
        self._h = h

    @classmethod
    def from_device(cls, csr_dev: "_lib.Csr", maps_dev: "Optional[_lib.Csr3Maps]", A_meta: CsrMatrix,
                    *, device: int = 0, stream: Optional[int] = None, kernel: str = "auto",
                    lanes: int = 0, nontemporal: bool = False, xcd_remap: Optional[bool] = None,
                    split_rows: bool = True, chunk_u: int = 0,
                    prefetch: Optional[bool] = None, xcd_chunk: int = 0,
                    groups_per_wave: int = 0, col16: Optional[bool] = None,
                    options: Optional[dict] = None) -> "SpMV":
        """Handle over caller-owned DEVICE arrays (HSPMV_FLAG_DEVICE_PTRS):
        csr_dev/maps_dev hold device pointers; A_meta supplies m, n, dtype."""
        self = cls.__new__(cls)
        self.A = A_meta
        self.maps = None
        self.dtype = A_meta.val.dtype
        flags = (_KERNELS[kernel] | lanes_flag(lanes) | (FLAG_NONTEMPORAL if nontemporal else 0)
                 | FLAG_DEVICE_PTRS | remap_flag(xcd_remap, xcd_chunk)
                 | _lib.groups_flag(groups_per_wave) | _lib.col16_flag(col16)
                 | (0 if split_rows else _lib.FLAG_NO_SPLIT) | (chunk_u << _lib.U_SHIFT)
                 | (_lib.FLAG_PREFETCH if prefetch else 0))
        h = C.c_void_p()
        opt = _lib.make_options(flags, options, device=device, stream=stream)
        check(lib().hspmv_create_ex(C.byref(h), C.byref(csr_dev),
                                    C.byref(maps_dev) if maps_dev is not None else None,
                                    C.byref(opt)), "hspmv_create_ex")
        self._h = h
        return self

    # -- vectors
    def set_x(self, x: np.ndarray) -> None:
        x = np.ascontiguousarray(x, dtype=self.dtype)
        if x.shape[0] != self.A.n:
            raise ValueError(f"x has {x.shape[0]} entries, expected n={self.A.n}")
        check(lib().hspmv_set_x(self._h, _ptr(x)), "hspmv_set_x")

    def bind_x_device(self, ptr: Optional[int]) -> None:
        check(lib().hspmv_bind_x_device(self._h, ptr), "hspmv_bind_x_device")

    def bind_y_device(self, ptr: Optional[int]) -> None:
        check(lib().hspmv_bind_y_device(self._h, ptr), "hspmv_bind_y_device")

    def x_device(self, gpu: int = 0) -> int:
        return lib().hspmv_x_device(self._h, gpu) or 0

    def y_device(self, gpu: int = 0) -> int:
        return lib().hspmv_y_device(self._h, gpu) or 0

    # -- compute
    def spmv(self) -> None:
        check(lib().hspmv_spmv(self._h), "hspmv_spmv")

    def synchronize(self) -> None:
        check(lib().hspmv_synchronize(self._h), "hspmv_synchronize")

    def run(self, warmup: int = 5, iters: int = 20) -> dict:
        t = _lib.Timing()
        check(lib().hspmv_run(self._h, int(warmup), int(iters), C.byref(t)), "hspmv_run")
        return {k: getattr(t, k) for k, _ in _lib.Timing._fields_}

    def get_y(self) -> np.ndarray:
        y = np.empty(self.A.m, dtype=self.dtype)
        check(lib().hspmv_get_y(self._h, _ptr(y)), "hspmv_get_y")
        return y

    def __call__(self, x: np.ndarray) -> np.ndarray:
        self.set_x(x)
        self.spmv()
        return self.get_y()

    def exchange(self):
        b, g = C.c_double(), C.c_double()
        check(lib().hspmv_exchange(self._h, C.byref(b), C.byref(g)), "hspmv_exchange")
        return b.value, g.value

    @property
    def info(self) -> dict:
        i = _lib.Info()
        check(lib().hspmv_get_info_sized(self._h, C.byref(i), C.sizeof(i)), "hspmv_get_info_sized")
        d = {k: getattr(i, k) for k, _ in _lib.Info._fields_}
        d["placement_us"] = [round(v, 3) for v in d["placement_us"][:d["placement_trials"]]]
        d["csort_part_begin"] = [int(v) for v in d["csort_part_begin"][:max(d["csort_parts"], 0)]]
        d["kernel_name"] = KERNEL_NAMES.get(d["kernel"], "?")
        return d

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().hspmv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
