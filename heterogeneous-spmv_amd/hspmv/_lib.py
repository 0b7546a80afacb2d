"""ctypes binding of libhspmv.so (the C ABI declared in include/hspmv.h).

The library is loaded from ``heterogeneous-spmv_amd/build/libhspmv.so.1`` (built
in-tree by ``make`` / ``__graft_entry__.build()``).  There is no fallback: if
the shared library is missing or fails to load, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # heterogeneous-spmv_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_PATH = Path(os.environ.get("HSPMV_LIB", PKG_ROOT / "build" / "libhspmv.so.1"))
HEADER = REPO_ROOT / "include" / "hspmv.h"

F32, F64 = 0, 1

KERNEL_AUTO, KERNEL_VECTOR, KERNEL_STREAM, KERNEL_CSR3, KERNEL_CSORT = 0, 1, 2, 3, 4
LANES_SHIFT = 4
FLAG_NO_COL16 = 1 << 11
FLAG_NONTEMPORAL = 1 << 12
FLAG_DEVICE_PTRS = 1 << 13
FLAG_NO_XCD_REMAP = 1 << 14
FLAG_NO_SPLIT = 1 << 15
U_SHIFT = 16
FLAG_PREFETCH = 1 << 21
FLAG_XCD_REMAP = 1 << 22
FLAG_COL16 = 1 << 23
XCD_CHUNK_SHIFT = 24
GROUPS_SHIFT = 29

E_CODES = {0: "OK", -1: "E_INVALID", -2: "E_IO", -3: "E_NOMEM", -4: "E_HIP",
           -5: "E_RCCL", -6: "E_NODEV", -7: "E_STATE"}


def remap_flag(xcd_remap, xcd_chunk: int = 0) -> int:
    """None = library default (remap when the matrix fits the Infinity Cache);
    xcd_chunk (a power of two) overrides: blocks per XCD turn, 1 = dispatch order."""
    if xcd_chunk:
        s = int(xcd_chunk)
        if s < 1 or s & (s - 1):
            raise ValueError("xcd_chunk must be a power of two >= 1")
        return (s.bit_length()) << XCD_CHUNK_SHIFT
    if xcd_remap is None:
        return 0
    return FLAG_XCD_REMAP if xcd_remap else FLAG_NO_XCD_REMAP


def col16_flag(col16) -> int:
    """None = library default (HBM-resident matrices, <= 1 high-bit plane);
    True forces 16-bit column offsets (<= 8 planes); False keeps 32-bit."""
    if col16 is None:
        return 0
    return FLAG_COL16 if col16 else FLAG_NO_COL16


def groups_flag(groups: int) -> int:
    if not groups:
        return 0
    g = int(groups)
    if g not in (1, 2, 4, 8, 16):
        raise ValueError("groups_per_wave must be one of 1, 2, 4, 8, 16")
    return g.bit_length() << GROUPS_SHIFT


def lanes_flag(lanes: int) -> int:
    return (int(lanes) & 0x7F) << LANES_SHIFT


class HspmvError(RuntimeError):
    def __init__(self, what: str, code: int, msg: str):
        super().__init__(f"{what}: {E_CODES.get(code, code)}: {msg}")
        self.code = code


class Csr(C.Structure):
    _fields_ = [("m", C.c_int64), ("n", C.c_int64), ("nnz", C.c_int64),
                ("row_ptr", C.c_void_p), ("col_idx", C.c_void_p), ("val", C.c_void_p),
                ("dtype", C.c_int32)]


class Csr3Maps(C.Structure):
    _fields_ = [("n_ssr", C.c_int64), ("n_sr", C.c_int64),
                ("outer", C.c_void_p), ("inner", C.c_void_p)]


class CsrBuf(C.Structure):
    _fields_ = [("m", C.c_int64), ("n", C.c_int64), ("nnz", C.c_int64),
                ("row_ptr", C.c_void_p), ("col_idx", C.c_void_p), ("val", C.c_void_p),
                ("dtype", C.c_int32), ("index_base", C.c_int32)]


class Csr3Buf(C.Structure):
    _fields_ = [("n_ssr", C.c_int64), ("n_sr", C.c_int64),
                ("outer", C.c_void_p), ("inner", C.c_void_p)]


class Timing(C.Structure):
    _fields_ = [("t_min", C.c_double), ("t_max", C.c_double), ("t_avg", C.c_double),
                ("wall_min", C.c_double), ("wall_max", C.c_double), ("wall_avg", C.c_double),
                ("gflops", C.c_double), ("gbps_alg", C.c_double),
                ("iters", C.c_int32), ("num_gpus", C.c_int32)]


class Info(C.Structure):
    _fields_ = [("kernel", C.c_int32), ("lanes", C.c_int32), ("waves_per_block", C.c_int32),
                ("num_gpus", C.c_int32), ("blocks", C.c_int64), ("alg_bytes", C.c_double),
                ("flops", C.c_double), ("device_bytes", C.c_int64), ("chunk_u", C.c_int32),
                ("n_split_rows", C.c_int32), ("xcd_remap", C.c_int32), ("groups_per_wave", C.c_int32),
                ("x_entries", C.c_int64), ("format_bytes", C.c_double), ("col16", C.c_int32),
                ("wave_tasks", C.c_int32), ("x_windows", C.c_int32), ("x_dict", C.c_int32),
                ("x_dict_entries", C.c_int64), ("x_slabs", C.c_int32),
                ("col16_group", C.c_int32), ("csort_parts", C.c_int32),
                ("placement_trials", C.c_int32), ("placement_pick", C.c_int32),
                ("placement_us", C.c_double * 8),
                ("deterministic", C.c_int32), ("csr3_plan", C.c_int32),
                ("csort_slot_bytes", C.c_int32), ("csort_row_blocks", C.c_int32),
                ("rccl_version", C.c_int32), ("reserved0", C.c_int32),
                ("csort_chunks", C.c_int64), ("csort_seg_chunks", C.c_int64),
                ("slab_kernel_rule", C.c_int32), ("lds_pad", C.c_int32),
                ("heavy_group_frac", C.c_double),
                # since 1.1
                ("csort_fixed_point", C.c_int32), ("serial_order", C.c_int32),
                ("csort_part_begin", C.c_int64 * 4)]


CSR3_PLANS = {"auto": 0, "aligned": 1, "packed": 2, "ssr": 3}
# hspmv_options.deterministic (HSPMV_DETERMINISTIC_*)
DETERMINISTIC = {"any": 0, "ordered": 1, "reproducible": 2, "serial": 3}
CSR3_PLAN_NAMES = {0: None, 1: "aligned", 2: "packed", 3: "ssr", 4: "row_groups"}


class Options(C.Structure):
    """hspmv_options (include/hspmv.h): explicit planner choices for
    hspmv_create_ex; 0 everywhere = the library's choice."""
    _fields_ = [("struct_size", C.c_uint32), ("flags", C.c_uint32),
                ("devices", C.POINTER(C.c_int)), ("n_devices", C.c_int32),
                ("device", C.c_int32), ("stream", C.c_void_p),
                ("csr3_plan", C.c_int32), ("task_nnz", C.c_int32), ("x_windows", C.c_int32),
                ("x_dict", C.c_int32), ("x_dict_cap", C.c_int32), ("x_slabs", C.c_int32),
                ("col16_group", C.c_int32), ("csort", C.c_int32), ("csort_parts", C.c_int32),
                ("csort_chunk_u", C.c_int32), ("stream_waves", C.c_int32),
                ("deterministic", C.c_int32), ("placement_trials", C.c_int32)]

    # planner fields a caller may set by name (SpMV(..., options={...}))
    TUNABLE = ("csr3_plan", "task_nnz", "x_windows", "x_dict", "x_dict_cap", "x_slabs",
               "col16_group", "csort", "csort_parts", "csort_chunk_u", "stream_waves",
               "deterministic", "placement_trials")


def make_options(flags: int, tuning: dict | None, *, device: int = 0, stream=None,
                 devices=None) -> Options:
    o = Options()
    o.struct_size = C.sizeof(Options)
    o.flags = flags
    o.device = int(device)
    o.stream = stream
    if devices is not None:
        arr = (C.c_int * len(devices))(*[int(d) for d in devices])
        o._devices_keepalive = arr
        o.devices = C.cast(arr, C.POINTER(C.c_int))
        o.n_devices = len(devices)
    for k, v in (tuning or {}).items():
        if k not in Options.TUNABLE:
            raise ValueError(f"unknown hspmv option {k!r} (one of {', '.join(Options.TUNABLE)})")
        if k == "csr3_plan" and isinstance(v, str):
            v = CSR3_PLANS[v]
        if k == "deterministic" and isinstance(v, str):
            v = DETERMINISTIC[v]
        setattr(o, k, int(v))
    return o


_P = C.c_void_p
_H = C.c_void_p
# name -> (restype, argtypes); every entry point declared in include/hspmv.h
SIGNATURES = {
    "hspmv_create": (C.c_int, [C.POINTER(_H), C.POINTER(Csr), C.POINTER(Csr3Maps), C.c_int, C.c_uint]),
    "hspmv_create_on_device": (C.c_int, [C.POINTER(_H), C.POINTER(Csr), C.POINTER(Csr3Maps),
                                         C.c_int, _P, C.c_uint]),
    "hspmv_create_sharded": (C.c_int, [C.POINTER(_H), C.POINTER(Csr), C.POINTER(Csr3Maps),
                                       C.POINTER(C.c_int), C.c_int, C.c_uint]),
    "hspmv_create_ex": (C.c_int, [C.POINTER(_H), C.POINTER(Csr), C.POINTER(Csr3Maps),
                                  C.POINTER(Options)]),
    "hspmv_set_x": (C.c_int, [_H, _P]),
    "hspmv_bind_x_device": (C.c_int, [_H, _P]),
    "hspmv_bind_y_device": (C.c_int, [_H, _P]),
    "hspmv_x_device": (_P, [_H, C.c_int]),
    "hspmv_y_device": (_P, [_H, C.c_int]),
    "hspmv_spmv": (C.c_int, [_H]),
    "hspmv_synchronize": (C.c_int, [_H]),
    "hspmv_run": (C.c_int, [_H, C.c_int, C.c_int, C.POINTER(Timing)]),
    "hspmv_get_y": (C.c_int, [_H, _P]),
    "hspmv_exchange": (C.c_int, [_H, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "hspmv_get_info": (C.c_int, [_H, C.POINTER(Info)]),
    "hspmv_get_info_sized": (C.c_int, [_H, C.POINTER(Info), C.c_uint32]),
    "hspmv_destroy": (None, [_H]),
    "hspmv_read_csr": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(CsrBuf)]),
    "hspmv_read_mtx": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(CsrBuf)]),
    "hspmv_rcm_reorder": (C.c_int, [C.POINTER(Csr), C.POINTER(CsrBuf), C.c_void_p]),
    "hspmv_read_csr3": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(CsrBuf), C.POINTER(Csr3Buf)]),
    "hspmv_write_csr": (C.c_int, [C.c_char_p, C.POINTER(Csr)]),
    "hspmv_write_csr3": (C.c_int, [C.c_char_p, C.POINTER(Csr), C.POINTER(Csr3Maps)]),
    "hspmv_save_bin": (C.c_int, [C.c_char_p, C.POINTER(Csr), C.POINTER(Csr3Maps)]),
    "hspmv_load_bin": (C.c_int, [C.c_char_p, C.POINTER(CsrBuf), C.POINTER(Csr3Buf)]),
    "hspmv_free_csr": (None, [C.POINTER(CsrBuf)]),
    "hspmv_free_csr3": (None, [C.POINTER(Csr3Buf)]),
    "hspmv_build_csr3_maps": (C.c_int, [C.POINTER(Csr), C.c_int, C.c_int, C.POINTER(Csr3Buf)]),
    "hspmv_build_csr3_bandk": (C.c_int, [C.POINTER(Csr), C.c_int, C.c_int, C.POINTER(CsrBuf),
                                         C.POINTER(Csr3Buf), _P]),
    "hspmv_build_csr2_maps": (C.c_int, [C.POINTER(Csr), C.c_int, C.POINTER(Csr3Buf)]),
    "hspmv_build_csr2_bandk": (C.c_int, [C.POINTER(Csr), C.c_int, C.POINTER(CsrBuf),
                                         C.POINTER(Csr3Buf), _P]),
    "hspmv_csr3_params": (C.c_int, [C.c_double, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "hspmv_partition_rows": (C.c_int, [C.c_int64, _P, C.POINTER(Csr3Maps), C.c_int, _P]),
    "hspmv_xdict_plan_ex": (C.c_int, [C.POINTER(Csr), C.POINTER(Csr3Maps), C.POINTER(Options), C.c_int64,
                                      C.POINTER(C.c_int64), C.POINTER(C.c_int64), _P, _P, _P]),
    "hspmv_xdict_plan": (C.c_int, [C.POINTER(Csr), C.POINTER(Csr3Maps), C.c_uint, C.c_int64,
                                   C.POINTER(C.c_int64), C.POINTER(C.c_int64), _P, _P, _P]),
    "hspmv_alg_bytes": (C.c_double, [C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int64, C.c_int64]),
    "hspmv_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "hspmv_rccl_version": (C.c_int, [C.POINTER(C.c_int)]),
    "hspmv_last_error": (C.c_char_p, []),
    "hspmv_version": (C.c_char_p, []),
}

_LIB = None


def lib() -> C.CDLL:
    """Loads libhspmv.so once (RTLD_GLOBAL off).  Raises if it is missing."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"libhspmv.so not found at {LIB_PATH}: build it with "
                f"`make -C {PKG_ROOT}` or `python -c 'import __graft_entry__ as g; g.build()'`")
        handle = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = handle
    return _LIB


def last_error() -> str:
    msg = lib().hspmv_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise HspmvError(what, rc, last_error())
