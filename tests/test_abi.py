"""The C-ABI library loads and exports every entry point include/hspmv.h
declares (no compute calls: this runs without a GPU)."""
import ctypes
import re
import subprocess

import pytest

import hspmv
from hspmv import _lib


def declared_symbols():
    text = _lib.HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hspmv_[a-z0-9_]+)\s*\(", text)))


def test_header_declarations_are_all_bound():
    syms = declared_symbols()
    assert len(syms) >= 29
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    L = hspmv.lib()
    for s in declared_symbols():
        assert getattr(L, s) is not None
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (hspmv_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_library_links_hip_runtime_and_rccl():
    out = subprocess.run(["readelf", "-d", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    assert "libamdhip64.so" in out and "librccl.so" in out
    # the kernels are compiled for gfx950
    blob = _lib.LIB_PATH.read_bytes()
    assert b"gfx950" in blob


def test_version_and_error_state():
    assert "gfx950" in hspmv.version()
    with pytest.raises(hspmv.HspmvError):
        hspmv.read_csr("/does/not/exist.csr")
    assert "cannot open" in _lib.last_error()


def test_create_without_arguments_is_an_error_not_a_crash():
    L = hspmv.lib()
    assert L.hspmv_create(None, None, None, 1, 0) == -1
    h = ctypes.c_void_p()
    rc = L.hspmv_create(ctypes.byref(h), None, None, 1, 0)
    assert rc < 0 and not h.value
    assert L.hspmv_spmv(None) == -1
    L.hspmv_destroy(None)


def test_no_torch_or_oracle_symbols_in_product():
    out = subprocess.run(["nm", "-D", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    assert "orc_" not in out and "torch" not in out


def test_struct_layouts_match_the_header(tmp_path):
    """The ctypes mirrors (hspmv/_lib.py) have the header's sizes and field
    offsets: a mismatch makes hspmv_get_info / hspmv_run write past the
    caller's struct (a C program built against an older header crashes the
    same way -- rebuild the tools after a header change)."""
    structs = {"hspmv_info": _lib.Info, "hspmv_timing": _lib.Timing, "hspmv_options": _lib.Options}
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "hspmv.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(_lib.HEADER.parent), str(src), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        cname, what, val = line.split()
        got[(cname, what)] = int(val)
    for cname, py in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_rccl_version_is_the_resolved_librccl():
    """hspmv_rccl_version (and hspmv_info.rccl_version on every handle)
    report ncclGetVersion() of the RCCL this process resolved: librccl.so.1
    is one SONAME for the ROCm and the PyTorch copy, so the first one
    loaded serves both."""
    v = ctypes.c_int()
    assert hspmv.lib().hspmv_rccl_version(ctypes.byref(v)) == 0
    assert v.value >= 21800  # RCCL 2.18 or newer: MAJOR*10000 + MINOR*100 + PATCH
    assert hspmv.lib().hspmv_rccl_version(None) == -1
    assert "rccl_version" in dict(_lib.Info._fields_)


def test_get_info_fills_only_the_0_1_layout():
    """hspmv_get_info never writes past the 0.1 struct (fields before
    `deterministic`), so an old caller cannot be overrun; the newer fields
    come from hspmv_get_info_sized.  Checked on the header offsets."""
    text = _lib.HEADER.read_text()
    assert "#define HSPMV_VERSION_MINOR 3" in text
    assert _lib.Info.deterministic.offset < ctypes.sizeof(_lib.Info)
    assert _lib.Info.rccl_version.offset > _lib.Info.csort_row_blocks.offset
