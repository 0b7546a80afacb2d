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
