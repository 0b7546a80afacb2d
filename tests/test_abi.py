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


def test_abi_major_is_in_the_soname():
    """ABI 1.0 declares 0.3's incompatible changes (hspmv_xdict_plan's third
    argument, hspmv_get_info's layout) by the major version: the library is
    libhspmv.so.1 and its SONAME says so, so a binary linked against 0.x
    (NEEDED libhspmv.so) does not load it and misread arguments."""
    text = _lib.HEADER.read_text()
    assert "#define HSPMV_VERSION_MAJOR 1" in text and "#define HSPMV_VERSION_MINOR 1" in text
    assert _lib.LIB_PATH.name == "libhspmv.so.1"
    out = subprocess.run(["readelf", "-d", str(_lib.LIB_PATH)], capture_output=True, text=True)
    assert out.returncode == 0 and "Library soname: [libhspmv.so.1]" in out.stdout
    assert hspmv.version().startswith("hspmv 1.1")
    cli = _lib.PKG_ROOT / "build" / "spmv-csr"
    out = subprocess.run(["readelf", "-d", str(cli)], capture_output=True, text=True)
    assert "Shared library: [libhspmv.so.1]" in out.stdout


def test_old_major_binary_does_not_resolve_the_library(tmp_path):
    """A binary with NEEDED libhspmv.so (what linking against a 0.x library
    gave) and the CLIs' search path (rpath = build/) finds no library: the
    link-time symlink lives in build/dev/, off every runtime path, and
    build/ holds only libhspmv.so.1."""
    build = _lib.LIB_PATH.parent
    assert not (build / "libhspmv.so").exists()
    dev = build / "dev" / "libhspmv.so"
    assert dev.is_symlink() and dev.resolve() == _lib.LIB_PATH.resolve()
    # a stand-in 0.x library: no SONAME, so NEEDED records libhspmv.so
    old = tmp_path / "old"
    old.mkdir()
    (tmp_path / "stub.c").write_text("int hspmv_version_stub(void) { return 0; }\n")
    subprocess.run(["gcc", "-shared", "-fPIC", str(tmp_path / "stub.c"), "-o", str(old / "libhspmv.so")],
                   check=True)
    (tmp_path / "main.c").write_text("int hspmv_version_stub(void);\n"
                                     "int main(void) { return hspmv_version_stub(); }\n")
    exe = tmp_path / "old_cli"
    subprocess.run(["gcc", str(tmp_path / "main.c"), "-o", str(exe), "-L", str(old), "-lhspmv",
                    f"-Wl,-rpath,{build}", "-Wl,--disable-new-dtags"], check=True)
    needed = subprocess.run(["readelf", "-d", str(exe)], capture_output=True, text=True).stdout
    assert "Shared library: [libhspmv.so]" in needed
    env = {k: v for k, v in __import__("os").environ.items() if k != "LD_LIBRARY_PATH"}
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env)
    assert r.returncode != 0 and "libhspmv.so" in r.stderr


def test_get_info_writes_the_frozen_1_0_layout():
    """hspmv_get_info writes HSPMV_INFO_SIZE_1_0 bytes in every 1.x library
    (a 1.0 binary's struct is that large); fields added later come only from
    hspmv_get_info_sized.  The constant ends at the last 1.0 field."""
    text = _lib.HEADER.read_text()
    import re as _re
    n = int(_re.search(r"#define HSPMV_INFO_SIZE_1_0 (\d+)", text).group(1))
    assert n == _lib.Info.heavy_group_frac.offset + 8
    assert ctypes.sizeof(_lib.Info) >= n


def test_get_info_rejects_null_without_a_handle():
    """hspmv_get_info / hspmv_get_info_sized with NULL arguments return
    HSPMV_E_INVALID (no GPU: the handle-free paths only; the NULL-output
    case on a live handle is test_get_info_null_output_and_canary)."""
    L = hspmv.lib()
    assert L.hspmv_get_info(None, None) == -1
    assert L.hspmv_get_info_sized(None, None, 16) == -1
    assert L.hspmv_last_error()


@pytest.mark.gpu
def test_get_info_null_output_and_canary():
    """On a live handle: hspmv_get_info(h, NULL) is HSPMV_E_INVALID (it
    used to dereference NULL); hspmv_get_info_sized with the 0.1-sized
    prefix writes exactly that many bytes -- a canary after it survives --
    and agrees with the full report on those bytes."""
    from hspmv import gen
    L = hspmv.lib()
    A = gen.laplace2d(30, 20)
    with hspmv.SpMV(A, device=0) as op:
        h = op._h
        assert L.hspmv_get_info(h, None) == -1 and b"NULL" in L.hspmv_last_error()
        full = _lib.Info()
        assert L.hspmv_get_info(h, ctypes.byref(full)) == 0 and full.num_gpus == 1
        n01 = _lib.Info.deterministic.offset
        buf = (ctypes.c_ubyte * (ctypes.sizeof(_lib.Info) + 64))()
        for i in range(len(buf)):
            buf[i] = 0xA5
        assert L.hspmv_get_info_sized(h, ctypes.cast(buf, ctypes.POINTER(_lib.Info)), n01) == 0
        assert all(buf[i] == 0xA5 for i in range(n01, len(buf)))
        assert bytes(buf[:n01]) == bytes(memoryview(full).cast("B")[:n01])
        # hspmv_get_info: exactly the frozen 1.0 size, whatever sizeof(hspmv_info) is
        n10 = _lib.Info.heavy_group_frac.offset + 8
        for i in range(len(buf)):
            buf[i] = 0xA5
        assert L.hspmv_get_info(h, ctypes.cast(buf, ctypes.POINTER(_lib.Info))) == 0
        assert all(buf[i] == 0xA5 for i in range(n10, len(buf)))
        assert bytes(buf[:n10]) == bytes(memoryview(full).cast("B")[:n10])


def test_options_deterministic_values_are_validated_before_any_device():
    """hspmv_options.deterministic: 0, 1 (ordered), 2 (reproducible), 3
    (serial); other values, an explicit column-sorted kernel with 1 or 3 and
    an explicit vector kernel with 3 are refused (HSPMV_E_INVALID) before any
    device is touched; 2 with the column-sorted kernel passes that check."""
    import numpy as np
    from hspmv import gen
    L = hspmv.lib()
    A = gen.laplace2d(8, 8)
    cs = A.c_struct()
    h = ctypes.c_void_p()
    for det, kern, ok in ((4, 0, False), (-1, 0, False), (1, 4, False), (3, 4, False), (3, 1, False),
                          (2, 4, True), (1, 0, True), (3, 0, True), (3, 2, True), (3, 3, True)):
        o = _lib.make_options(kern, {"deterministic": det} if det >= 0 else None)
        if det < 0:
            o.deterministic = det
        rc = L.hspmv_create_ex(ctypes.byref(h), ctypes.byref(cs), None, ctypes.byref(o))
        if ok:
            assert rc != -1 or b"deterministic" not in L.hspmv_last_error(), (det, kern)
        else:
            assert rc == -1, (det, kern)
        if rc == 0:
            L.hspmv_destroy(h)
    assert _lib.make_options(0, {"deterministic": "reproducible"}).deterministic == 2
    assert _lib.make_options(0, {"deterministic": "ordered"}).deterministic == 1
    assert _lib.make_options(0, {"deterministic": "serial"}).deterministic == 3


def test_deterministic_names_match_the_header():
    """hspmv._lib.DETERMINISTIC (the names the Python layer and tests use)
    carries the header's HSPMV_DETERMINISTIC_* values."""
    import re as _re
    text = _lib.HEADER.read_text()
    vals = {k.lower(): int(v) for k, v in _re.findall(r"#define HSPMV_DETERMINISTIC_(\w+) (\d+)", text)}
    assert vals == {"ordered": 1, "reproducible": 2, "serial": 3}
    for name, v in vals.items():
        assert _lib.DETERMINISTIC[name] == v
