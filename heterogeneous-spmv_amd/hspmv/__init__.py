"""hspmv -- host-side Python mirror of the MI355X-native CSR / CSR-3 SpMV
library (libhspmv.so, C ABI in include/hspmv.h).

Import with ``sys.path.insert(0, "<repo>/heterogeneous-spmv_amd")`` (the package
directory name carries a hyphen, so it is not itself importable).
"""
from ._lib import HspmvError, LIB_PATH, lib  # noqa: F401
from .api import (Csr3Maps, CsrMatrix, SpMV, alg_bytes, build_csr2_bandk, build_csr2_maps,  # noqa: F401
                  build_csr3_bandk, build_csr3_maps,
                  csr3_params, device_count, load_bin, partition_rows, rcm_reorder, read_csr,
                  read_csr3, read_mtx, save_bin, version, write_csr, write_csr3, xdict_plan)

__all__ = ["HspmvError", "LIB_PATH", "lib", "Csr3Maps", "CsrMatrix", "SpMV", "alg_bytes",
           "build_csr2_bandk", "build_csr2_maps", "build_csr3_bandk", "build_csr3_maps", "csr3_params", "device_count", "load_bin", "partition_rows",
           "rcm_reorder", "read_csr", "read_csr3", "read_mtx", "save_bin", "version", "write_csr", "write_csr3", "xdict_plan"]
