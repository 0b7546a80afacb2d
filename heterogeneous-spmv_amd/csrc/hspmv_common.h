// Host-side helpers shared by the host runtime units (hspmv_runtime.h) and
// the I/O units (hspmv_io.cpp, hspmv_mtx.cpp, hspmv_bandk.cpp).
#pragma once
#include <stdarg.h>
#include <stdint.h>

#include <string>

#include "hspmv.h"

namespace hspmv {

// Sets the thread-local message returned by hspmv_last_error(); returns code.
int set_error(int code, const char *fmt, ...);
void clear_error();

// Structural validation of a host CSR (row_ptr monotone from 0 to nnz,
// columns in [0, n)).  Returns HSPMV_OK or HSPMV_E_INVALID with a message.
int validate_host_csr(const hspmv_csr *A, bool check_cols);
int validate_host_maps(const hspmv_csr3_maps *maps, int64_t m);

inline size_t dtype_size(int dtype) { return dtype == HSPMV_F64 ? 8 : 4; }

}  // namespace hspmv
