// stream_f64.hip -- instantiates the STREAM / CSR3 row kernels for double
// (split from spmv_kernels.hip so hipcc compiles the dtypes in parallel).
#include "spmv_device.cuh"

namespace hspmv {
hipError_t launch_rows_f64(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const double *x,
                          double *y, hipStream_t st) {
  return dev::launch_rows<double>(A, dp, p, x, y, st);
}
}  // namespace hspmv
