// stream_f32.hip -- instantiates the STREAM / CSR3 row kernels for float
// (split from spmv_kernels.hip so hipcc compiles the dtypes in parallel).
#include "spmv_device.cuh"

namespace hspmv {
hipError_t launch_rows_f32(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const float *x,
                          float *y, hipStream_t st) {
  return dev::launch_rows<float>(A, dp, p, x, y, st);
}
}  // namespace hspmv
