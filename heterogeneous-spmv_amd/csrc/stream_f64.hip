// stream_f64.hip -- instantiates the STREAM / CSR3 row kernels for double
// (split from spmv_kernels.hip so hipcc compiles the dtypes in parallel).
#include "spmv_device.cuh"

namespace hspmv {
hipError_t launch_rows_f64(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const double *x,
                          double *y, hipStream_t st) {
  return dev::launch_rows<double>(A, dp, p, x, y, st);
}
}  // namespace hspmv

#if (HSPMV_DIAG & (8 | 512))
// Diagnostic builds only: copies the STREAM fp64 kernel's per-wave phase
// stamps (8) or the CSR3 kernel's per-workgroup timeline (512) (kTraceWaves x kTraceSlots u64) to host memory `dst`.
extern "C" int hspmv_diag_trace(void *dst, size_t bytes) {
  const size_t n = sizeof(unsigned long long) * hspmv::dev::kTraceWaves * hspmv::dev::kTraceSlots;
  if (bytes < n) return -1;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(hspmv::dev::g_trace), n, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? 0
             : -4;
}
extern "C" int hspmv_diag_trace_clear() {
  static unsigned long long zero[1024];
  const size_t n = sizeof(unsigned long long) * hspmv::dev::kTraceWaves * hspmv::dev::kTraceSlots;
  for (size_t off = 0; off < n; off += sizeof(zero))
    if (hipMemcpyToSymbol(HIP_SYMBOL(hspmv::dev::g_trace), zero, sizeof(zero), off,
                          hipMemcpyHostToDevice) != hipSuccess)
      return -4;
  return 0;
}
#endif
