// bw_probe.hip -- calibration microbenchmark (not product code): achievable
// HBM read bandwidth on this MI355X for the access shapes the SpMV kernels
// use, so roofline fractions can be read against a measured ceiling as well
// as the 8 TB/s spec.
//
//   hipcc -O3 --offload-arch=gfx950 bw_probe.hip -o bw_probe && ./bw_probe
//
// Shapes (each reads >= 1 GiB, far beyond the 256 MiB Infinity Cache):
//   x4   : float4 (dwordx4, 16 B/lane) grid-stride sum, R loads in flight
//   csr  : int32 + double streams read like the SpMV (dword + dwordx2 per lane,
//          U elements per lane per step), the STREAM kernel's col/val pattern
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                        \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

template <int R>
__global__ __launch_bounds__(256) void read_x4(const float4 *__restrict__ a, size_t n4,
                                               float *__restrict__ out) {
  float s = 0.f;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (R - 1) * stride < n4; i += R * stride) {
    float4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = a[i + r * stride];
#pragma unroll
    for (int r = 0; r < R; ++r) s += v[r].x + v[r].y + v[r].z + v[r].w;
  }
  for (; i < n4; i += stride) {
    float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.678f) out[0] = s;  // keep the loads alive
}

template <int U>
__global__ __launch_bounds__(256) void read_csr(const int *__restrict__ col,
                                                const double *__restrict__ val, size_t nnz,
                                                double *__restrict__ out) {
  double s = 0.0;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  const int lane = threadIdx.x & 63;
  for (size_t c = wave * 64 * U; c < nnz; c += nwaves * 64 * U) {
    int cv[U];
    double vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t j = std::min(c + u * 64 + lane, nnz - 1);
      cv[u] = col[j];
      vv[u] = val[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s += vv[u] * (double)cv[u];
  }
  if (s == 12345.678) out[0] = s;
}

template <typename F>
float time_ms(F launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  std::vector<float> t;
  for (int r = 0; r < reps + 3; ++r) {
    (void)hipEventRecord(a);
    launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r >= 3) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[0];
}

int main() {
  const size_t bytes = (size_t)2 << 30;  // 2 GiB
  float4 *a;
  float *out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, bytes));
  const size_t n4 = bytes / 16;
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  printf("{\"cus\": %d}\n", cus);
  for (int bpc : {4, 8, 16, 32}) {
    const int grid = cus * bpc;
    float ms1 = time_ms([&] { hipLaunchKernelGGL(read_x4<1>, dim3(grid), dim3(256), 0, 0, a, n4, out); }, 10);
    float ms4 = time_ms([&] { hipLaunchKernelGGL(read_x4<4>, dim3(grid), dim3(256), 0, 0, a, n4, out); }, 10);
    float ms8 = time_ms([&] { hipLaunchKernelGGL(read_x4<8>, dim3(grid), dim3(256), 0, 0, a, n4, out); }, 10);
    printf("{\"shape\": \"x4\", \"blocks_per_cu\": %d, \"R1_GBps\": %.1f, \"R4_GBps\": %.1f, \"R8_GBps\": %.1f}\n",
           bpc, bytes / ms1 * 1e-6, bytes / ms4 * 1e-6, bytes / ms8 * 1e-6);
  }
  // csr-shaped: 1.5 GiB of (int32, double) pairs
  const size_t nnz = (size_t)(1.5 * (1 << 30)) / 12;
  int *col;
  double *val;
  CK(hipMalloc(&col, nnz * 4));
  CK(hipMalloc(&val, nnz * 8));
  CK(hipMemset(col, 0, nnz * 4));
  CK(hipMemset(val, 0, nnz * 8));
  double *o2;
  CK(hipMalloc(&o2, 64));
  const double b2 = (double)nnz * 12;
  for (int bpc : {8, 32}) {
    const int grid = cus * bpc;
    float m2 = time_ms([&] { hipLaunchKernelGGL(read_csr<2>, dim3(grid), dim3(256), 0, 0, col, val, nnz, o2); }, 10);
    float m4 = time_ms([&] { hipLaunchKernelGGL(read_csr<4>, dim3(grid), dim3(256), 0, 0, col, val, nnz, o2); }, 10);
    float m8 = time_ms([&] { hipLaunchKernelGGL(read_csr<8>, dim3(grid), dim3(256), 0, 0, col, val, nnz, o2); }, 10);
    float m16 = time_ms([&] { hipLaunchKernelGGL(read_csr<16>, dim3(grid), dim3(256), 0, 0, col, val, nnz, o2); }, 10);
    printf("{\"shape\": \"csr(int32+f64)\", \"blocks_per_cu\": %d, \"U2_GBps\": %.1f, \"U4_GBps\": %.1f, \"U8_GBps\": %.1f, \"U16_GBps\": %.1f}\n",
           bpc, b2 / m2 * 1e-6, b2 / m4 * 1e-6, b2 / m8 * 1e-6, b2 / m16 * 1e-6);
  }
  return 0;
}
