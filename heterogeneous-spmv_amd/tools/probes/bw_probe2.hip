// bw_probe2.hip -- calibration microbenchmark (not product code): the STREAM
// kernel's col/val read shape without the row logic, to separate what the
// load shape costs from what the SpMV adds.  One wave per contiguous segment
// of SEG nonzeros (SEG = 64 rows x nnz/row: 640 ~ C4, 1728 ~ C3), four waves
// per 256-thread block, no grid stride (one segment per wave, like the
// kernel).  Within a segment the wave reads chunks of 64*U elements:
//   narrow: lane-strided dword col + dwordx2 val loads (the kernel today)
//   wide  : each lane reads 4 consecutive elements (dwordx4 col, 2x dwordx4
//           val), U/4 groups per chunk -- same bytes, 4x fewer instructions
// remap = XCD-contiguous block order vs dispatch order.
//
//   hipcc -O3 --offload-arch=gfx950 bw_probe2.hip -o bw_probe2 && ./bw_probe2
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                        \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

__device__ __forceinline__ long remap_blk(long b, long nb) {
  const long q = nb / 8, r = nb % 8, x = b % 8, i = b / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

template <int U, bool WIDE>
__global__ __launch_bounds__(256) void seg_read(const int *__restrict__ col,
                                                const double *__restrict__ val, long nnz, int seg,
                                                int remap, double *__restrict__ out) {
  const long blk = remap ? remap_blk(blockIdx.x, gridDim.x) : (long)blockIdx.x;
  const long w = blk * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long s0 = w * seg;
  if (s0 >= nnz) return;
  const long s1 = std::min(s0 + seg, nnz);
  double s = 0.0;
  for (long c = s0; c < s1; c += 64 * U) {
    if constexpr (WIDE) {
      constexpr int Q = U / 4;
      int4 cv[Q];
      double2 va[Q], vb[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const long j = std::min(c + q * 256 + lane * 4, nnz - 4) & ~3L;
        cv[q] = *(const int4 *)(col + j);
        va[q] = *(const double2 *)(val + j);
        vb[q] = *(const double2 *)(val + j + 2);
      }
#pragma unroll
      for (int q = 0; q < Q; ++q)
        s += va[q].x * cv[q].x + va[q].y * cv[q].y + vb[q].x * cv[q].z + vb[q].y * cv[q].w;
    } else {
      int cv[U];
      double vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long j = std::min(c + u * 64 + lane, nnz - 1);
        cv[u] = col[j];
        vv[u] = val[j];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) s += vv[u] * (double)cv[u];
    }
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

int main(int argc, char **argv) {
  // optional: bw_probe2 SEG REMAP -- one configuration (for counter passes)
  const int only_seg = argc > 1 ? atoi(argv[1]) : 0;
  const int only_remap = argc > 2 ? atoi(argv[2]) : -1;
  // 50M nonzeros = 600 MB of col+val (C3-sized), far beyond the 256 MiB MALL
  const long nnz = 50L << 20;
  int *col;
  double *val, *out;
  CK(hipMalloc(&col, nnz * 4));
  CK(hipMalloc(&val, nnz * 8));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(col, 0, nnz * 4));
  CK(hipMemset(val, 0, nnz * 8));
  const double bytes = (double)nnz * 12;
  for (int seg : {640, 1728, 4096}) {
    if (only_seg && seg != only_seg) continue;
    const long waves = (nnz + seg - 1) / seg;
    const unsigned grid = (unsigned)((waves + 3) / 4);
    for (int remap : {0, 1}) {
      if (only_remap >= 0 && remap != only_remap) continue;
#define RUN(U, W)                                                                              \
  bytes / time_ms([&] { hipLaunchKernelGGL((seg_read<U, W>), dim3(grid), dim3(256), 0, 0, col, \
                                           val, nnz, seg, remap, out); }, 10) * 1e-6
      const double n2 = RUN(2, false), n4 = RUN(4, false), n8 = RUN(8, false), n16 = RUN(16, false);
      const double w4 = RUN(4, true), w8 = RUN(8, true), w16 = RUN(16, true);
#undef RUN
      printf("{\"seg\": %d, \"remap\": %d, \"narrow_U2\": %.0f, \"narrow_U4\": %.0f, "
             "\"narrow_U8\": %.0f, \"narrow_U16\": %.0f, \"wide_U4\": %.0f, \"wide_U8\": %.0f, "
             "\"wide_U16\": %.0f}\n",
             seg, remap, n2, n4, n8, n16, w4, w8, w16);
      fflush(stdout);
    }
  }
  CK(hipGetLastError());
  return 0;
}
