// lds_atomic_probe.hip -- throughput of LDS atomic adds on gfx950, the
// operation the column-sorted kernel (csrc/csort.hip) spends its row sums
// on: f32 vs f64 vs u32 vs u64 slots, random slot per lane (as csort's
// column-sorted entries hit random rows of the block), at the slot counts
// csort uses (one 1024-thread workgroup per CU, or two).
//
//   build:  make -C heterogeneous-spmv_amd build/lds_atomic_probe
//   run:    build/lds_atomic_probe            -> one JSON line per case
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t v) {
  v ^= v >> 16;
  v *= 0x7feb352dU;
  v ^= v >> 15;
  v *= 0x846ca68bU;
  v ^= v >> 16;
  return v;
}

// Every thread adds ITER values into random slots of an S-slot LDS array
// (S dynamic), then the block writes its slots out (so nothing is elided).
template <typename T, int ITER, bool SEQ = false>
__global__ __launch_bounds__(1024) void probe(int32_t slots, uint32_t seed, T *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T *acc = reinterpret_cast<T *>(smem);
  for (int i = threadIdx.x; i < slots; i += blockDim.x) acc[i] = T(0);
  __syncthreads();
  uint32_t h = hash32(seed ^ (blockIdx.x * 1024u + threadIdx.x));
#pragma unroll 16
  for (int it = 0; it < ITER; ++it) {
    h = h * 1664525u + 1013904223u;  // LCG: 2 VALU ops
    // SEQ: lane-consecutive slots (no bank conflicts), a random base per
    // wave instruction -- the ceiling a conflict-free arrangement could reach
    const int s = SEQ ? (int)((__builtin_amdgcn_readfirstlane(__umulhi(h, (uint32_t)slots)) +
                               (threadIdx.x & 63)) % (uint32_t)slots)
                      : (int)__umulhi(h, (uint32_t)slots);
    atomicAdd(&acc[s], (T)(h & 7u));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < slots; i += blockDim.x) out[(size_t)blockIdx.x * slots + i] = acc[i];
}

template <typename T, bool SEQ = false>
int run(const char *name, int slots, int blocks, hipEvent_t a, hipEvent_t b) {
  constexpr int ITER = 256;
  T *out = nullptr;
  CHECK(hipMalloc(&out, sizeof(T) * (size_t)slots * blocks));
  const size_t lds = sizeof(T) * (size_t)slots;
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe<T, ITER, SEQ>), dim3(blocks), dim3(1024), lds, 0, slots, 1u, out);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((probe<T, ITER, SEQ>), dim3(blocks), dim3(1024), lds, 0, slots, (uint32_t)r + 7u, out);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double adds = (double)blocks * 1024.0 * ITER;
  printf("{\"type\":\"%s\",\"slots\":%d,\"lds_bytes\":%zu,\"blocks\":%d,\"us\":%.2f,"
         "\"gadds_per_s\":%.1f,\"adds_per_cu_clk\":%.2f}\n",
         name, slots, lds, blocks, best * 1e3, adds / (best * 1e-3) * 1e-9,
         adds / (best * 1e-3) / 256.0 / 2.4e9);
  CHECK(hipFree(out));
  return 0;
}

int main() {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  // csort today: 256 workgroups of ~15.6 K fp64 slots (one per CU); the
  // two-per-CU shapes: 512 workgroups of ~7.8 K fp64 or ~15.6 K fp32 slots
  if (getenv("LDS_PROBE_SEQ")) {  // conflict-free ceilings vs random, csort's shape
    const int s = 16000, g = 256;
    if (run<double>("f64", s, g, a, b) || run<double, true>("f64 seq", s, g, a, b)) return 1;
    if (run<unsigned long long>("u64", s, g, a, b) || run<unsigned long long, true>("u64 seq", s, g, a, b)) return 1;
    if (run<float>("f32", s, g, a, b) || run<float, true>("f32 seq", s, g, a, b)) return 1;
    return 0;
  }
  const int cases[][2] = {{16000, 256}, {7800, 512}, {16000, 512}, {4000, 512}};
  for (auto &c : cases) {
    const int s = c[0], g = c[1];
    if ((size_t)s * 8 <= 160 * 1024 && run<double>("f64", s, g, a, b)) return 1;
    if ((size_t)s * 4 <= 160 * 1024 && run<float>("f32", s, g, a, b)) return 1;
    if ((size_t)s * 8 <= 160 * 1024 && run<unsigned long long>("u64", s, g, a, b)) return 1;
    if ((size_t)s * 4 <= 160 * 1024 && run<unsigned int>("u32", s, g, a, b)) return 1;
  }
  return 0;
}
