// td_probe.hip -- calibration microbenchmark (not product code): does a
// direct-to-LDS load (global_load_lds) move L2-resident data through a CU
// faster than register loads and gathers do?  The column-sorted C5 kernel
// (csrc/csort.hip) is bound by the L1's texture-data return (TD_TD_BUSY 82 %,
// one access per (quad, 32-byte sector), profiles/r03/c5_csort_stall_counters);
// its x gathers are ~34.5 M of the 46.5 M accesses.  If an LDS-DMA sweep of
// the same x half costs fewer TD cycles per byte, x can be staged into LDS in
// windows and gathered from there.
//
// Shape = C5's: 256 workgroups x 1024 threads (one per CU), workgroup b reads
// half b % 2 (4 MiB of fp32) of an 8 MiB x; every half is read by 128
// workgroups, so it is an L2 (per XCD) / MALL hit after the first touch.
// Modes:
//   ld4      : coalesced global_load_dword (256 B per wave instruction)
//   ld16     : coalesced global_load_dwordx4 (1 KiB per wave instruction)
//   glds4    : global_load_lds_dword into a per-wave LDS ring (256 B / instr)
//   glds16   : global_load_lds_dwordx4 into the ring (1 KiB / instr)
//   gather   : C5-like sorted gathers: 187.5 K fp32 entries per workgroup at
//              1.5 entries per 32-byte sector, 8 per lane per chunk
//   glds16+lg: glds16 into a 16 KiB per-workgroup window, then the same
//              gathers as `gather` served from LDS (the staged design)
//   win      : the same entries as `gather`, but per 64-entry instruction the
//              x span it covers is loaded coalesced (16 B per lane, lanes past
//              the span masked) into a 2 KiB per-wave LDS window and the lanes
//              read their entries from there (fewer, wider L1 accesses)
// Reported: ms (min of 10), GB/s of the 1 GiB read (x halves x 128
// workgroups), and for the gathers ns per workgroup entry.
//
//   hipcc -O3 --offload-arch=gfx950 td_probe.hip -o td_probe && ./td_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      return 1;                                                             \
    }                                                                       \
  } while (0)

constexpr int kThreads = 1024, kWaves = 16, kBlocks = 256;
constexpr long kHalf = 1L << 20;  // fp32 entries per half (4 MiB)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glb_void;

enum { LD4 = 0, LD16 = 1, GLDS4 = 2, GLDS16 = 3, GATHER = 4, GLDS_GATHER = 5, WIN_GATHER = 6 };

// entries of a workgroup: e = 0 .. kEnt-1 at column (e * 16) / 3 of its half
constexpr long kEnt = kHalf * 3 / 16;

template <int MODE>
__global__ __launch_bounds__(kThreads) void probe(const float *__restrict__ x, float *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x, wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float *xh = x + (long)(b & 1) * kHalf;
  float acc = 0.f;
  if constexpr (MODE == LD4) {
    // wave w reads 256-B pieces w, w + 16, ...; 8 in flight
    for (long i = (long)wid * 64 * 8; i < kHalf; i += (long)kWaves * 64 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xh[i + u * 64 + lane];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
  } else if constexpr (MODE == LD16) {
    const f32x4 *p = reinterpret_cast<const f32x4 *>(xh);
    for (long i = (long)wid * 64 * 4; i < kHalf / 4; i += (long)kWaves * 64 * 4) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = p[i + u * 64 + lane];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
  } else if constexpr (MODE == GLDS4 || MODE == GLDS16) {
    constexpr int SZ = MODE == GLDS4 ? 4 : 16;
    constexpr int PER = 64 * SZ / 4;  // floats per wave instruction
    float *ring = smem + wid * 8 * PER;  // 8 instructions per batch
    for (long i = (long)wid * PER * 8; i < kHalf; i += (long)kWaves * PER * 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if constexpr (SZ == 4)
          __builtin_amdgcn_global_load_lds((glb_void *)(xh + i + u * PER + lane),
                                           (lds_void *)(ring + u * PER), 4, 0, 0);
        else
          __builtin_amdgcn_global_load_lds((glb_void *)(xh + i + u * PER + lane * 4),
                                           (lds_void *)(ring + u * PER), 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    acc = ring[lane];
  } else if constexpr (MODE == GATHER) {
    // chunks of 64 x 8 entries, wave w takes chunks w, w + 16, ...
    for (long c = wid; c * 512 < kEnt; c += kWaves) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long e = std::min(c * 512 + u * 64 + lane, kEnt - 1);
        v[u] = xh[(e * 16) / 3];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
  } else if constexpr (MODE == WIN_GATHER) {
    float *win = smem + wid * 512;  // 2 KiB per wave
    const f32x4 *p4 = reinterpret_cast<const f32x4 *>(xh);
    for (long c = wid; c * 512 < kEnt; c += kWaves) {
      f32x4 w0[8], w1[8];
      int32_t base[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long e0 = std::min(c * 512 + u * 64, kEnt - 1), e1 = std::min(e0 + 63, kEnt - 1);
        base[u] = (int32_t)(((e0 * 16) / 3) & ~3L);
        const int32_t nq = (int32_t)((((e1 * 16) / 3) - base[u]) / 4 + 1);  // <= 128
        w0[u] = lane < nq ? p4[base[u] / 4 + lane] : f32x4{0, 0, 0, 0};
        w1[u] = lane + 64 < nq ? p4[base[u] / 4 + 64 + lane] : f32x4{0, 0, 0, 0};
      }
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        *reinterpret_cast<f32x4 *>(win + lane * 4) = w0[u];
        *reinterpret_cast<f32x4 *>(win + 256 + lane * 4) = w1[u];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const long e = std::min(c * 512 + u * 64 + lane, kEnt - 1);
        v[u] = win[(int32_t)((e * 16) / 3) - base[u]];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
  } else {  // GLDS_GATHER: 16 KiB windows (4096 entries of x), two of them
    constexpr long W = 4096;
    float *win = smem;
    const long nwin = kHalf / W;
    // window k holds x[k*W, (k+1)*W): 16 KiB = one glds16 per wave
    for (long k = 0; k < nwin; ++k) {
      float *wb = win + (k & 1) * W;
      __builtin_amdgcn_global_load_lds((glb_void *)(xh + k * W + wid * 256 + lane * 4),
                                       (lds_void *)(wb + wid * 256), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      // entries whose columns fall in the window: e in [ceil(kW*3/16), ...)
      const long e0 = (k * W * 3 + 15) / 16, e1 = std::min(((k + 1) * W * 3 + 15) / 16, kEnt);
      for (long e = e0 + threadIdx.x; e < e1; e += kThreads) acc += wb[(e * 16) / 3 - k * W];
    }
  }
  if (acc == 123.456f) out[b * kThreads + threadIdx.x] = acc;  // keep it live
}

template <int MODE>
float run(const float *x, float *out, hipStream_t st, int lds) {
  hipEvent_t a, z;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&z);
  float best = 1e30f;
  for (int it = 0; it < 12; ++it) {
    (void)hipEventRecord(a, st);
    hipLaunchKernelGGL((probe<MODE>), dim3(kBlocks), dim3(kThreads), lds, st, x, out);
    (void)hipEventRecord(z, st);
    (void)hipEventSynchronize(z);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, z);
    if (it >= 2) best = std::min(best, ms);
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(z);
  return best;
}

int main() {
  float *x, *out;
  CK(hipMalloc(&x, 2 * kHalf * sizeof(float)));
  CK(hipMalloc(&out, kBlocks * kThreads * sizeof(float)));
  std::vector<float> h(2 * kHalf, 1.0f);
  CK(hipMemcpy(x, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  // LDS: 128 KiB everywhere (one workgroup per CU, as csort)
  const int lds = 128 * 1024;
  CK(hipFuncSetAttribute((const void *)probe<LD4>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void *)probe<LD16>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void *)probe<GLDS4>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void *)probe<GLDS16>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void *)probe<GATHER>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void *)probe<GLDS_GATHER>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void *)probe<WIN_GATHER>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const double bytes = (double)kBlocks * kHalf * 4;
  const char *names[] = {"ld4", "ld16", "glds4", "glds16", "gather", "glds16+lg", "win"};
  float ms[7];
  ms[0] = run<LD4>(x, out, st, lds);
  ms[1] = run<LD16>(x, out, st, lds);
  ms[2] = run<GLDS4>(x, out, st, lds);
  ms[3] = run<GLDS16>(x, out, st, lds);
  ms[4] = run<GATHER>(x, out, st, lds);
  ms[5] = run<GLDS_GATHER>(x, out, st, lds);
  ms[6] = run<WIN_GATHER>(x, out, st, lds);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  for (int i = 0; i < 7; ++i)
    printf("{\"probe\": \"td\", \"mode\": \"%s\", \"ms\": %.4f, \"x_GBps\": %.1f, \"ns_per_wg_entry\": %.4f}\n",
           names[i], ms[i], bytes / (ms[i] * 1e-3) / 1e9, ms[i] * 1e6 / kEnt);
  return 0;
}
