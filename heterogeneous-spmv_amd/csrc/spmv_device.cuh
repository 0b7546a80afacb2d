// spmv_device.cuh -- device building blocks of the row kernels (STREAM and
// CSR3), included by the per-dtype instantiation units stream_f32.hip /
// stream_f64.hip (split so hipcc compiles them in parallel).  The design is
// described in spmv_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "hspmv_internal.h"

namespace hspmv {
namespace dev {

// Ablation builds only (make diag): 1 = skip the ordered row sums, 2 = skip
// the x gather (x[col] := 1), 3 = both.  Results are wrong in those builds.
#ifndef HSPMV_DIAG
#define HSPMV_DIAG 0
#endif

constexpr int kWave = 64;
constexpr int kSerialMax = 32;  // longest row summed serially by one lane
constexpr int kNumXcd = 8;

template <bool NT, typename T>
__device__ __forceinline__ T ldg(const T *p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

// Orders a wave's LDS writes before its other lanes' LDS reads (the
// wave-scope equivalent of a barrier; no s_barrier involved).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks b and b+8 share an XCD under round-robin dispatch, so
// give XCD slot x = b % 8 the contiguous logical range of its q (+1) blocks.
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
  const int64_t q = nb / kNumXcd, r = nb % kNumXcd;
  const int64_t x = b % kNumXcd, i = b / kNumXcd;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

__device__ __forceinline__ unsigned long long bits_from(int i) {
  return i >= 64 ? 0ull : (~0ull << i);
}

// Loads through a wave-uniform GLOBAL (address_space 1) base pointer plus a
// 32-bit byte offset, so hipcc emits global_load ... v_off, s[base:base+1]
// (one offset VGPR per load, no 64-bit address pairs, and no flat_load,
// which would force vmcnt(0) + lgkmcnt(0) waits).
typedef __attribute__((address_space(1))) const char gchar;

template <bool NT, typename T>
__device__ __forceinline__ T ld_off(const gchar *base, uint32_t byte_off) {
  const __attribute__((address_space(1))) T *p =
      (const __attribute__((address_space(1))) T *)(base + byte_off);
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

template <typename T>
__device__ __forceinline__ const gchar *uniform_ptr(const T *p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const gchar *)(((uint64_t)hi << 32) | lo);
}

// Ordered sum of lds[lo..hi) into acc, left to right: the LDS reads are
// issued 4 at a time (one LDS latency per 4 nonzeros instead of per nonzero)
// but the additions stay in sequence, so the rounding is omp_spmv's.
template <typename T>
__device__ __forceinline__ T ordered_sum(T acc, const T *lds, int32_t lo, int32_t hi) {
  int32_t k = lo;
  for (; k + 4 <= hi; k += 4) {
    const T a0 = lds[k], a1 = lds[k + 1], a2 = lds[k + 2], a3 = lds[k + 3];
    acc = acc + a0;
    acc = acc + a1;
    acc = acc + a2;
    acc = acc + a3;
  }
  for (; k < hi; ++k) acc = acc + lds[k];
  return acc;
}

// One wavefront computes rows [g0, g1), g1 - g0 <= 64.  lds: kWave*U
// elements private to this wave.  Per chunk of 64*U nonzeros: stage A loads
// col/val (coalesced), stage B gathers x[col], stage C forms the products
// into LDS; then the row sums.  PF (software pipelining): the next chunk's
// stage A is issued between this chunk's stage B and C, so its latency
// overlaps the gather and the sums.
template <typename T, bool NT, int U, bool PF>
__device__ __forceinline__ void wave_rows(int32_t g0, int32_t g1, int32_t long_t,
                                          const int32_t *__restrict__ rp,
                                          const int32_t *__restrict__ ci,
                                          const T *__restrict__ val,
                                          const T *__restrict__ x,
                                          T *__restrict__ y, T *lds, int lane) {
  const int32_t row = g0 + lane;
  const bool valid = row < g1;
  const int32_t beg = valid ? rp[row] : 0;
  const int32_t end = valid ? rp[row + 1] : 0;
  const int32_t len = end - beg;
  const bool skip = len > long_t;
  const unsigned long long skipmask = __ballot(valid && skip);
  const unsigned long long coopmask = __ballot(valid && !skip && len > kSerialMax);
  const bool serial = valid && !skip && len <= kSerialMax;
  const gchar *xb = uniform_ptr(x);
  T acc = T(0);
  // Runs of consecutive non-split rows [a, b); normally one run = the group.
  int32_t a = g0;
  while (a < g1) {
    const unsigned long long rest = skipmask & bits_from(a - g0);
    const int32_t b = rest ? g0 + (__ffsll(rest) - 1) : g1;
    if (b > a) {
      const int32_t kb = __builtin_amdgcn_readfirstlane(__shfl(beg, a - g0, kWave));
      const int32_t ke = __builtin_amdgcn_readfirstlane(__shfl(end, b - 1 - g0, kWave));
      const int32_t n_run = ke - kb;
      const gchar *cb = uniform_ptr(ci + kb);
      const gchar *vb = uniform_ptr(val + kb);
      const unsigned long long coop = coopmask & bits_from(a - g0) & ~bits_from(b - g0);
      const bool mine = serial && row >= a && row < b;
      int32_t col[U];
      T v[U];
      auto stage_a = [&](int32_t c0, int32_t last) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          // clamp instead of branching: every load issues back to back
          const uint32_t j = (uint32_t)(c0 + min(u * kWave + lane, last));
          col[u] = ld_off<NT, int32_t>(cb, j * 4u);
          v[u] = ld_off<NT, T>(vb, j * (uint32_t)sizeof(T));
        }
      };
      if constexpr (PF) {
        if (n_run > 0) stage_a(0, min(kWave * U, n_run) - 1);
      }
      for (int32_t c0 = 0; c0 < n_run; c0 += kWave * U) {
        const int32_t last = min(kWave * U, n_run - c0) - 1;
        if constexpr (!PF) stage_a(c0, last);
        T xv[U], vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if constexpr ((HSPMV_DIAG & 2) != 0)
            xv[u] = T(col[u] & 1) + T(1);
          else
            xv[u] = ld_off<false, T>(xb, (uint32_t)col[u] * (uint32_t)sizeof(T));
          vv[u] = v[u];
        }
        if constexpr (PF) {
          __builtin_amdgcn_sched_barrier(0);
          const int32_t cn = c0 + kWave * U;
          stage_a(cn < n_run ? cn : n_run - 1, cn < n_run ? min(kWave * U, n_run - cn) - 1 : 0);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) lds[u * kWave + lane] = vv[u] * xv[u];
        wave_sync();
        const int32_t c = kb + c0;
        if constexpr ((HSPMV_DIAG & 1) != 0) {
          if (mine && max(beg, c) < min(end, c + last + 1)) acc += lds[max(beg, c) - c];
        } else {
          if (mine) acc = ordered_sum(acc, lds - c, max(beg, c), min(end, c + last + 1));
        }
        unsigned long long cm = coop;
        while (cm) {
          const int r = __ffsll(cm) - 1;
          cm &= cm - 1;
          const int32_t lo = max(__shfl(beg, r, kWave), c);
          const int32_t hi = min(__shfl(end, r, kWave), c + last + 1);
          if (lo < hi) {  // wave-uniform
            T s = T(0);
            for (int32_t k = lo + lane; k < hi; k += kWave) s += lds[k - c];
            s = wave_sum(s);
            if (lane == r) acc += s;
          }
        }
        wave_sync();
      }
    }
    a = b + 1;
  }
  if (valid && !skip) y[row] = acc;
}

template <typename T, bool NT, int U, bool PF>
__global__ __launch_bounds__(256) void hspmv_csr_stream(
    int32_t m, int32_t long_t, int32_t remap, const int32_t *__restrict__ rp,
    const int32_t *__restrict__ ci, const T *__restrict__ val, const T *__restrict__ x,
    T *__restrict__ y) {
  __shared__ T lds[4 * kWave * U];
  const int wid = threadIdx.x >> 6;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t blk = remap ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int64_t g0 = (blk * 4 + wid) * kWave;
  if (g0 >= m) return;  // wave-uniform; no block barrier in this kernel
  const int32_t g1 = (int32_t)min<int64_t>(g0 + kWave, m);
  wave_rows<T, NT, U, PF>((int32_t)g0, g1, long_t, rp, ci, val, x, y, lds + wid * kWave * U,
                          lane);
}

template <typename T, bool NT, int U, bool PF, int W>
__global__ __launch_bounds__(W * 64) void hspmv_csr3(
    int32_t n_tasks, int32_t long_t, int32_t remap, const int32_t *__restrict__ task_start,
    const int32_t *__restrict__ rp, const int32_t *__restrict__ ci, const T *__restrict__ val,
    const T *__restrict__ x, T *__restrict__ y) {
  __shared__ T lds[W * kWave * U];
  const int wid = threadIdx.x >> 6;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t blk = remap ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int64_t t = blk * W + wid;
  if (t >= n_tasks) return;
  const int32_t r0 = task_start[t];
  const int32_t r1 = task_start[t + 1];
  T *my = lds + wid * kWave * U;
  for (int32_t g0 = r0; g0 < r1; g0 += kWave)
    wave_rows<T, NT, U, PF>(g0, min(g0 + kWave, r1), long_t, rp, ci, val, x, y, my, lane);
}

// ------------------------------------------------------------------ launchers

template <typename T, bool NT, int U, bool PF>
void launch_rows_u(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const T *x, T *y,
                   hipStream_t st) {
  const T *val = static_cast<const T *>(A.val);
  if (p.kernel == kStream) {
    hipLaunchKernelGGL((hspmv_csr_stream<T, NT, U, PF>), dim3((unsigned)p.blocks), dim3(256), 0,
                       st, A.m, dp.long_t, (int32_t)p.xcd_remap, A.row_ptr, A.col_idx, val, x, y);
    return;
  }
#define HSPMV_CSR3(W)                                                                        \
  hipLaunchKernelGGL((hspmv_csr3<T, NT, U, PF, W>), dim3((unsigned)p.blocks), dim3(W * 64), 0, \
                     st, dp.n_tasks, dp.long_t, (int32_t)p.xcd_remap, dp.task_start,          \
                     A.row_ptr, A.col_idx, val, x, y)
  switch (p.waves_per_block) {
    case 1: HSPMV_CSR3(1); break;
    case 2: HSPMV_CSR3(2); break;
    case 4: HSPMV_CSR3(4); break;
    default: HSPMV_CSR3(8); break;
  }
#undef HSPMV_CSR3
}

template <typename T, bool NT, bool PF>
hipError_t launch_rows_pf(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const T *x,
                          T *y, hipStream_t st) {
  switch (p.u) {
    case 2: launch_rows_u<T, NT, 2, PF>(A, dp, p, x, y, st); break;
    case 3: launch_rows_u<T, NT, 3, PF>(A, dp, p, x, y, st); break;
    case 4: launch_rows_u<T, NT, 4, PF>(A, dp, p, x, y, st); break;
    case 6: launch_rows_u<T, NT, 6, PF>(A, dp, p, x, y, st); break;
    case 8: launch_rows_u<T, NT, 8, PF>(A, dp, p, x, y, st); break;
    case 16: launch_rows_u<T, NT, 16, PF>(A, dp, p, x, y, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_rows(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const T *x, T *y,
                       hipStream_t st) {
  if (p.nontemporal)
    return p.prefetch ? launch_rows_pf<T, true, true>(A, dp, p, x, y, st)
                      : launch_rows_pf<T, true, false>(A, dp, p, x, y, st);
  return p.prefetch ? launch_rows_pf<T, false, true>(A, dp, p, x, y, st)
                    : launch_rows_pf<T, false, false>(A, dp, p, x, y, st);
}

}  // namespace dev
}  // namespace hspmv
