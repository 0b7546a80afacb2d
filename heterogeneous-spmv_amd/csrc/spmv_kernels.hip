// spmv_kernels.hip -- hand-written CDNA4 (gfx950) SpMV kernels.
//
// The hot path of the reference is the row-wise nonzero dot product
//   y[r] = sum_{k=rp[r]}^{rp[r+1]-1} val[k] * x[col[k]]
// (spmv-csr/spmv.c:92-114; GPU forms cuda-spmv-csr/spmv.cu:117-182 and
// cuda-spmv-csrk/hip/csrk.cu:185-390).  It is an HBM-bound gather: 2 flops per
// 12 B (fp64) / 8 B (fp32) of matrix stream, so no MFMA anywhere here.
//
// Three kernels, all wave64-native:
//
//  * hspmv_csr_vector<T, L>  (HSPMV_KERNEL_VECTOR)
//      L lanes (a sub-wave, L | 64) per row, lanes stride the row's nonzeros
//      with coalesced val/col loads and FMA, reduced by __shfl_xor inside the
//      L-lane group.  Replaces cuda_spmv (thread per row, L = 1) and
//      cuSpMV_3_vec's veclevel lanes + barrier-free volatile-LDS tree
//      (csrk.cu:222-240) with a wave64-safe shuffle reduction.
//
//  * hspmv_csr_stream<T>     (HSPMV_KERNEL_STREAM)
//      one wavefront per group of 64 consecutive rows.  The group's nonzeros
//      are contiguous, so the wave streams them with fully coalesced loads
//      (U elements per lane per chunk), forms the products val*x[col] and
//      stages them in a per-wave LDS slice; then lane i sums row i's products
//      left to right.  The summation order and rounding (product rounded,
//      then sum rounded, starting from 0) are exactly those of omp_spmv, so
//      the result is BIT-IDENTICAL to the CPU reference.  Groups holding a
//      row longer than kSerialMax switch to a mixed path: short rows summed in
//      order straight from global memory (still bit-exact), long rows by the
//      whole wave (FMA + shuffle tree: within the 1e-6 fp64 tolerance).
//
//  * hspmv_csr3<T, W>        (HSPMV_KERNEL_CSR3)
//      CSR-3: one workgroup of W waves per super-super-row (outer map);
//      the workgroup's super-rows (inner map) are split between its waves by
//      binary search on rp[inner[s]] so every wave gets ~1/W of the
//      workgroup's nonzeros; each wave then runs the stream routine over its
//      contiguous row range.  Replaces cuSpMV_3 / cuSpMV_3_vec (thread/
//      sub-warp per row inside (8,12)-thread blocks, csrk.cu:185-319) and
//      cuSpMV_2 (degenerate outer level).
//
// Build: hipcc --offload-arch=gfx950 -ffp-contract=off.  Contraction is off so
// that only the explicit fma() calls (vector kernel, long rows) fuse.
#include <hip/hip_runtime.h>

#include "hspmv_internal.h"

namespace hspmv {
namespace {

constexpr int kWave = 64;
constexpr int kSerialMax = 32;  // longest row summed serially by one lane
constexpr int kStreamU = 8;     // elements per lane per LDS chunk

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

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, kWave));
  return v;
}

// One wavefront computes rows [g0, g1), g1 - g0 <= 64.  lds: kWave*U
// elements private to this wave.  See the file header for the algorithm.
template <typename T, bool NT, int U>
__device__ __forceinline__ void wave_rows(int32_t g0, int32_t g1,
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
  const int32_t kb = __shfl(beg, 0, kWave);
  const int32_t ke = __shfl(end, g1 - g0 - 1, kWave);
  const int32_t maxlen = wave_max(len);
  T acc = T(0);
  if (maxlen <= kSerialMax) {
    // Ordered path: coalesced stream of the group's nonzeros through LDS.
    for (int32_t c = kb; c < ke; c += kWave * U) {
      const int32_t last = min(kWave * U, ke - c) - 1;
      T prod[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // Clamp instead of branching so every load issues back to back
        // (a per-element predicate makes hipcc wait vmcnt(0) per element).
        const int32_t j = min(u * kWave + lane, last);
        const int32_t col = ldg<NT>(ci + c + j);
        prod[u] = ldg<NT>(val + c + j) * x[col];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) lds[u * kWave + lane] = prod[u];
      wave_sync();
      const int32_t lo = max(beg, c);
      const int32_t hi = min(end, c + last + 1);
      for (int32_t k = lo; k < hi; ++k) acc = acc + lds[k - c];
      wave_sync();
    }
  } else {
    // Mixed path: short rows in order from global memory, long rows by the
    // whole wave.
    if (len <= kSerialMax) {
      for (int32_t k = beg; k < end; ++k)
        acc = acc + ldg<NT>(val + k) * x[ldg<NT>(ci + k)];
    }
    unsigned long long longmask = __ballot(valid && len > kSerialMax);
    while (longmask) {
      const int r = __ffsll(longmask) - 1;
      longmask &= longmask - 1;
      const int32_t rb = __shfl(beg, r, kWave);
      const int32_t re = __shfl(end, r, kWave);
      T s0 = T(0), s1 = T(0);
      int32_t k = rb + lane;
      for (; k + kWave < re; k += 2 * kWave) {
        s0 = fma(ldg<NT>(val + k), x[ldg<NT>(ci + k)], s0);
        s1 = fma(ldg<NT>(val + k + kWave), x[ldg<NT>(ci + k + kWave)], s1);
      }
      if (k < re) s0 = fma(ldg<NT>(val + k), x[ldg<NT>(ci + k)], s0);
      const T s = wave_sum(s0 + s1);
      if (lane == r) acc = s;
    }
  }
  if (valid) y[row] = acc;
}

// ------------------------------------------------------------------ kernels

template <typename T, int L, bool NT>
__global__ __launch_bounds__(256) void hspmv_csr_vector(
    int32_t m, const int32_t *__restrict__ rp, const int32_t *__restrict__ ci,
    const T *__restrict__ val, const T *__restrict__ x, T *__restrict__ y) {
  const int lane = threadIdx.x & (L - 1);
  int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / L;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x / L;
  for (; row < m; row += stride) {
    const int32_t beg = rp[row];
    const int32_t end = rp[row + 1];
    T s = T(0);
    for (int32_t k = beg + lane; k < end; k += L)
      s = fma(ldg<NT>(val + k), x[ldg<NT>(ci + k)], s);
#pragma unroll
    for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
    if (lane == 0) y[row] = s;
  }
}

template <typename T, bool NT, int U>
__global__ __launch_bounds__(256) void hspmv_csr_stream(
    int32_t m, const int32_t *__restrict__ rp, const int32_t *__restrict__ ci,
    const T *__restrict__ val, const T *__restrict__ x, T *__restrict__ y) {
  __shared__ T lds[4 * kWave * U];
  const int wid = threadIdx.x >> 6;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t g0 = ((int64_t)blockIdx.x * 4 + wid) * kWave;
  if (g0 >= m) return;  // wave-uniform; no block barrier in this kernel
  const int32_t g1 = (int32_t)min<int64_t>(g0 + kWave, m);
  wave_rows<T, NT, U>((int32_t)g0, g1, rp, ci, val, x, y,
                      lds + wid * kWave * U, lane);
}

// First super-row s in [lo, hi] with rp[inner[s]] >= target (wave-uniform).
__device__ __forceinline__ int32_t sr_lower_bound(
    int32_t lo, int32_t hi, int64_t target, const int32_t *__restrict__ inner,
    const int32_t *__restrict__ rp) {
  while (lo < hi) {
    const int32_t mid = lo + ((hi - lo) >> 1);
    if ((int64_t)rp[inner[mid]] < target)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

template <typename T, bool NT, int U, int W>
__global__ __launch_bounds__(W * 64) void hspmv_csr3(
    int32_t n_ssr, const int32_t *__restrict__ outer,
    const int32_t *__restrict__ inner, const int32_t *__restrict__ rp,
    const int32_t *__restrict__ ci, const T *__restrict__ val,
    const T *__restrict__ x, T *__restrict__ y) {
  __shared__ T lds[W * kWave * U];
  const int wid = threadIdx.x >> 6;
  const int lane = threadIdx.x & (kWave - 1);
  const int32_t b = blockIdx.x;
  const int32_t s0 = outer[b];
  const int32_t s1 = outer[b + 1];
  int32_t sa = s0, sb = s1;
  if constexpr (W > 1) {
    const int64_t k0 = rp[inner[s0]];
    const int64_t k1 = rp[inner[s1]];
    if (wid > 0) sa = sr_lower_bound(s0, s1, k0 + (k1 - k0) * wid / W, inner, rp);
    if (wid < W - 1)
      sb = sr_lower_bound(s0, s1, k0 + (k1 - k0) * (wid + 1) / W, inner, rp);
  }
  const int32_t r0 = inner[sa];
  const int32_t r1 = inner[sb];
  T *my = lds + wid * kWave * U;
  for (int32_t g0 = r0; g0 < r1; g0 += kWave)
    wave_rows<T, NT, U>(g0, min(g0 + kWave, r1), rp, ci, val, x, y, my, lane);
}

// ------------------------------------------------------------------ dispatch

template <typename T, bool NT>
hipError_t launch_typed(const DevCSR &A, const LaunchPlan &p, const T *x, T *y,
                        hipStream_t st) {
  const int32_t *rp = A.row_ptr;
  const int32_t *ci = A.col_idx;
  const T *val = static_cast<const T *>(A.val);
  if (A.m == 0) return hipSuccess;
  const dim3 grid((unsigned)p.blocks);
  switch (p.kernel) {
    case kVector:
      switch (p.lanes) {
#define HSPMV_VEC(L)                                                         \
  case L:                                                                    \
    hipLaunchKernelGGL((hspmv_csr_vector<T, L, NT>), grid, dim3(256), 0, st, \
                       A.m, rp, ci, val, x, y);                              \
    break;
        HSPMV_VEC(1) HSPMV_VEC(2) HSPMV_VEC(4) HSPMV_VEC(8) HSPMV_VEC(16)
        HSPMV_VEC(32) HSPMV_VEC(64)
#undef HSPMV_VEC
        default:
          return hipErrorInvalidValue;
      }
      break;
    case kStream:
      hipLaunchKernelGGL((hspmv_csr_stream<T, NT, kStreamU>), grid, dim3(256),
                         0, st, A.m, rp, ci, val, x, y);
      break;
    case kCsr3:
      switch (p.waves_per_block) {
        case 1:
          hipLaunchKernelGGL((hspmv_csr3<T, NT, kStreamU, 1>), grid, dim3(64),
                             0, st, A.n_ssr, A.outer, A.inner, rp, ci, val, x, y);
          break;
        case 2:
          hipLaunchKernelGGL((hspmv_csr3<T, NT, kStreamU, 2>), grid, dim3(128),
                             0, st, A.n_ssr, A.outer, A.inner, rp, ci, val, x, y);
          break;
        case 4:
          hipLaunchKernelGGL((hspmv_csr3<T, NT, kStreamU, 4>), grid, dim3(256),
                             0, st, A.n_ssr, A.outer, A.inner, rp, ci, val, x, y);
          break;
        default:
          return hipErrorInvalidValue;
      }
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

int floor_pow2(double v) {
  int p = 1;
  while (p * 2 <= v && p < 64) p *= 2;
  return p;
}

}  // namespace

LaunchPlan plan_launch(const DevCSR &A, int dtype, unsigned flags,
                       double mean_rows_per_ssr) {
  (void)dtype;
  LaunchPlan p;
  const unsigned k = flags & 0xFu;
  p.nontemporal = (flags & (1u << 12)) != 0;
  const double d = A.m ? (double)A.nnz / (double)A.m : 0.0;
  if (k == kAuto)
    p.kernel = (A.n_ssr > 0) ? kCsr3 : kStream;
  else
    p.kernel = (int)k;
  if (p.kernel == kCsr3 && A.n_ssr <= 0) p.kernel = kStream;
  switch (p.kernel) {
    case kVector: {
      int lanes = (int)((flags >> 4) & 0x7Fu);
      if (lanes == 0) lanes = floor_pow2(d < 2.0 ? 2.0 : d);
      p.lanes = lanes;
      int64_t threads = (int64_t)A.m * lanes;
      int64_t blocks = (threads + 255) / 256;
      const int64_t cap = 256LL * 8 * 16;  // grid-stride beyond 16 waves/SIMD
      p.blocks = blocks < cap ? blocks : cap;
      if (p.blocks < 1) p.blocks = 1;
      break;
    }
    case kStream: {
      p.lanes = kWave;
      const int64_t tasks = ((int64_t)A.m + kWave - 1) / kWave;
      p.blocks = (tasks + 3) / 4;
      break;
    }
    case kCsr3: {
      p.lanes = kWave;
      p.waves_per_block =
          mean_rows_per_ssr >= 192.0 ? 4 : (mean_rows_per_ssr >= 96.0 ? 2 : 1);
      p.blocks = A.n_ssr;
      break;
    }
  }
  return p;
}

hipError_t launch_spmv(const DevCSR &A, int dtype, const LaunchPlan &plan,
                       const void *x, void *y, hipStream_t stream) {
  if (dtype == 1) {
    return plan.nontemporal
               ? launch_typed<double, true>(A, plan, (const double *)x, (double *)y, stream)
               : launch_typed<double, false>(A, plan, (const double *)x, (double *)y, stream);
  }
  return plan.nontemporal
             ? launch_typed<float, true>(A, plan, (const float *)x, (float *)y, stream)
             : launch_typed<float, false>(A, plan, (const float *)x, (float *)y, stream);
}

}  // namespace hspmv
