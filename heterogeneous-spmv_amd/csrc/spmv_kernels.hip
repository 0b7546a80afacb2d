// spmv_kernels.hip -- hand-written CDNA4 (gfx950) SpMV kernels.
//
// The hot path of the reference is the row-wise nonzero dot product
//   y[r] = sum_{k=rp[r]}^{rp[r+1]-1} val[k] * x[col[k]]
// (spmv-csr/spmv.c:92-114; GPU forms cuda-spmv-csr/spmv.cu:117-182 and
// cuda-spmv-csrk/hip/csrk.cu:185-390).  It is an HBM-bound gather: 2 flops per
// 12 B (fp64) / 8 B (fp32) of matrix stream, so no MFMA anywhere here.
//
// Kernels (all wave64-native):
//
//  * hspmv_csr_stream<T, NT, U>   (HSPMV_KERNEL_STREAM, the default for CSR)
//      one wavefront per group of 64 consecutive rows.  The group's nonzeros
//      are contiguous, so the wave streams them with fully coalesced loads
//      (U elements per lane per chunk), forms the products val*x[col] and
//      stages them in a per-wave LDS slice.  Then
//        - rows of <= kSerialMax nonzeros: lane i sums row i left to right.
//          Summation order and rounding (product rounded, then sum rounded,
//          starting from 0) are those of omp_spmv, so these rows are
//          BIT-IDENTICAL to the CPU reference;
//        - longer rows: the whole wave sums the row's products in the chunk
//          (shuffle tree), accumulated over chunks (fp64 tolerance);
//        - split rows (> kLongRow nonzeros) are skipped here and summed by
//          hspmv_long_chunks + hspmv_long_reduce (many workgroups per row).
//      The serial bound is an argument (DevPlan.serial_max): with
//      hspmv_options.deterministic = 3 every row takes the first branch,
//      and split rows go to hspmv_long_serial (one workgroup per row, the
//      adds still in order, on a stream forked beside this kernel) +
//      hspmv_long_scatter.
//      Replaces cuda_spmv's thread-per-row scalar loop (uncoalesced) with a
//      CSR-stream scheme (coalesced stream + LDS segmented sums).
//
//  * hspmv_csr3<T, NT, U, W>      (HSPMV_KERNEL_CSR3)
//      CSR-3: wave tasks planned on the host, four per workgroup: 64-row
//      aligned groups by default (cache-line-aligned y stores), super-rows
//      packed into <= 64-row tasks (HSPMV_TASK_FILL=0), or one workgroup of
//      W waves per super-super-row whose super-rows are split W ways by
//      nonzeros (HSPMV_CSR3_PLAN=ssr); each wave runs the stream routine
//      over its task (hspmv_tables.cpp build_tasks).  Replaces cuSpMV_3 / cuSpMV_3_vec (thread or
//      sub-warp per row inside (8,12)-thread blocks, csrk.cu:185-319) and
//      cuSpMV_2 (degenerate outer level).
//
//  * hspmv_csr_vector<T, L, NT>   (HSPMV_KERNEL_VECTOR)
//      L lanes (a sub-wave, L | 64) per row, lanes stride the row's nonzeros
//      with FMA, reduced by __shfl_xor inside the L-lane group.  Replaces
//      cuSpMV_3_vec's veclevel lanes + barrier-free volatile-LDS tree
//      (csrk.cu:222-240) with a wave64-safe shuffle reduction; L = 1 is the
//      thread-per-row cuda_spmv shape.
//
// Blocks are remapped so each of the 8 XCDs (private 4 MiB L2 each) gets a
// contiguous range of row groups: neighbouring rows share x[] lines and the
// edges of val/col lines, which then hit in one L2 instead of eight.
//
// Build: hipcc --offload-arch=gfx950 -ffp-contract=off.  Contraction is off so
// that only the explicit fma() calls (vector kernel, long rows) fuse.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "hspmv_internal.h"

namespace hspmv {
namespace {

constexpr int kWave = 64;

template <bool NT, typename T>
__device__ __forceinline__ T ldg(const T *p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

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

// Split rows, step 1: one 256-thread workgroup per chunk of <= kLongChunk
// nonzeros of one long row -> partials[chunk].
template <typename T, bool NT>
__global__ __launch_bounds__(256) void hspmv_long_chunks(
    int32_t n_chunks, const int32_t *__restrict__ chunk_k, const int32_t *__restrict__ ci,
    const T *__restrict__ val, const T *__restrict__ x, T *__restrict__ partials) {
  __shared__ T red[4];
  const int c = blockIdx.x;
  if (c >= n_chunks) return;  // block-uniform
  const int32_t k0 = chunk_k[2 * c], k1 = chunk_k[2 * c + 1];
  T s0 = T(0), s1 = T(0);
  int32_t k = k0 + threadIdx.x;
  for (; k + 256 < k1; k += 512) {
    s0 = fma(ldg<NT>(val + k), x[ldg<NT>(ci + k)], s0);
    s1 = fma(ldg<NT>(val + k + 256), x[ldg<NT>(ci + k + 256)], s1);
  }
  if (k < k1) s0 = fma(ldg<NT>(val + k), x[ldg<NT>(ci + k)], s0);
  const T s = wave_sum(s0 + s1);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partials[c] = (red[0] + red[1]) + (red[2] + red[3]);
}

// Split rows, step 2: one wave per long row adds its chunk partials.
template <typename T>
__global__ __launch_bounds__(256) void hspmv_long_reduce(
    int32_t n_long, const int32_t *__restrict__ long_row, const int32_t *__restrict__ cstart,
    const T *__restrict__ partials, T *__restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n_long) return;
  const int32_t c0 = cstart[j], c1 = cstart[j + 1];
  T s = T(0);
  for (int32_t c = c0 + lane; c < c1; c += kWave) s += partials[c];
  s = wave_sum(s);
  if (lane == 0) y[long_row[j]] = s;
}

// Serial order (hspmv_options.deterministic = 3), rows over kLongRow
// nonzeros: one 256-thread workgroup per row adds the row's products left
// to right from 0, as omp_spmv does -- which no number of lanes can share.
// Waves 1-3 form the next 16 KiB of products (multiply rounded on its
// own, no fma: -ffp-contract=off) into one LDS buffer while lane 0 of wave 0
// adds the current one: 32 products per step, read as 16-byte LDS loads
// issued one step ahead of the dependent adds, so the add chain (not the
// LDS round trip) bounds the row.  In the row kernels such a row was walked by
// one lane through its wave's product chunks, one LDS round trip per four
// adds (C5's 144 616-nonzero hub row: 2.1 ms for the launch).
constexpr int kLongSerialBytes = 16384;  // per LDS buffer (two: 32 KiB)

template <typename T, bool NT>
__global__ __launch_bounds__(256) void hspmv_long_serial(
    int32_t n_long, const int32_t *__restrict__ long_row, const int32_t *__restrict__ rp,
    const int32_t *__restrict__ ci, const T *__restrict__ val, const T *__restrict__ x,
    T *__restrict__ y, T *__restrict__ lsum) {
  constexpr int32_t kLongSerialChunk = kLongSerialBytes / (int)sizeof(T);
  __shared__ __attribute__((aligned(16))) T buf[2][kLongSerialChunk];
  const int j = blockIdx.x;
  if (j >= n_long) return;  // block-uniform
  const int32_t r = long_row[j];
  const int32_t k0 = rp[r], k1 = rp[r + 1];
  auto fill = [&](T *dst, int32_t c, int t, int nt) {
    const int32_t n = min(k1 - c, kLongSerialChunk);
    for (int32_t i = t; i < n; i += nt) {
      const T p = ldg<NT>(val + c + i) * x[ldg<NT>(ci + c + i)];
      dst[i] = p;
    }
  };
  fill(buf[0], k0, threadIdx.x, 256);
  __syncthreads();
  T acc = T(0);
  int s = 0;
  for (int32_t c = k0; c < k1; c += kLongSerialChunk, s ^= 1) {
    if (threadIdx.x >= kWave) {
      if (c + kLongSerialChunk < k1) fill(buf[s ^ 1], c + kLongSerialChunk, threadIdx.x - kWave, 256 - kWave);
    } else if (threadIdx.x == 0) {
      const int32_t n = min(k1 - c, kLongSerialChunk);
      const T *b = buf[s];
      constexpr int V = 16 / (int)sizeof(T), B = 32;
      typedef T tv __attribute__((ext_vector_type(V)));
      int32_t i = 0;
      // two register sets, no copies: each step's loads go out (a
      // sched_barrier keeps them there) before the other set's adds
      auto load = [&](tv(&q)[B / V], int32_t at) {
#pragma unroll
        for (int v = 0; v < B / V; ++v) q[v] = *reinterpret_cast<const tv *>(b + at + v * V);
      };
      auto add = [&](const tv(&q)[B / V]) {
#pragma unroll
        for (int v = 0; v < B / V; ++v)
#pragma unroll
          for (int e = 0; e < V; ++e) acc = acc + q[v][e];
      };
      if (n >= 2 * B) {
        tv q0[B / V], q1[B / V];
        load(q0, 0);
        for (; i + 2 * B <= n; i += 2 * B) {
          load(q1, i + B);
          __builtin_amdgcn_sched_barrier(0);
          add(q0);
          __builtin_amdgcn_sched_barrier(0);
          load(q0, i + 3 * B <= n ? i + 2 * B : i);  // (a harmless reload at the end)
          __builtin_amdgcn_sched_barrier(0);
          add(q1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      for (; i < n; ++i) acc = acc + b[i];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (lsum)
      lsum[j] = acc;  // forked: hspmv_long_scatter writes y after the row kernel
    else
      y[r] = acc;
  }
}

// The forked long rows' sums into y, on the launch stream after the row
// kernel (whose x-slab passes also write those rows: empty segments).
template <typename T>
__global__ __launch_bounds__(256) void hspmv_long_scatter(int32_t n_long, const int32_t *__restrict__ long_row,
                                                          const T *__restrict__ lsum, T *__restrict__ y) {
  const int32_t j = (int32_t)(blockIdx.x * 256 + threadIdx.x);
  if (j < n_long) y[long_row[j]] = lsum[j];
}

// ------------------------------------------------------------------ dispatch

template <typename T, bool NT>
hipError_t launch_typed(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const T *x,
                        T *y, hipStream_t st) {
  if (A.m == 0) return hipSuccess;
  const int32_t *rp = A.row_ptr;
  const int32_t *ci = A.col_idx;
  const T *val = static_cast<const T *>(A.val);
  hipError_t e = hipSuccess;
  // serial order: the long rows' workgroups start first, on their own
  // stream (forked from st, joined back below), beside the row kernel, and
  // leave their sums in dp.partials for hspmv_long_scatter -- C5: 289 us of
  // x-slab passes and a 497 us add chain otherwise in sequence
  const bool fork = dp.n_long > 0 && dp.long_serial && dp.long_stream;
  if (fork) {
    if ((e = hipEventRecord(dp.long_fork, st)) != hipSuccess ||
        (e = hipStreamWaitEvent(dp.long_stream, dp.long_fork, 0)) != hipSuccess)
      return e;
    hipLaunchKernelGGL((hspmv_long_serial<T, NT>), dim3((unsigned)dp.n_long), dim3(256), 0, dp.long_stream,
                       dp.n_long, dp.long_row, rp, ci, val, x, y, static_cast<T *>(dp.partials));
    if ((e = hipGetLastError()) != hipSuccess || (e = hipEventRecord(dp.long_join, dp.long_stream)) != hipSuccess)
      return e;
  }
  switch (p.kernel) {
    case kVector:
      switch (p.lanes) {
#define HSPMV_VEC(L)                                                                    \
  case L:                                                                               \
    hipLaunchKernelGGL((hspmv_csr_vector<T, L, NT>), dim3((unsigned)p.blocks), dim3(256), \
                       0, st, A.m, rp, ci, val, x, y);                                  \
    break;
        HSPMV_VEC(1) HSPMV_VEC(2) HSPMV_VEC(4) HSPMV_VEC(8) HSPMV_VEC(16)
        HSPMV_VEC(32) HSPMV_VEC(64)
#undef HSPMV_VEC
        default:
          return hipErrorInvalidValue;
      }
      return hipGetLastError();  // the vector kernel sums split rows itself
    case kStream:
    case kCsr3:
      if (dp.n_slabs > 0) {  // one pass per x slab, each continuing the rows from y
        DevCSR As = A;
        As.col_idx = dp.slab_col;
        As.val = dp.slab_val;
        As.col16 = nullptr;
        As.cbase = nullptr;
        As.cplanes = nullptr;
        As.n_cplanes = 0;
        LaunchPlan ps = p;
        for (int32_t b = 0; b < dp.n_slabs && e == hipSuccess; ++b) {
          As.row_ptr = dp.slab_rp + (size_t)b * (size_t)(A.m + 1);
          ps.carry = b > 0;
          if constexpr (sizeof(T) == 8)
            e = launch_rows_f64(As, dp, ps, x, y, st);
          else
            e = launch_rows_f32(As, dp, ps, x, y, st);
        }
      } else if constexpr (sizeof(T) == 8) {
        e = launch_rows_f64(A, dp, p, x, y, st);
      } else {
        e = launch_rows_f32(A, dp, p, x, y, st);
      }
      if (e != hipSuccess) return e;
      break;
    case kCsort:
      return launch_csort(dp.cs, sizeof(T) == 8 ? 1 : 0, x, y, st);
    default:
      return hipErrorInvalidValue;
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (fork) {
    if ((e = hipStreamWaitEvent(st, dp.long_join, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL((hspmv_long_scatter<T>), dim3((unsigned)((dp.n_long + 255) / 256)), dim3(256), 0, st,
                       dp.n_long, dp.long_row, static_cast<const T *>(dp.partials), y);
    e = hipGetLastError();
  } else if (dp.n_long > 0 && dp.long_serial) {
    hipLaunchKernelGGL((hspmv_long_serial<T, NT>), dim3((unsigned)dp.n_long), dim3(256), 0, st, dp.n_long,
                       dp.long_row, rp, ci, val, x, y, static_cast<T *>(nullptr));
    e = hipGetLastError();
  } else if (dp.n_long > 0) {
    hipLaunchKernelGGL((hspmv_long_chunks<T, NT>), dim3((unsigned)dp.n_chunks), dim3(256), 0, st,
                       dp.n_chunks, dp.chunk_k, ci, val, x, static_cast<T *>(dp.partials));
    hipLaunchKernelGGL((hspmv_long_reduce<T>), dim3((unsigned)((dp.n_long + 3) / 4)), dim3(256),
                       0, st, dp.n_long, dp.long_row, dp.long_cstart,
                       static_cast<const T *>(dp.partials), y);
    e = hipGetLastError();
  }
  return e;
}

int floor_pow2(double v) {
  int p = 1;
  while (p * 2 <= v && p < 64) p *= 2;
  return p;
}

// Elements per lane per LDS chunk.  Measured on MI355X (profiles/r01_sweep*):
// the chunk must stay small enough for 8 waves/SIMD (U = 4: 62 VGPRs fp64),
// and a 64-row group that fits one chunk of U <= 6 should be done in one.
// fp32 (profiles/r01_ab_f32_u.jsonl): two chunks of U = 6 beat U = 8 on C4's
// 640-nonzero groups (34.3 vs 40.2 us), and long groups take U = 16 (C3's
// 27-point rows: 62.3 vs 67.4 us) -- except on x-slab passes, where U = 8
// measured best (C5: 273 vs 291 us, r01_ab_c5_slabs_u.jsonl).
int pick_u(double nnz_per_pass, int dtype, bool slabs) {
  if (nnz_per_pass <= 128.0) return 2;
  if (nnz_per_pass <= 192.0) return 3;
  if (nnz_per_pass <= 256.0) return 4;
  // 5-nonzero rows fill U = 5 exactly (C2 14.76 -> 14.28 us, l4k 208 -> 199;
  // profiles/r01_ab_u5.jsonl)
  if (nnz_per_pass <= 320.0) return 5;
  if (nnz_per_pass <= 384.0) return 6;
  // two chunks, as full as possible: C4's 640-nonzero groups take 2 x 320
  // (U = 5: fp64 51.1 -> 50.2 us, fp32 35.0 -> 33.0; r01_ab_u5.jsonl)
  if (nnz_per_pass <= 768.0) {
    const int u = (int)((nnz_per_pass + 127.0) / 128.0);
    return u <= 4 ? 4 : (u == 5 ? 5 : 6);
  }
  if (dtype == 1) return 4;
  return slabs ? 8 : 16;
}

}  // namespace

LaunchPlan plan_launch(const DevCSR &A, int dtype, unsigned flags, double rows_per_ssr,
                       int64_t packed_tasks, const Tuning &t) {
  LaunchPlan p;
  const unsigned k = flags & 0xFu;
  p.nontemporal = (flags & (1u << 12)) != 0;  // HSPMV_FLAG_NONTEMPORAL
  p.prefetch = (flags & (1u << 21)) != 0;  // HSPMV_FLAG_PREFETCH
  // (with x slabs each pass sees ~d / n_slabs per row, but the chunk size
  // is still picked from d: U = 8 over U = 4/6 on C5's slab passes, 284 vs
  // 320 us -- more gathers in flight per wave; profiles/r01_ab_c5_slabs_u.jsonl)
  const double d_all = A.m ? (double)A.nnz / (double)A.m : 0.0;
  const double d = d_all;
  // XCD block order: a contiguous eighth of the rows per XCD keeps x in that
  // XCD's L2, which pays when the matrix is served from the Infinity Cache;
  // from HBM the dispatch order (the whole chip on one compact window)
  // streams 3-8 % faster (profiles/r01_sweep2-4: C2 full remap 15.6 vs
  // 16.9 us; C3 132 vs 128, C4 70.6 vs 65.4).  Chunked orders in between:
  // xcd_chunk_remap in spmv_device.cuh.
  const double sv = dtype == 1 ? 8.0 : 4.0;
  const double footprint = (double)A.nnz * (sv + 4.0) + (double)A.m * (sv + 4.0) + (double)A.n * sv;
  const unsigned chunk_code = (flags >> 24) & 0x1Fu;  // HSPMV_XCD_CHUNK(s)
  bool full = false;
  int32_t chunk = 1;
  if (chunk_code)
    chunk = 1 << (chunk_code - 1);
  else if (flags & (1u << 14))  // HSPMV_FLAG_NO_XCD_REMAP
    chunk = 1;
  else if (flags & (1u << 22))  // HSPMV_FLAG_XCD_REMAP
    full = true;
  else if (footprint <= 192.0 * 1024 * 1024)
    full = true;
  else if (A.has_xdict || A.has_xdict_tasks)
    // x dictionaries: each XCD takes 4 consecutive workgroups in turn, so the
    // x runs neighbouring workgroups stage are still in that XCD's L2
    // (C3 CSR-3 fp64 112.7 -> 105.2 us, fp32 63.7 -> 62.6; 2 / 8 / 16 / 64
    // blocks: 112.3 / 105.8 / 109.4 / 109.6; profiles/r02k_ab_xcd.jsonl)
    chunk = 4;
  // (packed tasks without super-super-rows: a CSR matrix whose 64-row
  // groups exceed the task budget, hspmv_tables.cpp build_tasks)
  const bool tasks = A.n_ssr > 0 || packed_tasks > 0;
  if (k == kAuto)
    p.kernel = A.has_csort ? kCsort : (tasks && !A.slab_stream ? kCsr3 : kStream);
  else
    p.kernel = (int)k;
  if (p.kernel == kCsort && !A.has_csort) p.kernel = tasks ? kCsr3 : kStream;
  if (p.kernel == kCsr3 && !tasks) p.kernel = kStream;
  const int forced_u = (int)((flags >> 16) & 0x1Fu);  // HSPMV_U(u)
  switch (p.kernel) {
    case kCsort:  // the workgroup shape is fixed; the host tables hold the rest
      p.lanes = kWave;
      p.waves_per_block = kCsortThreads / kWave;
      p.blocks = 0;  // set from the tables (build_plan_tables)
      break;
    case kVector: {
      int lanes = (int)((flags >> 4) & 0x7Fu);
      if (lanes == 0) lanes = floor_pow2(d_all < 2.0 ? 2.0 : d_all);
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
      p.u = forced_u ? forced_u : pick_u(64.0 * (d < kLongRow ? d : kLongRow), dtype, A.n_slabs > 1);
      const int64_t tasks = ((int64_t)A.m + kWave - 1) / kWave;
      const unsigned gcode = (flags >> 29) & 0x7u;  // HSPMV_GROUPS(g)
      p.groups = gcode ? 1 << (gcode - 1) : 1;
      const int64_t waves = (tasks + p.groups - 1) / p.groups;
      // waves per workgroup.  The STREAM waves never meet at a barrier, so
      // small workgroups free their CU slots wave by wave: one wave per
      // workgroup for Infinity-Cache-resident matrices (C2 bench 737 -> 760
      // GFLOP/s), two for HBM-resident ones, where one-wave workgroups run
      // into the per-CU workgroup limit (honeycomb 166.0 -> 161.8 us with
      // two, flat with one; l4k 211.2 -> 207.5; profiles/r01_ab_stream_w.jsonl).
      // LDS-windowed HBM matrices took one wave until r04 (C4 53.2 -> 50.4
      // us in r01); on today's kernel two measure 47.1 vs 47.7-48.0 on C4's
      // 8-rank shard and tie at 4 / 2 / 1 ranks (profiles/r04/
      // sweep_stream_waves.jsonl, 7 rounds, one process).  Four (the
      // dictionaries' 256-row blocks) with x dictionaries.
      p.waves_per_block = A.has_xdict ? 4 : (footprint <= 192.0 * 1024 * 1024 ? 1 : 2);
      if ((t.stream_waves == 1 || t.stream_waves == 2 || t.stream_waves == 4) && !A.has_xdict)
        p.waves_per_block = t.stream_waves;
      p.blocks = (waves + p.waves_per_block - 1) / p.waves_per_block;
      break;
    }
    case kCsr3: {
      p.lanes = kWave;
      if (packed_tasks > 0) {  // host-planned wave tasks: task_waves per block
        p.waves_per_block = (A.task_waves == 1 || A.task_waves == 2 || A.task_waves == 8) ? A.task_waves : 4;
        const double rows_per_task = (double)A.m / (double)packed_tasks;
        const double per_pass = (rows_per_task < 64.0 ? rows_per_task : 64.0) * d;
        p.u = forced_u ? forced_u : pick_u(per_pass < 64.0 * kLongRow ? per_pass : 64.0 * kLongRow, dtype, A.n_slabs > 1);
        p.blocks = (packed_tasks + p.waves_per_block - 1) / p.waves_per_block;
        break;
      }
      // ~64 rows per wave (one lane per row in the ordered sums)
      p.waves_per_block = ssr_waves(rows_per_ssr);
      const double rows_per_task = rows_per_ssr / p.waves_per_block;
      const double per_pass = (rows_per_task < 64.0 ? rows_per_task : 64.0) * d;
      p.u = forced_u ? forced_u : pick_u(per_pass < 64.0 * kLongRow ? per_pass : 64.0 * kLongRow, dtype, A.n_slabs > 1);
      p.blocks = A.n_ssr;
      break;
    }
  }
  // The STREAM / CSR3 kernels address x and the matrix streams as a 64-bit
  // base plus a 32-bit byte offset (spmv_device.cuh ld_off): x of 4 GiB or
  // more (fp64: n >= 2^29), or -- without split rows -- a row group that
  // could stream 4 GiB, would wrap.  Such matrices take a kernel that
  // indexes through pointers: csort when it was built, else VECTOR.
  const double max_run_bytes =
      (flags & (1u << 15)) ? (double)A.nnz * (sv > 4.0 ? sv : 4.0) : 64.0 * kLongRow * sv;
  if ((p.kernel == kStream || p.kernel == kCsr3) &&
      ((double)A.n * sv > 4294967295.0 || max_run_bytes > 4294967295.0))
    p.kernel = A.has_csort ? kCsort : kVector;
  if (p.kernel == kVector && !(k == kVector)) {  // re-plan the vector launch shape
    p.lanes = floor_pow2(d_all < 2.0 ? 2.0 : d_all);
    const int64_t threads = (int64_t)A.m * p.lanes;
    const int64_t cap = 256LL * 8 * 16;
    p.blocks = (threads + 255) / 256 < cap ? (threads + 255) / 256 : cap;
    if (p.blocks < 1) p.blocks = 1;
  }
  if (p.kernel == kVector || p.kernel == kCsort) {
    full = false;
    chunk = 1;  // dispatch order (csort: the column parts alternate XCDs)
  }
  if (full) {
    const int64_t per_xcd = p.blocks / 8;
    chunk = per_xcd > 1 ? (int32_t)per_xcd : 1;
  }
  p.xcd_chunk = chunk;
  // HBM-resident matrices: nontemporal y stores; and nontemporal col/val
  // streams when the x gather is irregular (column spans of 2^18+ per
  // 256-nonzero block) and x exceeds an XCD's 4 MiB L2, so the streamed
  // bytes do not evict x (C5: -5 %; banded C3/C4: +3-7 %, left off).
  // HSPMV_YNT / HSPMV_NT (0/1) override, for A/B runs.
  const bool hbm = footprint > 192.0 * 1024 * 1024;
  p.y_nt = hbm;
  // (not on x-slab passes, whose gathers are L2-resident anyway: C5 284 ->
  // 265 us with plain loads, profiles/r01_ab_nt_slabs.jsonl)
  if (!p.nontemporal && hbm && A.col_span_bits > 17 && (double)A.n * sv > 4.0 * 1024 * 1024 &&
      A.n_slabs <= 1)
    p.nontemporal = true;
  // fp64 CSR3 tasks with x dictionaries: the next chunk's col/val loads are
  // issued during this chunk's gathers and sums (C3 112.2 -> 105.8 us on one
  // box, 112.4 -> 110.3 on another; slower everywhere else: C3 fp32 +14 %,
  // C4 +13 %, honeycomb +10 %, C2 +14 %; profiles/r02q_ab_c3_u.jsonl,
  // r02r_ab_pf.jsonl)
  if (!p.prefetch && dtype == 1 && p.kernel == kCsr3 && A.has_xdict_tasks && !forced_u)
    p.prefetch = true;
  // Bank-padded product buffers (STREAM, no prefetch): when
  // the typical serially summed row is a multiple of 16 LDS words long
  // (fp32 rows of 16 / 32, fp64 rows of 8 / 16 / 24 / 32 ...), the lanes
  // walking those rows hit at most two banks.  Dense 32x32 blocks: fp64
  // 129.6 -> 95.1 us, fp32 99.6 -> 67.1; fp64 rows of 24: 103.2 -> 95.9;
  // fp32 rows of 24 (8-word multiples) lose 3 % padded, so they are left
  // alone (profiles/r05j/ab_lds_pad.jsonl).  Decided after the A/B
  // overrides, so that hspmv_info.lds_pad reports the launch that runs (the
  // PF variant has no padded form).  Never with x dictionaries: those are
  // sized (hspmv_xdict.cpp xd_target_entries) against unpadded product
  // buffers, and the pad would cost the launch a workgroup per CU.
  if (t.pf >= 0) p.prefetch = t.pf != 0;  // A/B knobs (diagnostic builds only)
  if (t.y_nt >= 0) p.y_nt = t.y_nt != 0;
  if (t.nt >= 0) p.nontemporal = t.nt != 0;
  {
    const int words = A.serial_len * (dtype == 1 ? 2 : 1);
    const bool conflicting = words > 0 && (words % 16) == 0;
    const bool can_pad = p.kernel == kStream && !p.prefetch && !A.has_xdict;
    p.lds_pad = can_pad && conflicting;
    if (t.lds_pad >= 0) p.lds_pad = can_pad && t.lds_pad > 0;
  }
  p.dyn_lds = t.dyn_lds;
  return p;
}

hipError_t launch_spmv(const DevCSR &A, const DevPlan &dp, int dtype, const LaunchPlan &plan,
                       const void *x, void *y, hipStream_t stream) {
  if (dtype == 1) {
    return plan.nontemporal
               ? launch_typed<double, true>(A, dp, plan, (const double *)x, (double *)y, stream)
               : launch_typed<double, false>(A, dp, plan, (const double *)x, (double *)y, stream);
  }
  return plan.nontemporal
             ? launch_typed<float, true>(A, dp, plan, (const float *)x, (float *)y, stream)
             : launch_typed<float, false>(A, dp, plan, (const float *)x, (float *)y, stream);
}

}  // namespace hspmv
