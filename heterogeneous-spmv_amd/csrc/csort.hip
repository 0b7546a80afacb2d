// csort.hip -- the column-sorted row-block kernel (HSPMV_KERNEL_CSORT) for
// matrices whose gathers are irregular (power-law / random columns, C5).
//
// Why: with random columns every nonzero of the row kernels is its own L2
// request (one 4-8 B x entry per 128 B line), and C5's 48 M gathers hit the
// L2 request rate (x slabs: 4 passes x 12.6 M TCC requests, TCC busy 83 %,
// profiles/r01_pmc_c5_slabs).  Here each workgroup owns a nnz-balanced block
// of rows and one of H column parts, and walks the block's nonzeros IN
// COLUMN ORDER: the 64 lanes of a gather then fall on a few x lines (one
// request serves several lanes) and all CUs of an XCD sweep x together, so
// the lines they fetch are L2 hits for each other.  Workgroup b = (row block
// b / H, column part b % H); under round-robin dispatch the parts alternate
// XCDs, so each XCD's L2 only ever holds its part of x.  Probe:
// profiles/r02*_c5_csort_probe.jsonl (C5: 264 us library -> 109 us).
//
// Row sums: one fp64 LDS slot per row of the block (plus one per long-row
// slice and a dummy slot for padding), accumulated with ds_add_f64.  The
// products are formed exactly as omp_spmv forms them for fp64 (v*x rounded),
// and exactly (fp32 x fp32 in fp64) for fp32.  Each column part's fp64 row
// sums are stored as partials (fp32 for fp32 data: part32, the default) and
// added in a fixed order, in fp64, by the finishing pass, which rounds y.
// The order of the slot additions is the atomic order, so unlike the
// STREAM/CSR3 kernels this path is NOT bitwise equal to omp_spmv: fp32
// results are within an fp32 rounding of y and of each part's sum of the
// exact sum (more accurate than omp_spmv's fp32 running sum), equal run to
// run except where an fp64 sum sits within an fp64 rounding of an fp32 tie;
// fp64 results agree with omp_spmv to the fp64 rounding of the sum.  FIX
// (hspmv_options.deterministic = 2): int64 fixed-point slots instead (see
// fix_q), the same bits on every run.
//
// Layout (built on the host, hspmv_csort_build.cpp build_csort): entries padded to
// whole chunks of 64*U; per chunk a base column (cbase); per entry idx =
// slot << 16 | (col - base) (a chunk never spans more than 65535 columns)
// and the value: fp32 as one 8-byte {idx, val} record (one load per
// element), fp64 as idx[] + val[] (FIX: the values scaled per row by
// 2^rexp).  The partial sums of the H parts (part[h * m + row]) and of the
// long-row slices (spart[slice], fp64) are combined in a fixed order by
// hspmv_csort_finish.
#include <hip/hip_runtime.h>

#include "hspmv_internal.h"

// Ablation builds only (wrong results by design; the csort-abl libraries of
// the Makefile): 1 = the slot adds as ds_add_u64 of the bit pattern, 2 = no
// slot adds (products summed in a register), 3 = a plain LDS read of the
// slot instead of the add, 4 = every gather of a chunk within the chunk's
// first x sector (the x sweep removed, the entry stream kept).
#ifndef HSPMV_CSORT_ABL
#define HSPMV_CSORT_ABL 0
#endif

namespace hspmv {
namespace {

constexpr int kWave = 64;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT, typename P>
__device__ __forceinline__ P ld(const P *p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

__device__ __forceinline__ int32_t wave_uniform(int32_t v) {
  return __builtin_amdgcn_readfirstlane(v);
}

// One DPP move (both dwords for fp64); lanes the pattern does not feed read
// `old` (keys: a sentinel no slot equals; values: 0).
template <int CTRL, int ROW_MASK, typename S>
__device__ __forceinline__ S dpp_val(S v) {
  if constexpr (sizeof(S) == 8) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROW_MASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, ROW_MASK, 0xf, false);
    return __builtin_bit_cast(S, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  } else {
    return __builtin_bit_cast(S, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                             ROW_MASK, 0xf, false));
  }
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_key(uint32_t k) {
  return (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)k, CTRL, ROW_MASK, 0xf, false);
}

// Inclusive segmented scan over the wave's 64 lanes; k = the lane's run id,
// non-decreasing along the lanes (so k[l - d] == k[l] means lanes l-d .. l
// are one run): row_shr 1/2/4/8 inside the 16-lane rows, then row_bcast
// 15 / 31 across them.
template <typename S>
__device__ __forceinline__ S seg_scan(S v, uint32_t k) {
#define HSPMV_SEG_STEP(CTRL, MASK)                        \
  {                                                      \
    const uint32_t kp = dpp_key<CTRL, MASK>(k);          \
    const S vp = dpp_val<CTRL, MASK>(v);                 \
    v += kp == k ? vp : S(0);                            \
  }
  HSPMV_SEG_STEP(0x111, 0xf)
  HSPMV_SEG_STEP(0x112, 0xf)
  HSPMV_SEG_STEP(0x114, 0xf)
  HSPMV_SEG_STEP(0x118, 0xf)
  HSPMV_SEG_STEP(0x142, 0xa)
  HSPMV_SEG_STEP(0x143, 0xc)
#undef HSPMV_SEG_STEP
  return v;
}

// Loads chunk c's U entries per lane (idx, value): entry u of the lane is
// the chunk's sorted entry u*64 + lane.  WIDE: 16-byte loads over a layout
// interleaved on the host (build_csort) so that one load brings the lane
// two (fp32 records, fp64 values) or four (fp64 indices) of its entries;
// the entry -> (u, lane) mapping, and so every gather, is unchanged.
template <typename T, int U, bool NT, bool WIDE>
__device__ __forceinline__ void load_entries(const void *__restrict__ ent, const T *__restrict__ val,
                                             int32_t c, int lane, uint32_t (&ix)[U], T (&vv)[U]) {
  const int64_t k0 = (int64_t)c * (kWave * U);
  if constexpr (WIDE) {
    if constexpr (sizeof(T) == 4) {  // records of entries u*64 + lane, (u+1)*64 + lane side by side
      const u32x4 *p = reinterpret_cast<const u32x4 *>(reinterpret_cast<const u32x2 *>(ent) + k0) + lane;
#pragma unroll
      for (int u = 0; u < U; u += 2) {
        const u32x4 r = ld<NT>(p + (u / 2) * kWave);
        ix[u] = r.x;
        vv[u] = __uint_as_float(r.y);
        ix[u + 1] = r.z;
        vv[u + 1] = __uint_as_float(r.w);
      }
    } else {
      static_assert(U % 4 == 0, "fp64 wide entries: U multiple of 4");
      const u32x4 *pi = reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint32_t *>(ent) + k0) + lane;
#pragma unroll
      for (int u = 0; u < U; u += 4) {
        const u32x4 r = ld<NT>(pi + (u / 4) * kWave);
        ix[u] = r.x;
        ix[u + 1] = r.y;
        ix[u + 2] = r.z;
        ix[u + 3] = r.w;
      }
      typedef double f64x2 __attribute__((ext_vector_type(2)));
      const f64x2 *pv = reinterpret_cast<const f64x2 *>(reinterpret_cast<const double *>(val) + k0) + lane;
#pragma unroll
      for (int u = 0; u < U; u += 2) {
        const f64x2 r = ld<NT>(pv + (u / 2) * kWave);
        vv[u] = r.x;
        vv[u + 1] = r.y;
      }
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t k = k0 + lane + u * kWave;
    if constexpr (sizeof(T) == 4) {
      const u32x2 p = ld<NT>(reinterpret_cast<const u32x2 *>(ent) + k);
      ix[u] = p.x;
      vv[u] = __uint_as_float(p.y);
    } else {
      ix[u] = ld<NT>(reinterpret_cast<const uint32_t *>(ent) + k);
      vv[u] = ld<NT>(val + k);
    }
  }
}

// Reproducible (fixed-point) slots, FIXP: each product v' x (v' = v 2^rexp,
// scaled per row on the host so that |v'| < 1) is rounded ONCE to a
// multiple of 2^-E, E = kCsortFixBits - xexp (|x| < 2^xexp): with M = 1.5 *
// 2^(52 - E) -- a per-SpMV constant -- fma(v', x, M) lands in M's binade,
// whose ulp is 2^-E, so it IS M + rint(v' x 2^E) 2^-E, and the int64
// difference of the bit patterns is that integer q (|q| < 2^50).  One fma
// and a 64-bit subtraction per product, where the fp64-slot path has a mul.
// Integer adds are associative, so the slot's sum -- and y -- is the same
// bits whatever order the LDS atomics land in (ds_add_u64 costs what
// ds_add_f64 does: profiles/r03/ab_c5_lds_add_ablation.jsonl).
__device__ __forceinline__ long long fix_q(double v, double x, double M, unsigned long long mbits) {
  const double r = __builtin_fma(v, x, M);
  return (long long)(__builtin_bit_cast(unsigned long long, r) - mbits);
}

// The chunks of one workgroup (see hspmv_csort).  FIXP: integer slots (the
// products rounded by fix_q at scale 2^E); otherwise S slots (ds_add_f64,
// or ds_add_f32 with fp32 slots).
template <typename T, typename S, int U, bool NT, bool PF, bool WIDE, bool FIXP>
__device__ __forceinline__ int32_t csort_chunks(int32_t c0, int32_t c1, int wid, int lane, int32_t dyn,
                                                int32_t *next_chunk, const int32_t *__restrict__ cbase,
                                                const void *__restrict__ ent, const T *__restrict__ val,
                                                const T *__restrict__ x, void *slots, double M) {
  constexpr int NW = kCsortThreads / kWave;
  S *acc = reinterpret_cast<S *>(slots);
  unsigned long long *acq = reinterpret_cast<unsigned long long *>(slots);
  const unsigned long long mbits = __builtin_bit_cast(unsigned long long, M);
  uint32_t ix[U];
  T vv[U];
#if HSPMV_CSORT_ABL == 2 || HSPMV_CSORT_ABL == 3
  S sink = S(0);  // ablation builds only
#endif
  // PF: the next chunk's entries are loaded while this chunk's gathers are
  // in flight (software pipelining across the wave's chunks)
  if constexpr (PF)
    if (c0 + wid < c1) load_entries<T, U, NT, WIDE>(ent, val, c0 + wid, lane, ix, vv);
  // Chunk order.  dyn: wave w starts at chunk c0 + w and then takes the
  // next unclaimed chunk of the workgroup (one LDS atomic per chunk, claimed
  // a chunk ahead so PF can load it).  Without it wave w takes every NW-th
  // chunk -- and the 16 waves finish in four tiers of four (one wave per
  // SIMD each, oldest first: C5 ~39 / 57 / 77 / 94 us), the last quarter of
  // the workgroup's time run by 4 waves (profiles/r05b/csort_trace.jsonl).
  int32_t cn_done = 0;
  for (int32_t c = c0 + wid; c < c1;) {  // wave-uniform
    int32_t cn = c + NW;
    if (dyn) {
      int32_t got = 0;
      if (lane == 0) got = atomicAdd(next_chunk, 1);
      cn = __builtin_amdgcn_readfirstlane(got);
    }
    ++cn_done;
    // bit 31 of the chunk base: a "segmented" chunk (see below)
    const uint32_t cb = (uint32_t)wave_uniform(cbase[wave_uniform(c)]);
    const int32_t base = (int32_t)(cb & 0x7fffffffu);
    const bool seg = (cb >> 31) != 0u;
    if constexpr (!PF) load_entries<T, U, NT, WIDE>(ent, val, c, lane, ix, vv);
    T xv[U];
#pragma unroll
#if HSPMV_CSORT_ABL == 4
    for (int u = 0; u < U; ++u) xv[u] = x[base + (int32_t)(ix[u] & 0x7u)];  // one x sector per chunk
#else
    for (int u = 0; u < U; ++u) xv[u] = x[base + (int32_t)(ix[u] & 0xffffu)];
#endif
    uint32_t ixc[U];
    T vvc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ixc[u] = ix[u];
      vvc[u] = vv[u];
    }
    if constexpr (PF) {
      __builtin_amdgcn_sched_barrier(0);
      if (cn < c1) load_entries<T, U, NT, WIDE>(ent, val, cn, lane, ix, vv);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (!seg) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (FIXP) {
          const long long q = fix_q((double)vvc[u], (double)xv[u], M, mbits);
          atomicAdd(&acq[ixc[u] >> 16], (unsigned long long)q);
        } else {
          S pr;
          if constexpr (sizeof(T) == 4 && sizeof(S) == 8)
            pr = (double)vvc[u] * (double)xv[u];  // exact
          else
            pr = (S)(vvc[u] * xv[u]);  // omp_spmv's rounded product
#if HSPMV_CSORT_ABL == 1
          if constexpr (sizeof(S) == 8)
            atomicAdd(reinterpret_cast<unsigned long long *>(&acc[ixc[u] >> 16]),
                      (unsigned long long)__builtin_bit_cast(long long, pr));
          else
            atomicAdd(&acc[ixc[u] >> 16], pr);
#elif HSPMV_CSORT_ABL == 2
          sink += pr + (S)(ixc[u] >> 16);
#elif HSPMV_CSORT_ABL == 3
          sink += pr * acc[ixc[u] >> 16];
#else
          atomicAdd(&acc[ixc[u] >> 16], pr);
#endif
        }
      }
    } else {
      // Segmented chunk: the host found rows whose entries crowd one
      // instruction (a hub row's contiguous columns after an RCM ordering:
      // up to 64 lanes on one slot, and same-address LDS atomics serialise)
      // and stored those rows' entries slot-sorted (consecutive lanes, in
      // column order within a row), the chunk's other entries after them in
      // column order.  Each instruction's runs of one slot are summed first
      // (DPP segmented scan), and the last lane of a run adds it: one atomic
      // per run.
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t sl = ixc[u] >> 16;
        // runs = maximal stretches of lanes with one slot; run id = the
        // number of run starts up to this lane (ballot + mbcnt)
        const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)sl, 0x138, 0xf, 0xf, false);
        const bool start = lane == 0 || prev != sl;  // (0x138: wave_shr 1)
        const unsigned long long msk = __ballot(start);
        const uint32_t rid = __builtin_amdgcn_mbcnt_hi((uint32_t)(msk >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)msk, 0u)) +
                             (start ? 1u : 0u);
        const bool last = lane == kWave - 1 || ((msk >> (lane + 1)) & 1ull);
        if constexpr (FIXP) {
          unsigned long long q = (unsigned long long)fix_q((double)vvc[u], (double)xv[u], M, mbits);
          q = seg_scan(q, rid);  // integer: the same sum in any association
          if (last) atomicAdd(&acq[sl], q);
        } else {
          S v;
          if constexpr (sizeof(T) == 4 && sizeof(S) == 8)
            v = (double)vvc[u] * (double)xv[u];
          else
            v = (S)(vvc[u] * xv[u]);
          v = seg_scan(v, rid);
          if (last) atomicAdd(&acc[sl], v);
        }
      }
    }
    c = cn;
  }
#if HSPMV_CSORT_ABL == 2 || HSPMV_CSORT_ABL == 3
  if (sink != S(0)) atomicAdd(&acc[0], sink * S(0));  // keeps the products live (adds 0)
#endif
  return cn_done;
}

// A slot's value: S slots as they are; fixed-point slots scaled back by
// 2^-(E + rexp) -- the int64 -> double conversion and the scaling round
// deterministically.
template <typename S, bool FIXP>
__device__ __forceinline__ S slot_value(const void *slots, int32_t i, int32_t e) {
  if constexpr (FIXP)
    return (S)__builtin_ldexp((double)(long long)reinterpret_cast<const unsigned long long *>(slots)[i], -e);
  else
    return reinterpret_cast<const S *>(slots)[i];
}

// The max exponent of |x| the workgroup's fixed-point scale comes from,
// reduced by each wave from the pre-pass's per-block maxima.
__device__ __forceinline__ int32_t wave_xexp(const int32_t *__restrict__ xexp_part, int32_t n, int lane) {
  int32_t e = -0x40000000;
  for (int32_t i = lane; i < n; i += kWave) e = max(e, xexp_part[i]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) e = max(e, __shfl_xor(e, off, kWave));
  return __builtin_amdgcn_readfirstlane(e);
}

// frexp exponent of |v| (|v| < 2^e; zeros ignored), kCsortXexpNonFinite for
// Inf, NaN or |v| >= 2^1020 (the rounding constant M would overflow)
__device__ __forceinline__ int32_t xexp_max(int32_t e, double v) {
  v = __builtin_fabs(v);
  if (!(v < 0x1p1020)) return kCsortXexpNonFinite;
  return v != 0.0 ? max(e, __builtin_amdgcn_frexp_exp(v)) : e;
}

// S: the LDS row-slot / partial-sum type (double; float only for fp32 data,
// an A/B variant with half the LDS per row).  FIX: reproducible fixed-point
// slots (DevCsort.fixed), falling back to S slots for an x with a non-finite
// entry (whose rows are then +-Inf / NaN in any order).
template <typename T, typename S, typename P, int U, bool NT, bool PF, bool WIDE, bool FIX>
__global__ __launch_bounds__(kCsortThreads) void hspmv_csort(
    int32_t H, int64_t m, int32_t direct, const int32_t *__restrict__ blk_c,
    const int32_t *__restrict__ blk_r, const int32_t *__restrict__ blk_v,
    const int32_t *__restrict__ vslice, const int32_t *__restrict__ cbase,
    const void *__restrict__ ent, const T *__restrict__ val, const T *__restrict__ x,
    P *__restrict__ part, S *__restrict__ spart, T *__restrict__ y,
    unsigned long long *__restrict__ trace, int32_t dyn, const int16_t *__restrict__ rexp,
    const int16_t *__restrict__ sexp, const int32_t *xexp_part, int32_t n_xexp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int32_t next_chunk;  // dyn: the workgroup's chunk queue head
  static_assert(!FIX || sizeof(S) == 8, "fixed-point slots are 8 bytes");
  constexpr int NW = kCsortThreads / kWave;
  const int b = blockIdx.x;
  unsigned long long *tr = trace ? trace + (int64_t)b * kCsortTraceSlots : nullptr;
  if (tr && threadIdx.x == 0) {  // diagnostic builds only (DevCsort.trace)
    tr[0] = __builtin_amdgcn_s_memrealtime();
    tr[2] = __builtin_amdgcn_s_getreg((31 << 11) | 20) |
            ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 32);
  }
  const int h = b % H;  // the column part; its rows: the part's own row block
  const int32_t c0 = blk_c[b], c1 = blk_c[b + 1];
  const int32_t r0 = blk_r[2 * b], r1 = blk_r[2 * b + 1];
  const int32_t v0 = blk_v[b], v1 = blk_v[b + 1];
  const int32_t nr = r1 - r0, nv = v1 - v0;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
  // FIX: the SpMV's x exponent (every wave reduces the pre-pass's maxima:
  // no LDS, no extra barrier); a non-finite x -> the S-slot fallback
  int32_t xe = 0;
  if constexpr (FIX) xe = wave_xexp(xexp_part, n_xexp, lane);
  const bool fixp = FIX && xe != kCsortXexpNonFinite;  // uniform over the grid
  // an x below 2^-1000 is scaled as if it reached 2^-1000 (M stays normal)
  const int32_t E = fixp ? kCsortFixBits - max(xe, -1000) : 0;
  const double M = fixp ? __builtin_ldexp(1.5, 52 - E) : 0.0;
  for (int32_t i = threadIdx.x; i <= nr + nv; i += kCsortThreads)  // + dummy; 0 = +0.0 = integer 0
    reinterpret_cast<S *>(smem)[i] = S(0);
  if (threadIdx.x == 0) next_chunk = c0 + NW;
  __syncthreads();
  if (tr && threadIdx.x == 0) tr[3] = __builtin_amdgcn_s_memrealtime();
  int32_t cn_done;
  if (fixp)
    cn_done = csort_chunks<T, S, U, NT, PF, WIDE, FIX>(c0, c1, wid, lane, dyn, &next_chunk, cbase, ent, val,
                                                       x, smem, M);
  else
    cn_done = csort_chunks<T, S, U, NT, PF, WIDE, false>(c0, c1, wid, lane, dyn, &next_chunk, cbase, ent,
                                                         val, x, smem, 0.0);
  if (tr && lane == 0) {  // this wave's end and chunk count (its LDS adds issued)
    tr[4 + wid] = __builtin_amdgcn_s_memrealtime();
    tr[4 + NW + wid] = (unsigned long long)cn_done;
  }
  __syncthreads();
  if (tr && threadIdx.x == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
  // FIX: the slot of row r is at scale 2^(E + rexp[r]) (the fallback: 2^rexp[r])
  auto val_at = [&](int32_t i, int32_t e) -> S {
    if constexpr (FIX) {
      if (fixp) return slot_value<S, true>(smem, i, E + e);
      return (S)__builtin_ldexp((double)reinterpret_cast<const S *>(smem)[i], -e);
    } else {
      return slot_value<S, false>(smem, i, 0);
    }
  };
  if (direct) {  // one column part, no long rows: y straight from the slots
    for (int32_t i = threadIdx.x; i < nr; i += kCsortThreads)
      y[r0 + i] = (T)val_at(i, FIX ? (int32_t)rexp[r0 + i] : 0);
    return;
  }
  P *out = part + (int64_t)h * m + r0;
  for (int32_t i = threadIdx.x; i < nr; i += kCsortThreads) out[i] = (P)val_at(i, FIX ? (int32_t)rexp[r0 + i] : 0);
  for (int32_t i = threadIdx.x; i < nv; i += kCsortThreads) {
    const int32_t sl = vslice[v0 + i];
    spart[sl] = val_at(nr + i, FIX ? (int32_t)sexp[sl] : 0);
  }
}

// Pre-pass of the fixed-point csort (one per SpMV, before it): per block the
// max frexp exponent of |x| (|x| < 2^e), kCsortXexpNonFinite if the block saw
// an Inf or a NaN -- or an |x| >= 2^1020, whose rounding constant M would
// overflow (that SpMV then adds in fp64 slots); zeros do not count.  Block j
// takes chunks j, j + grid, ... of kXexpChunk entries, each of its 1024
// threads 8 of a chunk; VEC (x 16-byte aligned): all 8 in 16-byte loads
// issued before any is used -- one memory round trip per chunk, 16 waves
// per CU in flight (a strided scalar loop of 256-thread blocks ran C5's 8 MB
// in 12.5 us, profiles/r06c; 32 per thread of 256 still 5.7 us average,
// r06d).  Every csort wave max-reduces the n_xexp block results itself
// (wave_xexp).
constexpr int kXexpThreads = 1024;
constexpr int kXexpPerThread = 8;
constexpr int64_t kXexpChunk = kXexpThreads * kXexpPerThread;
static_assert(kXexpChunk == kCsortXexpChunk, "the host sizes the pre-pass grid by kCsortXexpChunk");

template <typename T, bool VEC>
__global__ __launch_bounds__(kXexpThreads) void hspmv_csort_xexp(int64_t n, const T *__restrict__ x,
                                                                 int32_t *__restrict__ out) {
  __shared__ int32_t wmax[kXexpThreads / kWave];
  int32_t e = -0x40000000;
  for (int64_t c0 = (int64_t)blockIdx.x * kXexpChunk; c0 < n; c0 += (int64_t)gridDim.x * kXexpChunk) {
    if (VEC && c0 + kXexpChunk <= n) {
      constexpr int V = 16 / (int)sizeof(T), L = kXexpPerThread / V;
      typedef T tv __attribute__((ext_vector_type(V)));
      const tv *p = reinterpret_cast<const tv *>(x + c0) + threadIdx.x;
      tv v[L];
#pragma unroll
      for (int j = 0; j < L; ++j) v[j] = p[j * kXexpThreads];
#pragma unroll
      for (int j = 0; j < L; ++j)
#pragma unroll
        for (int k = 0; k < V; ++k) e = xexp_max(e, (double)v[j][k]);
    } else {
      for (int64_t i = c0 + threadIdx.x; i < min(n, c0 + kXexpChunk); i += kXexpThreads)
        e = xexp_max(e, (double)x[i]);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) e = max(e, __shfl_xor(e, off, kWave));
  if ((threadIdx.x & (kWave - 1)) == 0) wmax[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x < kWave) {
    e = threadIdx.x < kXexpThreads / kWave ? wmax[threadIdx.x] : -0x40000000;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) e = max(e, __shfl_xor(e, off, kWave));
    if (threadIdx.x == 0) out[blockIdx.x] = e;
  }
}

// y[r] = part[r] + part[m + r] + ... (parts in order), except long rows:
// blocks past the row blocks sum each long row's slices (one wave per row,
// fixed lane assignment and shuffle tree).
// R rows per thread (1, 2, 4): R-element partial loads (16 / 32 bytes for
// R = 2 / 4; m a multiple of R keeps every part's rows aligned).
template <typename T, typename S, typename P, int R>
__global__ __launch_bounds__(256) void hspmv_csort_finish(
    int64_t m, int32_t H, int64_t row_blocks, const P *__restrict__ part,
    const uint32_t *__restrict__ long_mask, int32_t n_long, const int32_t *__restrict__ long_row,
    const int32_t *__restrict__ long_cs, const S *__restrict__ spart, T *__restrict__ y) {
  if ((int64_t)blockIdx.x < row_blocks) {
    if constexpr (R > 1) {
      typedef S sr __attribute__((ext_vector_type(R)));
      typedef P pr __attribute__((ext_vector_type(R)));
      typedef T tr __attribute__((ext_vector_type(R)));
      const int64_t r = R * ((int64_t)blockIdx.x * 256 + threadIdx.x);
      if (r >= m) return;
      const pr p0 = *reinterpret_cast<const pr *>(part + r);
      sr s;
#pragma unroll
      for (int j = 0; j < R; ++j) s[j] = (S)p0[j];
      for (int32_t h = 1; h < H; ++h) {
        const pr q = *reinterpret_cast<const pr *>(part + (int64_t)h * m + r);
#pragma unroll
        for (int j = 0; j < R; ++j) s[j] += (S)q[j];
      }
      // R <= 4 rows never straddle a 32-row mask word (r is a multiple of R)
      const uint32_t lm = long_mask ? (long_mask[r >> 5] >> (r & 31)) & ((1u << R) - 1u) : 0u;
      if (lm == 0u) {
        tr o;
#pragma unroll
        for (int j = 0; j < R; ++j) o[j] = (T)s[j];
        *reinterpret_cast<tr *>(y + r) = o;
      } else {  // a long row's y comes from its slices
#pragma unroll
        for (int j = 0; j < R; ++j)
          if (!((lm >> j) & 1u)) y[r + j] = (T)s[j];
      }
      return;
    } else {
      const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
      if (r >= m) return;
      if (long_mask && ((long_mask[r >> 5] >> (r & 31)) & 1u)) return;
      S s = (S)part[r];
      for (int32_t h = 1; h < H; ++h) s += (S)part[(int64_t)h * m + r];
      y[r] = (T)s;
      return;
    }
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t j = ((int64_t)blockIdx.x - row_blocks) * 4 + (threadIdx.x >> 6);
  if (j >= n_long) return;
  S s = S(0);
  for (int32_t i = long_cs[j] + lane; i < long_cs[j + 1]; i += kWave) s += spart[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
  if (lane == 0) y[long_row[j]] = (T)s;
}

template <typename T, typename S, typename P, int R>
void launch_finish(const DevCsort &c, const P *part, const S *spart, T *y, hipStream_t st) {
  const int64_t lb = ((int64_t)c.n_long + 3) / 4;
  const int64_t rb = (c.m / R + 255) / 256;
  hipLaunchKernelGGL((hspmv_csort_finish<T, S, P, R>), dim3((unsigned)(rb + lb)), dim3(256), 0, st, c.m, c.H,
                     rb, part, c.long_mask, c.n_long, c.long_row, c.long_cs, spart, y);
}

template <typename T, typename S, typename P, int U, bool NT, bool PF, bool WIDE>
void launch_csort_main(const DevCsort &c, const T *x, P *part, S *spart, T *y, hipStream_t st) {
  if constexpr (sizeof(S) == 8) {
    if (c.fixed) {
      const bool vec = reinterpret_cast<uintptr_t>(x) % 16 == 0;
      if (vec)
        hipLaunchKernelGGL((hspmv_csort_xexp<T, true>), dim3((unsigned)c.n_xexp), dim3(kXexpThreads), 0, st,
                           c.n_x, x, c.xexp_part);
      else
        hipLaunchKernelGGL((hspmv_csort_xexp<T, false>), dim3((unsigned)c.n_xexp), dim3(kXexpThreads), 0, st,
                           c.n_x, x, c.xexp_part);
      hipLaunchKernelGGL((hspmv_csort<T, S, P, U, NT, PF, WIDE, true>), dim3((unsigned)c.n_wg),
                         dim3(kCsortThreads), (unsigned)c.lds_bytes, st, c.H, c.m, c.direct, c.blk_c, c.blk_r,
                         c.blk_v, c.vslice, c.cbase, c.ent, static_cast<const T *>(c.val), x, part, spart, y,
                         c.trace, c.dyn ? 1 : 0, c.rexp, c.sexp, c.xexp_part, c.n_xexp);
      return;
    }
  }
  hipLaunchKernelGGL((hspmv_csort<T, S, P, U, NT, PF, WIDE, false>), dim3((unsigned)c.n_wg), dim3(kCsortThreads),
                     (unsigned)c.lds_bytes, st, c.H, c.m, c.direct, c.blk_c, c.blk_r, c.blk_v,
                     c.vslice, c.cbase, c.ent, static_cast<const T *>(c.val), x, part, spart, y,
                     c.trace, c.dyn ? 1 : 0, nullptr, nullptr, nullptr, 0);
}

template <typename T, typename S, typename P, int U, bool NT>
hipError_t launch_csort_p(const DevCsort &c, const T *x, T *y, hipStream_t st) {
  P *part = static_cast<P *>(c.part);
  S *spart = static_cast<S *>(c.spart);
  if constexpr (sizeof(T) == 8 && U % 4 != 0) {
    if (c.wide) return hipErrorInvalidValue;
    if (c.prefetch) launch_csort_main<T, S, P, U, NT, true, false>(c, x, part, spart, y, st);
    else launch_csort_main<T, S, P, U, NT, false, false>(c, x, part, spart, y, st);
  } else {
    if (c.prefetch) {
      if (c.wide) launch_csort_main<T, S, P, U, NT, true, true>(c, x, part, spart, y, st);
      else launch_csort_main<T, S, P, U, NT, true, false>(c, x, part, spart, y, st);
    } else {
      if (c.wide) launch_csort_main<T, S, P, U, NT, false, true>(c, x, part, spart, y, st);
      else launch_csort_main<T, S, P, U, NT, false, false>(c, x, part, spart, y, st);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || c.direct) return e;
  // rows per finishing thread: 4 (32-byte partial loads; C5 104.4 -> 103.5
  // us, c5r 110.0 -> 107.8 against 2, r04c/ab_c5_fin_rows.jsonl), fewer when
  // m is not a multiple or y (a caller's buffer, hspmv_bind_y_device: any
  // element-aligned pointer) is not aligned for the R-wide vector store;
  // c.fin_rows overrides (A/B)
  const int fr = c.fin_rows > 0 ? c.fin_rows : 4;
  const uintptr_t ya = reinterpret_cast<uintptr_t>(y);
  // (8 rows per thread, 32-byte partial loads: C5 / c5r t_min +0.4 ... +2.6
  // us against 4 in one process, profiles/r06l/ab_c5_fin_rows8_negative.jsonl)
  if (fr >= 4 && c.m % 4 == 0 && ya % (4 * sizeof(T)) == 0)
    launch_finish<T, S, P, 4>(c, part, spart, y, st);
  else if (fr >= 2 && c.m % 2 == 0 && ya % (2 * sizeof(T)) == 0)
    launch_finish<T, S, P, 2>(c, part, spart, y, st);
  else
    launch_finish<T, S, P, 1>(c, part, spart, y, st);
  return hipGetLastError();
}

// part32 (fp32 data over fp64 slots; the default, hspmv_csort_build.cpp):
// the column parts' row partials stored as fp32 (half the partial traffic;
// y then rounds twice on rows with entries in both parts)
template <typename T, typename S, int U, bool NT>
hipError_t launch_csort_u(const DevCsort &c, const T *x, T *y, hipStream_t st) {
  if constexpr (sizeof(T) == 4 && sizeof(S) == 8)
    if (c.part32) return launch_csort_p<T, S, float, U, NT>(c, x, y, st);
  return launch_csort_p<T, S, S, U, NT>(c, x, y, st);
}

template <typename T, typename S, bool NT>
hipError_t launch_csort_nt(const DevCsort &c, const T *x, T *y, hipStream_t st) {
  switch (c.u) {
    case 4: return launch_csort_u<T, S, 4, NT>(c, x, y, st);
    case 8: return launch_csort_u<T, S, 8, NT>(c, x, y, st);
    case 16: return launch_csort_u<T, S, 16, NT>(c, x, y, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_csort(const DevCsort &c, int dtype, const void *x, void *y, hipStream_t st) {
  if (c.m == 0) return hipSuccess;
  if (c.n_wg <= 0 || c.lds_bytes > kCsortMaxLds) return hipErrorInvalidValue;
  if (c.fixed && (c.slot32 || !c.rexp || !c.xexp_part || c.n_xexp <= 0 || c.n_xexp > kCsortXexpBlocks))
    return hipErrorInvalidValue;
  if (dtype == 1) {
    if (c.slot32) return hipErrorInvalidValue;
    return c.nontemporal ? launch_csort_nt<double, double, true>(c, (const double *)x, (double *)y, st)
                         : launch_csort_nt<double, double, false>(c, (const double *)x, (double *)y, st);
  }
  const float *xf = (const float *)x;
  float *yf = (float *)y;
  if (c.slot32)
    return c.nontemporal ? launch_csort_nt<float, float, true>(c, xf, yf, st)
                         : launch_csort_nt<float, float, false>(c, xf, yf, st);
  return c.nontemporal ? launch_csort_nt<float, double, true>(c, xf, yf, st)
                       : launch_csort_nt<float, double, false>(c, xf, yf, st);
}

}  // namespace hspmv
