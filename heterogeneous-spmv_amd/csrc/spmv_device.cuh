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
// the x gather (x[col] := 1), 3 = both; 16 = skip the x-dictionary staging
// (and its barrier), 32 = the barrier without the staging loads, 256 = no y
// stores (the sums kept live), 1024 = 1-byte dictionary positions (half the
// index bytes; the bound on any position compression: C3 107.3 -> 102.7 us,
// fp32 62.1 -> 51.2, profiles/r03/ab_c3_1byte_positions_ablation.jsonl --
// run-coded positions (a run-start mask per 64 nonzeros + 2 bytes per run,
// 0.86 B/nnz on C3) measured 108.7 -> 114.2 us, fp32 62.2 -> 99.4: the
// decode's dependent loads cost more than the bytes).  Results are wrong in
// those builds.
#ifndef HSPMV_DIAG
#define HSPMV_DIAG 0
#endif

// HSPMV_DIAG & 8: per-wave phase timestamps (s_memtime) of the STREAM
// kernel into g_trace (read back by hspmv_diag_trace, stream_f64.hip).  Each
// stamp first waits for all of the wave's outstanding loads, so the traced
// build measures a serialised wave; results are correct.
constexpr int kTraceWaves = 1 << 17;
constexpr int kTraceSlots = 8;
#if (HSPMV_DIAG & 8)
static __device__ unsigned long long g_trace[kTraceWaves * kTraceSlots];
__device__ __forceinline__ unsigned long long diag_stamp() {
  unsigned long long t;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(t)::"memory");
  return t;
}
#define HSPMV_TRACE(ts, i, v)            \
  do {                                   \
    if ((ts) != nullptr && lane == 0) (ts)[i] = (v); \
  } while (0)
#else
#define HSPMV_TRACE(ts, i, v) \
  do {                        \
  } while (0)
#endif
// HSPMV_DIAG & 512: per-workgroup timeline of the CSR3 kernel -- slot 0 the
// workgroup's start, 1..4 each wave's end (after its y store is issued), 6
// HW_ID, 7 XCC_ID (s_memrealtime, 100 MHz; no waits, results correct) --
// into g_trace[block * kTraceSlots] (tools/block_trace.py).
#if (HSPMV_DIAG & 512)
#if !(HSPMV_DIAG & 8)
static __device__ unsigned long long g_trace[kTraceWaves * kTraceSlots];
#endif
__device__ __forceinline__ unsigned long long diag_realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#endif

constexpr int kWave = 64;
#ifndef HSPMV_COOP_GROUPS
#define HSPMV_COOP_GROUPS 1
#endif
// kSerialMax (hspmv_internal.h): the longest row summed serially by one lane.
// The kernels take the bound as an argument (DevPlan.serial_max): kSerialMax,
// or INT32_MAX for hspmv_options.deterministic = 3, where every row is summed
// serially -- omp_spmv's order for every row, the long ones by one lane.
constexpr int kNumXcd = 8;

// PAD: a wave's product buffer holds chunk position i at lds_ix(i) = i + i /
// 32 -- one pad element per 32 -- so that the lanes of an ordered sum, each
// walking its own row with rows one row length apart, do not meet in one
// LDS bank.  Rows of 32 nonzeros put every lane of a chunk on one bank
// (fp32 32-way; fp64 8-way per 256-nonzero chunk), and the ordered sums were
// 40 % of the dense-32x32-block matrix's time (HSPMV_DIAG 1 ablation,
// profiles/r05h/ab_blocks32_ablation.jsonl).  The index math and the bigger
// buffer cost latency and LDS elsewhere (C3 fp32 +8 %, C4 fp32 +8 % with
// padding everywhere, profiles/r05j/ab_lds_pad.jsonl), so the planner pads
// only STREAM launches whose rows are conflicting (LaunchPlan.lds_pad).
template <bool PAD>
__device__ __forceinline__ int32_t lds_ix(int32_t i) { return PAD ? i + (i >> 5) : i; }
template <int U, bool PAD>
constexpr int wave_lds() {  // elements of one wave's product buffer
  return kWave * U + (PAD ? 2 * U : 0);
}

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

// One DPP move of v (both dwords for fp64); lanes the pattern does not feed
// read 0.
template <int CTRL, int ROW_MASK, typename T>
__device__ __forceinline__ T dpp_move(T v) {
  if constexpr (sizeof(T) == 8) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROW_MASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, ROW_MASK, 0xf, false);
    return __builtin_bit_cast(T, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  } else {
    return __builtin_bit_cast(
        T, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, false));
  }
}

// Wave sum by DPP (row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast 15/31 across rows: an inclusive scan whose lane 63 holds the
// total), returned wave-uniform.  No LDS round trips, unlike __shfl_xor
// (ds_bpermute): the cooperative rows' reductions are on the critical path
// of each chunk (mid-density rows, profiles/r02z*).
// Lane l's value of v, wave-uniform (v_readlane; l wave-uniform).
template <typename T>
__device__ __forceinline__ T lane_value(T v, int l) {
  if constexpr (sizeof(T) == 8) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
  }
}

// Sums of the four 16-lane DPP rows: lane 16 q + 15 holds row q's total.
template <typename T>
__device__ __forceinline__ T row16_sum_dpp(T v) {
  v += dpp_move<0x111, 0xf>(v);
  v += dpp_move<0x112, 0xf>(v);
  v += dpp_move<0x114, 0xf>(v);
  v += dpp_move<0x118, 0xf>(v);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum_dpp(T v) {
  v += dpp_move<0x111, 0xf>(v);
  v += dpp_move<0x112, 0xf>(v);
  v += dpp_move<0x114, 0xf>(v);
  v += dpp_move<0x118, 0xf>(v);
  v += dpp_move<0x142, 0xa>(v);
  v += dpp_move<0x143, 0xc>(v);
  return lane_value(v, 63);
}

// Bijective XCD-aware block order (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective").  Blocks b and b+8 share an XCD under round-robin
// dispatch; with chunk s > 1 each XCD takes s consecutive logical blocks in
// turn, so at any moment the 8 XCDs work on 8 adjacent runs of s blocks:
// s = nb/8 gives each XCD one contiguous eighth of the rows (x stays in
// that XCD's L2), small s keeps the whole chip's read front compact (HBM
// page locality) while rows still share x lines within an XCD.  s <= 1 is
// the dispatch order.  Blocks past the last full 8*s span keep their index.
__device__ __forceinline__ uint32_t xcd_chunk_remap(uint32_t b, uint32_t nb, uint32_t s) {
  if (s <= 1) return b;
  const uint32_t span = kNumXcd * s;
  if (b >= (nb / span) * span) return b;
  const uint32_t i = b / kNumXcd, x = b % kNumXcd;
  return (i / s) * span + x * s + (i % s);
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

// Scalar (s_load) read of 8 bytes at p + byte_off; p and byte_off must be
// wave-uniform.
__device__ __forceinline__ int64_t sload_i64(const void *p, uint64_t byte_off) {
  const uint64_t v = reinterpret_cast<uint64_t>(p) + byte_off;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  typedef __attribute__((address_space(4))) const int64_t ci64;
  return *(ci64 *)(((uint64_t)hi << 32) | lo);
}

// Ordered sum of lds[lo..hi) into acc, left to right: the LDS reads are
// issued 4 at a time (one LDS latency per 4 nonzeros instead of per nonzero),
// the last 1-3 together (C4's 10-nonzero rows: 54.2 -> 51.7 us,
// profiles/r01_ab_ordered_sum_tail.jsonl), but the additions stay in
// sequence, so the rounding is omp_spmv's.
// (An 8-wide batch for the dictionary kernels measured flat on C3, -0.4 %;
// 8-wide clamped batches everywhere slower: C3 +13 %, honeycomb +5 %.)
// lds holds chunk position i (nonzero c + i) at lds_ix(i).
template <bool PAD, typename T>
__device__ __forceinline__ T ordered_sum(T acc, const T *lds, int32_t c, int32_t lo, int32_t hi) {
  int32_t k = lo;
  for (; k + 4 <= hi; k += 4) {
    const T a0 = lds[lds_ix<PAD>(k - c)], a1 = lds[lds_ix<PAD>(k + 1 - c)], a2 = lds[lds_ix<PAD>(k + 2 - c)],
            a3 = lds[lds_ix<PAD>(k + 3 - c)];
    acc = acc + a0;
    acc = acc + a1;
    acc = acc + a2;
    acc = acc + a3;
  }
  if (k < hi) {  // the last 1-3 in one LDS round trip (clamped reads, selected adds)
    const T a0 = lds[lds_ix<PAD>(k - c)], a1 = lds[lds_ix<PAD>(min(k + 1, hi - 1) - c)],
            a2 = lds[lds_ix<PAD>(min(k + 2, hi - 1) - c)];
    acc = acc + a0;
    if (k + 1 < hi) acc = acc + a1;
    if (k + 2 < hi) acc = acc + a2;
  }
  return acc;
}

// Row bounds of a 64-row group for this lane (0, 0 past g1).  Issued one
// group ahead by the kernels, so a wave's next col/val loads never wait on
// a row-pointer round trip.
__device__ __forceinline__ void group_bounds(const int32_t *__restrict__ rp, int32_t g0,
                                             int32_t g1, int lane, int32_t &beg, int32_t &end) {
  const int32_t row = g0 + lane;
  const bool valid = row < g1;
  beg = valid ? rp[row] : 0;
  end = valid ? rp[row + 1] : 0;
}

// Where a row kernel reads column indices from (DevCSR's col_idx, or the
// 16-bit offsets + block bases + high-bit planes of the col16 format).
struct ColSrc {
  const int32_t *ci;
  const uint16_t *c16;
  const int32_t *cbase;
  const uint64_t *cplanes;
  int32_t n_planes, plane_words;
};

// x window of a STREAM group (XW): x[lo, lo + w) staged in the wave's LDS
// slot `xs`, so the group's gathers are LDS reads; w == 0: global gathers.
template <typename T>
struct XWin {
  const T *xs;
  int32_t lo, w;
};

// One wavefront computes rows [g0, g1), g1 - g0 <= 64, whose bounds
// (group_bounds) are in beg/end.  lds: kWave*U elements private to this
// wave.  Per chunk of 64*U nonzeros: stage A loads col/val (coalesced),
// stage B gathers x[col] (from the LDS window when XW and win.w > 0), stage
// C forms the products into LDS; then the row sums.  PF (software
// pipelining): the next chunk's stage A is issued between this chunk's
// stage B and C, so its latency overlaps the gather and the sums.
template <typename T, bool NT, int U, bool PF, int C16, bool XW, bool XD, bool GROUPS, bool PAD = false>
__device__ __forceinline__ void wave_rows(int32_t g0, int32_t g1, int32_t beg, int32_t end,
                                          int32_t long_t, int32_t serial_max, const ColSrc &cs,
                                          const T *__restrict__ val,
                                          const T *__restrict__ x,
                                          T *__restrict__ y, T *lds, int lane,
                                          const XWin<T> &win, bool y_nt, bool carry,
                                          int32_t gbase, unsigned long long *ts = nullptr) {
  const int32_t row = g0 + lane;
  const bool valid = row < g1;
  const int32_t len = end - beg;
  (void)ts;
  (void)win;
  const bool skip = len > long_t;
  const unsigned long long skipmask = __ballot(valid && skip);
  const unsigned long long coopmask = __ballot(valid && !skip && len > serial_max);
  const bool serial = valid && !skip && len <= serial_max;
  const gchar *xb = uniform_ptr(x);
  const bool inwin = (XW && win.w > 0) || XD;
  // x slabs: passes after the first continue each row's sum from y, so a
  // row's products are still added left to right from 0 across the passes
  T acc = (carry && valid && !skip) ? y[row] : T(0);
  // Runs of consecutive non-split rows [a, b); normally one run = the group.
  int32_t a = g0;
  while (a < g1) {
    const unsigned long long rest = skipmask & bits_from(a - g0);
    const int32_t b = rest ? g0 + (__ffsll(rest) - 1) : g1;
    if (b > a) {
      const int32_t kb = __builtin_amdgcn_readfirstlane(__shfl(beg, a - g0, kWave));
      const int32_t ke = __builtin_amdgcn_readfirstlane(__shfl(end, b - 1 - g0, kWave));
      const int32_t n_run = ke - kb;
      const unsigned long long coop = coopmask & bits_from(a - g0) & ~bits_from(b - g0);
      const bool mine = serial && row >= a && row < b;
      int32_t col[U];
      T v[U];
      const gchar *cb = (C16 || XD) ? uniform_ptr(cs.c16 + kb) : uniform_ptr(cs.ci + kb);
      const gchar *vb = uniform_ptr(val + kb);
      // (A raw-buffer form -- SGPR descriptors bounded to the run, no
      // clamp VALU -- measured 0-2.5 % slower in one-process A/B runs,
      // tools/ab.py, profiles/r01_ab_buffer_loads.jsonl.)
      auto stage_a = [&](int32_t c0, int32_t last) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          // clamp instead of branching: every load issues back to back
          const uint32_t j = (uint32_t)(c0 + min(u * kWave + lane, last));
          if constexpr (XD && (HSPMV_DIAG & 1024) != 0) {
            col[u] = (int32_t)ld_off<NT, uint8_t>(cb, j);  // ablation: 1-byte positions (wrong x)
          } else if constexpr (XD) {
            col[u] = (int32_t)ld_off<NT, uint16_t>(cb, j * 2u);  // position in the block's xs
          } else if constexpr (C16 == 2) {
            // group-base offsets: col = the 64-row group's smallest column
            // + 16-bit offset (one scalar load per group, one add here)
            col[u] = gbase + (int32_t)ld_off<NT, uint16_t>(cb, j * 2u);
          } else if constexpr (C16 == 1) {
            // col = base of the nonzero's 256-block + 16-bit offset.  The 64
            // lanes of a slice lie in at most two consecutive blocks: one
            // scalar load brings both bases (s_load, no vector memory op)
            const uint32_t e0 = (uint32_t)kb + (uint32_t)(c0 + min(u * kWave, last));
            const uint32_t ja = (uint32_t)kb + j;
            const uint32_t b0 = __builtin_amdgcn_readfirstlane(e0 >> kC16Shift);
            const int64_t bp = sload_i64(cs.cbase, (uint64_t)b0 * 4u);
            const int32_t base = ((ja >> kC16Shift) == b0) ? (int32_t)bp : (int32_t)(bp >> 32);
            int32_t high = 0;
            if (cs.n_planes > 0) {  // wave-uniform; the two words a slice spans, by s_load
              const uint32_t w0 = __builtin_amdgcn_readfirstlane(e0 >> 6);
              const bool first = (ja >> 6) == w0;
              for (int p = 0; p < cs.n_planes; ++p) {
                const uint64_t at = ((uint64_t)p * (uint64_t)cs.plane_words + w0) * 8u;
                const uint64_t m0 = (uint64_t)sload_i64(cs.cplanes, at);
                const uint64_t m1 = (uint64_t)sload_i64(cs.cplanes, at + 8u);
                high |= (int32_t)(((first ? m0 : m1) >> (ja & 63u)) & 1u) << p;
              }
            }
            col[u] = base + (int32_t)ld_off<NT, uint16_t>(cb, j * 2u) + (high << 16);
          } else {
            col[u] = ld_off<NT, int32_t>(cb, j * 4u);
          }
          v[u] = ld_off<NT, T>(vb, j * (uint32_t)sizeof(T));
        }
      };
      if constexpr (PF) {
        if (n_run > 0) stage_a(0, min(kWave * U, n_run) - 1);
      }
      for (int32_t c0 = 0; c0 < n_run; c0 += kWave * U) {
        const int32_t last = min(kWave * U, n_run - c0) - 1;
        if constexpr (!PF) stage_a(c0, last);
#if (HSPMV_DIAG & 8)
        if (c0 == 0) HSPMV_TRACE(ts, 2, diag_stamp());
#endif
        T xv[U], vv[U];
        if (inwin) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            xv[u] = XD ? win.xs[col[u]] : win.xs[col[u] - win.lo];
            vv[u] = v[u];
          }
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if constexpr ((HSPMV_DIAG & 2) != 0)
              xv[u] = T(col[u] & 1) + T(1);
            else
              xv[u] = ld_off<false, T>(xb, (uint32_t)col[u] * (uint32_t)sizeof(T));
            vv[u] = v[u];
          }
        }
        if constexpr (PF) {
          __builtin_amdgcn_sched_barrier(0);
          const int32_t cn = c0 + kWave * U;
          stage_a(cn < n_run ? cn : n_run - 1, cn < n_run ? min(kWave * U, n_run - cn) - 1 : 0);
          __builtin_amdgcn_sched_barrier(0);
        }
#if (HSPMV_DIAG & 8)
        if (c0 == 0) HSPMV_TRACE(ts, 3, diag_stamp());
#endif
#pragma unroll
        for (int u = 0; u < U; ++u) lds[lds_ix<PAD>(u * kWave + lane)] = vv[u] * xv[u];
        wave_sync();
        const int32_t c = kb + c0;
        if constexpr ((HSPMV_DIAG & 1) != 0) {
          if (mine && max(beg, c) < min(end, c + last + 1)) acc += lds[lds_ix<PAD>(max(beg, c) - c)];
        } else {
          if (mine) acc = ordered_sum<PAD>(acc, lds, c, max(beg, c), min(end, c + last + 1));
        }
        // only the cooperative rows this chunk touches (rows are contiguous:
        // the others would add nothing), bounds by readlane (scalar)
        unsigned long long cm = coop ? coop & __ballot(end > c && beg <= c + last) : 0ull;
        // three or more pieces (rows of 33..~100 nonzeros): four at a time,
        // one 16-lane DPP row each.  CSR3 kernel only -- the tasks that
        // mid-density CSR matrices run as (hspmv_tables.cpp build_tasks): in
        // the STREAM kernel the extra code cost the honeycomb matrix 4 %
        // (161 -> 168 us) with no such rows at all (r02z9).  d33 173 ->
        // 137 us, d48 132 -> 109, d64 103 -> 95 (profiles/r02z8).
        if (GROUPS && __popcll(cm) >= 3) {
          const int g = lane >> 4, gl = lane & 15;
          while (cm) {
            int rq[4];
            int32_t lq[4], hq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              rq[q] = -1;
              lq[q] = 0;
              hq[q] = 0;
              if (cm) {  // wave-uniform
                rq[q] = __ffsll(cm) - 1;
                cm &= cm - 1;
                lq[q] = max(__builtin_amdgcn_readlane(beg, rq[q]), c);
                hq[q] = min(__builtin_amdgcn_readlane(end, rq[q]), c + last + 1);
              }
            }
            const int32_t lo = g == 0 ? lq[0] : (g == 1 ? lq[1] : (g == 2 ? lq[2] : lq[3]));
            const int32_t hi = g == 0 ? hq[0] : (g == 1 ? hq[1] : (g == 2 ? hq[2] : hq[3]));
            T s = T(0);
            for (int32_t k = lo + gl; k < hi; k += 16) s += lds[lds_ix<PAD>(k - c)];
            s = row16_sum_dpp(s);
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (rq[q] >= 0) {  // wave-uniform
                const T t = lane_value(s, 16 * q + 15);
                if (lane == rq[q]) acc += t;
              }
          }
        }
        while (cm) {
          const int r = __ffsll(cm) - 1;
          cm &= cm - 1;
          const int32_t lo = max(__builtin_amdgcn_readlane(beg, r), c);
          const int32_t hi = min(__builtin_amdgcn_readlane(end, r), c + last + 1);
          if (lo < hi) {  // wave-uniform
            T s = T(0);
            for (int32_t k = lo + lane; k < hi; k += kWave) s += lds[lds_ix<PAD>(k - c)];
            s = wave_sum_dpp(s);
            if (lane == r) acc += s;
          }
        }
        wave_sync();
#if (HSPMV_DIAG & 8)
        if (c0 == 0) HSPMV_TRACE(ts, 4, diag_stamp());
        if (c0 + kWave * U >= n_run) HSPMV_TRACE(ts, 7, (unsigned long long)(c0 / (kWave * U) + 1));
#endif
      }
    }
    a = b + 1;
  }
#if (HSPMV_DIAG & 8)
  HSPMV_TRACE(ts, 5, diag_stamp());
#endif
  if constexpr ((HSPMV_DIAG & 256) != 0) {  // ablation: no y stores (kept live)
    if (valid && !skip && acc == T(12345.678)) y[row] = acc;
  } else if (valid && !skip) {
    if (y_nt)  // HBM-resident: streaming stores (bw_probe3/4: y writes cost ~20 % of time)
      __builtin_nontemporal_store(acc, y + row);
    else
      y[row] = acc;
  }
}

// Stages x[lo, lo + w) (w <= kXWin) into the wave's LDS window slot.  The
// loads are contiguous (coalesced), unlike the gathers they replace.
template <typename T>
__device__ __forceinline__ void stage_xwin(T *xs, const T *__restrict__ x, int32_t lo, int32_t w,
                                           int lane) {
  const gchar *xb = uniform_ptr(x + lo);
  T t[kXWin / kWave];
#pragma unroll
  for (int i = 0; i < kXWin / kWave; ++i) {
    const int32_t e = min(i * kWave + lane, w - 1);
    t[i] = ld_off<false, T>(xb, (uint32_t)e * (uint32_t)sizeof(T));
  }
#pragma unroll
  for (int i = 0; i < kXWin / kWave; ++i) xs[i * kWave + lane] = t[i];
  wave_sync();
}

// Block x dictionary (XD): the x entries a workgroup's rows reference,
// as runs of consecutive columns.  blk[b], blk[b+1] bound block b's records
// in runs: {x_start, lds_off} per run, then a sentinel {0, total}; run i
// stages x[x_start, x_start + len) at xs[lds_off ...], len = the next
// record's lds_off - lds_off.  The col stream then holds each nonzero's
// 16-bit position in xs (the host builds both, hspmv_xdict.cpp build_xdict).
struct XDict {
  const int32_t *blk;
  const int2 *runs;
};

// The workgroup stages its dictionary into xs (NTH threads, contiguous loads
// per run instead of one gather per nonzero) and waits at a block barrier.
// Every wave of the block must call this (before any early return).
template <typename T, int NTH>
__device__ __forceinline__ void stage_xdict(T *xs, const T *__restrict__ x, const XDict &xd,
                                            int64_t blk, int tid) {
  constexpr int kBatch = 8;
  if constexpr ((HSPMV_DIAG & 16) != 0) return;  // ablation: no staging, no barrier
  if constexpr ((HSPMV_DIAG & 32) != 0) {        // ablation: the barrier only
    __syncthreads();
    return;
  }
  // HSPMV_DIAG & 64 / 128 (A/B, results correct): the staging waves at
  // issue priority 3 / 1 until the barrier, ahead of other blocks' streams
  if constexpr ((HSPMV_DIAG & 64) != 0) __builtin_amdgcn_s_setprio(3);
  if constexpr ((HSPMV_DIAG & 128) != 0) __builtin_amdgcn_s_setprio(1);
  const int64_t rr = sload_i64(xd.blk, (uint64_t)blk * 4u);
  const int32_t r0 = (int32_t)rr;
  const int32_t nr = (int32_t)(rr >> 32) - r0 - 1;  // runs (<= 63), then the sentinel
  const int lane = tid & (kWave - 1);
  int2 rec = make_int2(0, 0);
  if (nr >= 0 && lane <= nr) rec = xd.runs[r0 + lane];
  const int32_t total = nr >= 0 ? __builtin_amdgcn_readlane(rec.y, nr) : 0;
  const int32_t delta = rec.x - rec.y;  // x index = xs index + delta inside the run
  const gchar *xb = uniform_ptr(x);
  for (int32_t e0 = 0; e0 < total; e0 += NTH * kBatch) {  // block-uniform
    int32_t e[kBatch], d[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      e[j] = e0 + j * NTH + tid;
      d[j] = 0;
    }
    for (int r = 0; r < nr; ++r) {  // runs are sorted by lds_off: the last run starting <= e
      const int32_t o = __builtin_amdgcn_readlane(rec.y, r);
      const int32_t dl = __builtin_amdgcn_readlane(delta, r);
#pragma unroll
      for (int j = 0; j < kBatch; ++j) d[j] = e[j] >= o ? dl : d[j];
    }
    T v[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j)
      v[j] = ld_off<false, T>(xb, (uint32_t)(min(e[j], total - 1) + d[j]) * (uint32_t)sizeof(T));
#pragma unroll
    for (int j = 0; j < kBatch; ++j)
      if (e[j] < total) xs[e[j]] = v[j];
  }
  __syncthreads();
  if constexpr ((HSPMV_DIAG & (64 | 128)) != 0) __builtin_amdgcn_s_setprio(0);
}

// STREAM: wave w walks `groups` consecutive 64-row groups starting at row
// w * groups * 64, loading the next group's row pointers before streaming
// the current one.  XW: groups whose x window (xwin[g] = {lo, w}) fits
// kXWin entries gather from an LDS copy of it.
template <typename T, bool NT, int U, bool PF, int C16, bool XW, bool XD, int W = 4, bool PAD = false>
__global__ __launch_bounds__(W * 64) void hspmv_csr_stream(
    int32_t m, int32_t long_t, int32_t serial_max, uint32_t xcd_chunk, int32_t groups, int32_t y_nt,
    int32_t carry,
    const int32_t *__restrict__ rp, ColSrc cs, const int2 *__restrict__ xwin, XDict xd,
    const T *__restrict__ val, const T *__restrict__ x, T *__restrict__ y) {
  static_assert(!XD || W == 4, "dictionaries are planned for 256-row blocks");
  __shared__ T lds[W * wave_lds<U, PAD>()];
  __shared__ T xlds[XW ? W * kXWin : 1];
  extern __shared__ __attribute__((aligned(16))) unsigned char xdyn[];  // XD: the block's xs
  const int wid = threadIdx.x >> 6;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t blk = xcd_chunk_remap(blockIdx.x, gridDim.x, xcd_chunk);
  // XD (groups == 1): the block's 256 rows share one staged dictionary; the
  // only block barrier of the kernel is at the end of the staging.
  if constexpr (XD) stage_xdict<T, 256>(reinterpret_cast<T *>(xdyn), x, xd, blk, threadIdx.x);
  int64_t g0 = (blk * W + wid) * (int64_t)groups * kWave;
  if (g0 >= m) return;  // wave-uniform
  const int64_t gend = min<int64_t>(g0 + (int64_t)groups * kWave, m);
  T *my = lds + wid * wave_lds<U, PAD>();
  unsigned long long *ts = nullptr;
#if (HSPMV_DIAG & 8)
  const int64_t wv = blk * W + wid;
  if (wv < kTraceWaves) ts = g_trace + wv * kTraceSlots;
  HSPMV_TRACE(ts, 0, diag_stamp());
  {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    HSPMV_TRACE(ts, 6, (unsigned long long)hw);
  }
#endif
  int32_t beg, end;
  group_bounds(rp, (int32_t)g0, (int32_t)min<int64_t>(g0 + kWave, gend), lane, beg, end);
#if (HSPMV_DIAG & 8)
  HSPMV_TRACE(ts, 1, diag_stamp());
#endif
  while (true) {
    const int32_t g1 = (int32_t)min<int64_t>(g0 + kWave, gend);
    XWin<T> win{XD ? reinterpret_cast<const T *>(xdyn) : nullptr, 0, 0};
    if constexpr (XW) {
      const int64_t wv = sload_i64(xwin, (uint64_t)(g0 / kWave) * 8u);
      win.lo = (int32_t)wv;
      win.w = (int32_t)(wv >> 32);
      win.xs = xlds + wid * kXWin;
      if (win.w > 0) stage_xwin(xlds + wid * kXWin, x, win.lo, win.w, lane);
    }
    int32_t nbeg = 0, nend = 0;
    if (g1 < gend) group_bounds(rp, g1, (int32_t)min<int64_t>(g1 + kWave, gend), lane, nbeg, nend);
    int32_t gbase = 0;
    if constexpr (C16 == 2) gbase = (int32_t)sload_i64(cs.cbase, (uint64_t)(g0 / kWave) * 4u);
    wave_rows<T, NT, U, PF, C16, XW, XD, false, PAD>((int32_t)g0, g1, beg, end, long_t, serial_max, cs, val,
                                                     x, y, my,
                                         lane, win, y_nt != 0, carry != 0, gbase, ts);
    ts = nullptr;  // trace the first group only
    if (g1 >= gend) break;
    g0 = g1;
    beg = nbeg;
    end = nend;
  }
}

template <typename T, bool NT, int U, bool PF, int C16, int W, bool XW, bool XD>
__global__ __launch_bounds__(W * 64) void hspmv_csr3(
    int32_t n_tasks, int32_t long_t, int32_t serial_max, uint32_t xcd_chunk, int32_t y_nt, int32_t carry,
    int32_t align,
    const int32_t *__restrict__ task_start, const int2 *__restrict__ xwin, XDict xd,
    const int32_t *__restrict__ rp, ColSrc cs, const T *__restrict__ val,
    const T *__restrict__ x, T *__restrict__ y) {
  __shared__ T lds[W * wave_lds<U, false>()];
  __shared__ T xlds[XW ? W * kXWin : 1];
  extern __shared__ __attribute__((aligned(16))) unsigned char xdyn[];  // XD: the block's xs
  const int wid = threadIdx.x >> 6;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t blk = xcd_chunk_remap(blockIdx.x, gridDim.x, xcd_chunk);
#if (HSPMV_DIAG & 512)
  unsigned long long *bt = blk < kTraceWaves ? g_trace + blk * kTraceSlots : nullptr;
  if (bt && threadIdx.x == 0) {
    bt[0] = diag_realtime();
    bt[6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    bt[7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
#endif
  // XD: the W packed tasks of the block share one staged dictionary (loads
  // of the task / row bounds and of the first chunk issued ahead of the
  // staging measured -0.3 ... -0.6 % and cost 20 VGPRs: profiles/r05c,
  // r05d; removed)
  if constexpr (XD) stage_xdict<T, W * 64>(reinterpret_cast<T *>(xdyn), x, xd, blk, threadIdx.x);
  const int64_t t = blk * W + wid;
  if (t >= n_tasks) return;
#if (HSPMV_DIAG & 8)
  const unsigned long long tb_stamp = diag_stamp();
#endif
  // both task bounds in one scalar load (K$), not a vector round trip
  const int64_t tb = sload_i64(task_start, (uint64_t)t * 4u);
  const int32_t r0 = (int32_t)tb;
  const int32_t r1 = (int32_t)(tb >> 32);
  if (r0 >= r1) return;
  T *my = lds + wid * wave_lds<U, false>();
  // group-base columns: one base per packed task
  int32_t gbase = 0;
  if constexpr (C16 == 2) gbase = (int32_t)sload_i64(cs.cbase, (uint64_t)t * 4u);
  XWin<T> win{XD ? reinterpret_cast<const T *>(xdyn) : nullptr, 0, 0};
  if constexpr (XW) {  // the task's x window (packed tasks: <= 64 rows)
    const int64_t wv = sload_i64(xwin, (uint64_t)t * 8u);
    win.lo = (int32_t)wv;
    win.w = (int32_t)(wv >> 32);
    win.xs = xlds + wid * kXWin;
    if (win.w > 0) stage_xwin(xlds + wid * kXWin, x, win.lo, win.w, lane);
  }
  unsigned long long *ts = nullptr;
#if (HSPMV_DIAG & 8)
  if (t < kTraceWaves) ts = g_trace + t * kTraceSlots;
  HSPMV_TRACE(ts, 0, tb_stamp);
  HSPMV_TRACE(ts, 6, (unsigned long long)(r1 - r0));
#endif
  // align: groups end on multiples of 64 rows (the SSR plan's aligned
  // pieces: every y store but an SSR's first and last covers whole lines)
  const int32_t g1_first = min(align ? (r0 & ~(kWave - 1)) + kWave : r0 + kWave, r1);
  int32_t beg, end;
  group_bounds(rp, r0, g1_first, lane, beg, end);
#if (HSPMV_DIAG & 8)
  HSPMV_TRACE(ts, 1, diag_stamp());
#endif
  for (int32_t g0 = r0, g1 = g1_first; g0 < r1; g0 = g1, g1 = min(g1 + kWave, r1)) {
    int32_t nbeg = 0, nend = 0;
    if (g1 < r1) group_bounds(rp, g1, min(g1 + kWave, r1), lane, nbeg, nend);
    wave_rows<T, NT, U, PF, C16, XW, XD, HSPMV_COOP_GROUPS != 0>(g0, g1, beg, end, long_t, serial_max, cs, val,
                                                                 x, y, my, lane,
                                         win, y_nt != 0, carry != 0, gbase, ts);
    ts = nullptr;
    beg = nbeg;
    end = nend;
  }
#if (HSPMV_DIAG & 512)
  if (bt && lane == 0 && wid < 4) bt[1 + wid] = diag_realtime();
#endif
}

// ------------------------------------------------------------------ launchers

inline ColSrc col_src(const DevCSR &A) {
  return ColSrc{A.col_idx, A.col16, A.cbase, A.cplanes, A.n_cplanes, A.cplane_words};
}

template <typename T, bool NT, int U, bool PF, int C16, bool XD>
void launch_rows_u(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const T *x, T *y,
                   hipStream_t st) {
  const T *val = static_cast<const T *>(A.val);
  const ColSrc cs = col_src(A);
  const XDict xd{dp.xd_blk, reinterpret_cast<const int2 *>(dp.xd_runs)};
  // dynamic LDS: the block's x dictionary (XD), or occupancy experiments (HSPMV_DYNLDS)
  const unsigned dyn = XD ? (unsigned)dp.xd_lds_bytes + (unsigned)p.dyn_lds : (unsigned)p.dyn_lds;
  if (p.kernel == kStream) {
    const int2 *xw = reinterpret_cast<const int2 *>(dp.xwin);
#define HSPMV_STREAM(C, XW, XDX, W, PAD)                                                            \
  hipLaunchKernelGGL((hspmv_csr_stream<T, NT, U, PF, C, XW, XDX, W, PAD>), dim3((unsigned)p.blocks), \
                     dim3(W * 64), dyn, st, A.m, dp.long_t, dp.serial_max, (uint32_t)p.xcd_chunk,       \
                     (int32_t)p.groups,                                                               \
                     (int32_t)p.y_nt, p.carry, A.row_ptr, cs, xw, xd, val, x, y)
    if constexpr (XD) {  // never padded (plan_launch: dictionaries are sized unpadded)
      HSPMV_STREAM(false, false, true, 4, false);
      return;
    }
    // padded product buffers (LaunchPlan.lds_pad): conflicting row lengths,
    // no prefetch variant (the planner never pairs them)
    if constexpr (!PF) {
      if (p.lds_pad) {
        if (p.waves_per_block == 1 && xw) HSPMV_STREAM(C16, true, false, 1, true);
        else if (p.waves_per_block == 1) HSPMV_STREAM(C16, false, false, 1, true);
        else if (p.waves_per_block != 4 && xw) HSPMV_STREAM(C16, true, false, 2, true);
        else if (p.waves_per_block != 4) HSPMV_STREAM(C16, false, false, 2, true);
        else if (xw) HSPMV_STREAM(C16, true, false, 4, true);
        else HSPMV_STREAM(C16, false, false, 4, true);
        return;
      }
    }
    if (p.waves_per_block == 1 && xw) HSPMV_STREAM(C16, true, false, 1, false);
    else if (p.waves_per_block == 1) HSPMV_STREAM(C16, false, false, 1, false);
    else if (p.waves_per_block != 4 && xw) HSPMV_STREAM(C16, true, false, 2, false);
    else if (p.waves_per_block != 4) HSPMV_STREAM(C16, false, false, 2, false);
    else if (xw) HSPMV_STREAM(C16, true, false, 4, false);
    else HSPMV_STREAM(C16, false, false, 4, false);
#undef HSPMV_STREAM
    return;
  }
  {
  const int2 *xw = reinterpret_cast<const int2 *>(dp.xwin);
#define HSPMV_CSR3(W, C, XW, X)                                                               \
  hipLaunchKernelGGL((hspmv_csr3<T, NT, U, PF, C, W, XW, X>), dim3((unsigned)p.blocks),      \
                     dim3(W * 64), dyn, st, dp.n_tasks, dp.long_t, dp.serial_max,             \
                     (uint32_t)p.xcd_chunk,                                                   \
                     (int32_t)p.y_nt, p.carry, dp.task_align, dp.task_start, xw, xd, A.row_ptr, cs, \
                     val, x, y)
  if constexpr (XD) {  // packed tasks only (4 or 8 per block)
    if (p.waves_per_block == 8)
      HSPMV_CSR3(8, false, false, true);
    else
      HSPMV_CSR3(4, false, false, true);
    return;
  } else {
    if (xw && p.waves_per_block == 4) {  // x windows: packed tasks only (4 per block)
      HSPMV_CSR3(4, C16, true, false);
      return;
    }
    switch (p.waves_per_block) {
      case 1: HSPMV_CSR3(1, C16, false, false); break;
      case 2: HSPMV_CSR3(2, C16, false, false); break;
      case 4: HSPMV_CSR3(4, C16, false, false); break;
      default: HSPMV_CSR3(8, C16, false, false); break;
    }
  }
#undef HSPMV_CSR3
  }
}

template <typename T, bool NT, bool PF, int C16, bool XD>
hipError_t launch_rows_pf(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const T *x,
                          T *y, hipStream_t st) {
  switch (p.u) {
    case 2: launch_rows_u<T, NT, 2, PF, C16, XD>(A, dp, p, x, y, st); break;
    case 3: launch_rows_u<T, NT, 3, PF, C16, XD>(A, dp, p, x, y, st); break;
    case 4: launch_rows_u<T, NT, 4, PF, C16, XD>(A, dp, p, x, y, st); break;
    case 5: launch_rows_u<T, NT, 5, PF, C16, XD>(A, dp, p, x, y, st); break;
    case 6: launch_rows_u<T, NT, 6, PF, C16, XD>(A, dp, p, x, y, st); break;
    case 8: launch_rows_u<T, NT, 8, PF, C16, XD>(A, dp, p, x, y, st); break;
    case 16: launch_rows_u<T, NT, 16, PF, C16, XD>(A, dp, p, x, y, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T, int C16, bool XD>
hipError_t launch_rows_c(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const T *x,
                         T *y, hipStream_t st) {
  if (p.nontemporal)
    return p.prefetch ? launch_rows_pf<T, true, true, C16, XD>(A, dp, p, x, y, st)
                      : launch_rows_pf<T, true, false, C16, XD>(A, dp, p, x, y, st);
  return p.prefetch ? launch_rows_pf<T, false, true, C16, XD>(A, dp, p, x, y, st)
                    : launch_rows_pf<T, false, false, C16, XD>(A, dp, p, x, y, st);
}

// XD (block x dictionaries) replaces both the 32-bit columns and the col16
// offsets: its col stream is the 16-bit xs positions.
template <typename T>
hipError_t launch_rows(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p, const T *x, T *y,
                       hipStream_t st) {
  if (dp.xd_blk) {
    if (!A.col16 || (p.kernel == kStream && p.groups != 1) ||
        (p.kernel == kCsr3 && (!dp.task_start || (p.waves_per_block != 4 && p.waves_per_block != 8))))
      return hipErrorInvalidValue;  // the host built the dictionary for another block shape
    return launch_rows_c<T, 0, true>(A, dp, p, x, y, st);
  }
  if (A.col16 && A.c16_mode == 2) {
    if (p.kernel == kCsr3 && !dp.task_start)
      return hipErrorInvalidValue;  // built for the host-planned wave tasks (one base per task)
    return launch_rows_c<T, 2, false>(A, dp, p, x, y, st);
  }
  return A.col16 ? launch_rows_c<T, 1, false>(A, dp, p, x, y, st)
                 : launch_rows_c<T, 0, false>(A, dp, p, x, y, st);
}

}  // namespace dev
}  // namespace hspmv
