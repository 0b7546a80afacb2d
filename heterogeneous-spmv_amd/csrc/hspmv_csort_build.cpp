// hspmv_csort_build.cpp -- host build of the column-sorted row blocks (csort.hip)
// (see hspmv_runtime.h for the split of the host runtime).
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <thread>
#include <vector>

#include "hspmv_runtime.h"

namespace hspmv {

// Column-sorted row blocks (csort.hip; the kernel's header says why).
// Host build: rows are cut into nnz-balanced blocks of at most
// kCsortMaxSlots - (slices) rows, about one block per CU and column part;
// every workgroup (block, part) gets the block's nonzeros whose column lies
// in its part, sorted by column, plus its share of the long-row slices
// (rows > kLongRow nonzeros, cut per part into kCsortSlice-nonzero slices
// dealt round-robin over the blocks, each an extra LDS slot).  Entries are
// padded to whole chunks of 64*U, and a chunk is closed early when its
// columns would span more than 65535 (16-bit offsets from the chunk base).
// Padding entries add 0 * x[base] to a dummy slot that is never read.
// Auto: HBM-resident matrices with irregular gathers from an x beyond the
// L1 (> 256 KiB; it replaced the x-slab rule: C5 264 -> ~110 us), unless the
// handle asks for ordered sums (deterministic = 1: the slots add in atomic
// order); deterministic = 2 builds it with fixed-point (reproducible) slots;
// HSPMV_KERNEL_CSORT forces it, Tuning.csort = -1 turns auto off,
// Tuning.csort_parts = 1/2/4 sets the column parts, csort_u = 4/8/16 the
// chunk.  The row blocks are capped by the device's LDS per workgroup.
constexpr int32_t kCsortSlice = 2048;
// a chunk whose instructions would serialise more than this many same-slot
// lanes in all is stored slot-sorted (segmented)
constexpr int64_t kCsortSegExtra = 128;
constexpr int64_t kCsortSegHeavy = 8;  // entries of one row in a chunk that make it a run
constexpr double kPartSlack = 1.25;    // widest column part / (n / H) when balancing cost
constexpr double kSweepPerRowBlock = 0.13;  // a column's sweep cost, in entries, per row block
// Row-partition weight of crowded entries (>= 8 of one row to a chunk, so
// their chunks are segmented): c5r's hub blocks ran 96-104 us against a
// part median of 85 with the same entries and 100-160 segmented chunks
// (profiles/r04/csort_trace_wg_cost_balanced.jsonl): ~1.6x per entry.
constexpr int32_t kWUnit = 16, kWCrowded = 26;

struct CsEnt {
  uint32_t col, slot, k;
  bool operator<(const CsEnt &o) const {
    return col != o.col ? col < o.col : (slot != o.slot ? slot < o.slot : k < o.k);
  }
};

int build_csort(Shard &s, const int32_t *rp, const int32_t *col, const void *val, int64_t m,
                int64_t n, int dtype, unsigned flags) {
  if (m == 0 || n == 0 || !val) return HSPMV_OK;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s.device) != hipSuccess ||
      cus <= 0)
    cus = 256;
  int lds_max = 0;  // the row slots must fit one workgroup's LDS on THIS device
  if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, s.device) != hipSuccess ||
      lds_max <= 0)
    return HSPMV_OK;
  // the kernel's static LDS (its chunk-queue head, 16 B with alignment)
  // comes out of the same budget
  lds_max = std::min(lds_max, kCsortMaxLds) - 16;
  const Tuning &tn = s.tune;
  if (tn.csort_lds_cap > 0) lds_max = std::min(lds_max, tn.csort_lds_cap);  // A/B
  const bool slot32 = dtype == HSPMV_F32 && tn.csort_slot32 == 1;
  const int64_t slot_bytes = slot32 ? 4 : 8;
  const int32_t max_slots = (int32_t)(lds_max / slot_bytes) - 1;
  int H = n >= 2 ? 2 : 1;
  if (tn.csort_parts == 1 || tn.csort_parts == 2 || tn.csort_parts == 4)
    H = (int)std::min<int64_t>(tn.csort_parts, n);
  int U = dtype == HSPMV_F32 ? 16 : 8;
  if (tn.csort_u == 4 || tn.csort_u == 8 || tn.csort_u == 16) U = tn.csort_u;
  const int bpc = tn.csort_blocks_per_cu > 0 ? std::min(tn.csort_blocks_per_cu, 8) : 1;
  // 16-byte entry loads: needs U a multiple of 2 (fp32 records) / 4 (fp64 indices)
  // 16-byte entry loads + the next chunk's entries loaded during this chunk's
  // gathers: fp32 C5 107 -> 103 us, RCM'd C5 192 -> 190, in four one-process
  // A/Bs (profiles/r03/ab_c5_wide_pf*.jsonl); fp64 keeps 8-byte loads
  // (unmeasured).  Neither alone moves C5 (wide 108.8 vs 108.0, PF 109.4).
  const bool wide_default = dtype == HSPMV_F32;
  const bool wide = (tn.csort_wide >= 0 ? tn.csort_wide == 1 : wide_default) &&
                    (dtype == HSPMV_F32 ? U % 2 == 0 : U % 4 == 0);
  const int64_t C = 64 * U;
  const size_t sv = dtype_size(dtype);
  const int32_t long_t = (flags & HSPMV_FLAG_NO_SPLIT) ? INT32_MAX
                         : (s.tune.csort_long > 0 ? s.tune.csort_long : kLongRow);
  const int64_t nb0 = std::max<int64_t>(1, (int64_t)cus * bpc / H);
  // Column parts: [pb[h], pb[h+1]).  Equal widths, or (Tuning.csort_balance
  // >= 0, the default) boundaries at equal shares of the parts' COST, each
  // part's width kept within kPartSlack of n / H.  A workgroup's time is
  // ~alpha per entry + beta per column of its part (the x sweep): from the
  // per-workgroup timelines of c5r (profiles/r04c/csort_trace_wg*.jsonl),
  // alpha = 2.5e-4 us, beta = 3.0-3.4e-5 us per fp32 column, so a column
  // weighs kSweepPerRowBlock * (row blocks) entries (x 2 * 8 / 12 for fp64
  // x and entries).  An RCM ordering concentrates a power-law matrix's
  // entries in the upper columns (c5r: 59 % in the upper half): equal widths
  // gave that half's workgroups 1.42x the entries (123.4 us), equal entries
  // over-corrected onto the wider lower part (108.8 us, its sweep 43 % wider).
  std::vector<int64_t> pb((size_t)H + 1, 0);
  for (int h = 0; h <= H; ++h) pb[(size_t)h] = (n * h + H - 1) / H;  // c in part floor(c*H/n)
  if (H > 1 && tn.csort_balance >= 0) {
    std::vector<int64_t> colcnt((size_t)n + 1, 0);
    for (int64_t k = 0; k < rp[m]; ++k) ++colcnt[(size_t)col[k]];
    const double nb_part = (double)std::max<int64_t>(1, (int64_t)cus * bpc / H);
    const double wsw = tn.csort_sweep_w > 0 ? tn.csort_sweep_w : kSweepPerRowBlock;
    const double wcol = wsw * nb_part * (dtype == HSPMV_F64 ? 2.0 * 8.0 / 12.0 : 1.0);
    const double tot = (double)rp[m] + wcol * (double)n;
    double acc = 0.0;
    int64_t c = 0;
    for (int h = 1; h < H; ++h) {
      const double target = tot * h / H;
      while (c < n && acc + (double)colcnt[(size_t)c] + wcol <= target) acc += (double)colcnt[(size_t)c++] + wcol;
      const int64_t eq = (n * h + H - 1) / H;
      const double ps = tn.csort_slack > 1.0 ? tn.csort_slack : kPartSlack;  // A/B knob
      const int64_t slack = (int64_t)((ps - 1.0) * (double)(n / H));
      const int64_t lo = std::max(pb[(size_t)h - 1] + 1, eq - slack), hi = std::max(lo, eq + slack);
      pb[(size_t)h] = std::min(std::max(c, lo), hi);
    }
  }
  std::vector<uint8_t> part_tab;
  if (H > 1) {
    part_tab.assign((size_t)n, 0);
    for (int h = 0; h < H; ++h)
      std::fill(part_tab.begin() + pb[(size_t)h], part_tab.begin() + pb[(size_t)h + 1], (uint8_t)h);
  }
  auto part_of = [&](int64_t c) { return H > 1 ? (int)part_tab[(size_t)c] : 0; };
  // long rows and their slices (per part, kCsortSlice nonzeros each)
  std::vector<int32_t> lrow, lcs(1, 0);
  std::vector<std::vector<uint32_t>> slice_k;  // source nonzeros per slice
  std::vector<int> slice_part;
  int64_t long_nnz = 0;
  for (int64_t r = 0; r < m; ++r) {
    const int32_t k0 = rp[r], k1 = rp[r + 1];
    if (k1 - k0 <= long_t) continue;
    long_nnz += k1 - k0;
    lrow.push_back((int32_t)r);
    std::vector<std::vector<uint32_t>> byp((size_t)H);
    for (int32_t k = k0; k < k1; ++k) byp[(size_t)part_of(col[k])].push_back((uint32_t)k);
    for (int h = 0; h < H; ++h)
      for (size_t i = 0; i < byp[(size_t)h].size(); i += kCsortSlice) {
        const size_t e = std::min(byp[(size_t)h].size(), i + kCsortSlice);
        slice_k.emplace_back(byp[(size_t)h].begin() + (ptrdiff_t)i, byp[(size_t)h].begin() + (ptrdiff_t)e);
        slice_part.push_back(h);
      }
    lcs.push_back((int32_t)slice_k.size());
  }
  const int64_t n_slices = (int64_t)slice_k.size();
  // Reproducible (fixed-point) slots (Tuning.deterministic == 2, csort.hip
  // fix_q): every value of row r is stored scaled by 2^rexp[r], exactly (a
  // power of two), so that the row's |v'| < 2^-extra: rexp = -(ilogb max|v| +
  // 1) - extra, extra = ceil(log2 len) - 12 for a row kept whole over 4096
  // nonzeros (HSPMV_FLAG_NO_SPLIT), else 0 -- every product then rounds to an
  // integer below 2^kCsortFixBits and a slot of <= 4096 of them stays below
  // 2^62.  A value that the scaling takes below the type's normal range loses
  // bits only below the products' rounding unit (2^-kCsortFixBits of the
  // row's largest).
  // A matrix with an Inf or NaN value has no fixed-point scale for its row
  // (the product must stay non-finite): such a handle keeps fp64 slots and
  // reports csort_fixed_point = 0, deterministic = 0.
  bool fixed = tn.deterministic == 2 && !slot32;
  std::vector<int16_t> rexp(fixed ? (size_t)m : 0, 0), sexp;
  if (fixed) {
    for (int64_t r = 0; r < m && fixed; ++r) {
      double mx = 0.0;
      for (int32_t k = rp[r]; k < rp[r + 1]; ++k) {
        const double v = dtype == HSPMV_F32 ? (double)static_cast<const float *>(val)[k]
                                            : static_cast<const double *>(val)[k];
        mx = std::max(mx, std::fabs(v));
        if (!std::isfinite(v)) fixed = false;
      }
      if (!(mx > 0.0) || !std::isfinite(mx)) continue;  // empty / zero rows
      const int64_t len = rp[r + 1] - rp[r];
      int extra = 0;  // (a sliced row's slots hold kCsortSlice <= 4096 products each)
      while (len <= long_t && ((int64_t)4096 << extra) < len) ++extra;
      rexp[(size_t)r] = (int16_t)(-(std::ilogb(mx) + 1) - extra);
    }
    if (!fixed) std::vector<int16_t>().swap(rexp);
  }
  if (fixed) {
    sexp.resize((size_t)std::max<int64_t>(n_slices, 1), 0);
    for (size_t j = 0; j + 1 < lcs.size(); ++j)
      for (int32_t sl = lcs[j]; sl < lcs[j + 1]; ++sl) sexp[(size_t)sl] = rexp[(size_t)lrow[j]];
  }
  // the (scaled) value of nonzero k of row r
  auto value_f32 = [&](uint32_t k, int64_t r) -> uint32_t {
    float v = static_cast<const float *>(val)[k];
    if (fixed) v = std::ldexp(v, rexp[(size_t)r]);
    uint32_t b;
    memcpy(&b, &v, 4);
    return b;
  };
  auto value_f64 = [&](uint32_t k, int64_t r) -> double {
    const double v = static_cast<const double *>(val)[k];
    return fixed ? std::ldexp(v, rexp[(size_t)r]) : v;
  };
  // Row blocks PER COLUMN PART.  Part h is a fixed slice of x, [pb[h],
  // pb[h+1]) (above), and workgroup j works on part
  // j % H: under round-robin dispatch (workgroup j on XCD j % 8;
  // tools/xcd_map_probe.hip records it per box) every XCD sweeps one slice,
  // which its 4 MiB L2 keeps for all its CUs.  Each part has its OWN row
  // partition, balanced on the nonzeros that fall in that part and capped in
  // rows (the LDS slots), so the parts' workgroups carry equal work whatever
  // the ordering: with one row partition for all parts an RCM-ordered
  // power-law matrix put ~90 % of a block's entries in one part (322 us vs
  // 108 us on the same matrix unordered), and quantile splits per block, which
  // balance the work but let every XCD sweep all of x, still took 205 us.
  const int64_t reserve = n_slices / nb0 + 2;
  const int64_t row_cap = max_slots - 1 - reserve;
  if (row_cap < 64) return HSPMV_OK;  // too many slices for the LDS: not this path
  // [h][r]: row r's in-kernel nonzeros in part h, then its partition weight
  std::vector<int32_t> cnt((size_t)(H * m), 0);
  std::vector<int64_t> tot_part((size_t)H, 0);
  const int ntc = (int)std::max<int64_t>(1, std::min<int64_t>(16, m / 65536));
  auto par_rows = [&](auto &&body) {
    std::vector<std::thread> th;
    for (int t = 0; t < ntc; ++t) th.emplace_back([&, t]() { body(t, m * t / ntc, m * (t + 1) / ntc); });
    for (auto &x : th) x.join();
  };
  par_rows([&](int, int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      if (rp[r + 1] - rp[r] > long_t) continue;
      for (int32_t k = rp[r]; k < rp[r + 1]; ++k) ++cnt[(size_t)(part_of(col[k]) * m + r)];
    }
  });
  for (int h = 0; h < H; ++h)
    for (int64_t r = 0; r < m; ++r) tot_part[(size_t)h] += cnt[(size_t)(h * m + r)];
  // a row's partition weight (int32: a row of > 2^31 / kWCrowded entries,
  // possible only unsplit, saturates)
  auto weigh = [](int64_t plain, int64_t crowded) {
    return (int32_t)std::min<int64_t>(INT32_MAX / 2, plain * kWUnit + crowded * kWCrowded);
  };
  if (tn.csort_balance >= 0) {
    // Crowded entries: ones with >= kCsortSegHeavy entries of the same row
    // within the columns one chunk of a block covers (cspan) -- the entries
    // that make their chunks segmented.  An RCM ordering clusters a hub
    // row's columns, so the row's whole span says little: each entry's own
    // window is counted (sorted copy of the row's part, two pointers).
    std::vector<double> cspan((size_t)H, 0.0);
    for (int h = 0; h < H; ++h)
      cspan[(size_t)h] = tot_part[(size_t)h] ? (double)C * (double)(pb[(size_t)h + 1] - pb[(size_t)h]) *
                                                   (double)nb0 / (double)tot_part[(size_t)h]
                                             : 0.0;
    par_rows([&](int, int64_t r0, int64_t r1) {
      std::vector<int32_t> cs;
      std::vector<int32_t> crowded((size_t)H);
      for (int64_t r = r0; r < r1; ++r) {
        const int32_t len = rp[r + 1] - rp[r];
        if (len > long_t || len < kCsortSegHeavy) {
          for (int h = 0; h < H; ++h) cnt[(size_t)(h * m + r)] = weigh(cnt[(size_t)(h * m + r)], 0);
          continue;
        }
        cs.assign(col + rp[r], col + rp[r + 1]);
        std::sort(cs.begin(), cs.end());
        std::fill(crowded.begin(), crowded.end(), 0);
        for (size_t i = 0, j = 0; i < cs.size(); ++i) {  // entries i..j-1 within cspan of cs[i]
          const int h = part_of(cs[i]);
          const double lim = (double)cs[i] + cspan[(size_t)h];
          if (j < i + 1) j = i + 1;
          while (j < cs.size() && (double)cs[j] < lim && part_of(cs[j]) == h) ++j;
          if ((int64_t)(j - i) >= kCsortSegHeavy) ++crowded[(size_t)h];
        }
        for (int h = 0; h < H; ++h) {
          const size_t i = (size_t)(h * m + r);
          const int32_t cr = std::min(cnt[i], crowded[(size_t)h]);
          cnt[i] = weigh(cnt[i] - cr, cr);
        }
      }
    });
  } else {
    for (auto &v : cnt) v = weigh(v, 0);
  }
  // Greedy cuts at `target` weight or row_cap rows; the target is the
  // smallest that yields at most nb0 blocks (one block more would run a
  // second round of workgroups on one CU and double the launch).
  auto cut_w = [&](const int32_t *c, int64_t target, std::vector<int32_t> *out) -> int64_t {
    int64_t start = 0, acc = 0, nblk = 1;
    if (out) out->assign(1, 0);
    for (int64_t r = 0; r < m; ++r) {
      if (r > start && (r - start >= row_cap || acc >= target)) {
        if (out) out->push_back((int32_t)r);
        ++nblk;
        start = r;
        acc = 0;
      }
      acc += c[r];
    }
    if (out) out->push_back((int32_t)m);
    return nblk;
  };
  // the smallest target giving at most nb0 blocks
  auto partition = [&](const int32_t *c, std::vector<int32_t> &out) {
    int64_t tot_h = 0;
    for (int64_t r = 0; r < m; ++r) tot_h += c[r];
    int64_t lo = std::max<int64_t>(1, (tot_h + nb0 - 1) / nb0), hi = std::max<int64_t>(lo, tot_h + 1);
    if (cut_w(c, lo, nullptr) > nb0) {
      if (cut_w(c, hi, nullptr) > nb0) lo = hi;  // the row cap alone needs more blocks
      while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (cut_w(c, mid, nullptr) <= nb0) hi = mid; else lo = mid + 1;
      }
    }
    cut_w(c, lo, &out);
  };
  std::vector<std::vector<int32_t>> brh((size_t)H);
  int64_t NB = 0;
  for (int h = 0; h < H; ++h) {
    partition(cnt.data() + (size_t)h * (size_t)m, brh[(size_t)h]);
    NB = std::max<int64_t>(NB, (int64_t)brh[(size_t)h].size() - 1);
  }
  std::vector<int32_t>().swap(cnt);
  const int64_t G = NB * H;
  if (G >= INT32_MAX) return HSPMV_OK;
  // workgroup j: part j % H, that part's block j / H (empty past its blocks)
  std::vector<int32_t> wg_rows((size_t)(2 * G), (int32_t)m);
  for (int64_t j = 0; j < G; ++j) {
    const auto &b = brh[(size_t)(j % H)];
    const int64_t i = j / H;
    if (i + 1 < (int64_t)b.size()) {
      wg_rows[(size_t)(2 * j)] = b[(size_t)i];
      wg_rows[(size_t)(2 * j + 1)] = b[(size_t)i + 1];
    }
  }
  // slices dealt round-robin over the blocks of their part
  std::vector<std::vector<int32_t>> wg_sl((size_t)G);
  {
    std::vector<int64_t> next((size_t)H, 0);
    for (int64_t sl = 0; sl < n_slices; ++sl) {
      const int h = slice_part[(size_t)sl];
      const int64_t nbh = (int64_t)brh[(size_t)h].size() - 1;
      const int64_t i = next[(size_t)h]++ % nbh;
      wg_sl[(size_t)(i * H + h)].push_back((int32_t)sl);
    }
  }
  // per workgroup: sorted entries, chunk count (pass 1)
  std::vector<std::vector<CsEnt>> ents((size_t)G);
  std::vector<int64_t> nchunks((size_t)G, 0);
  std::vector<int32_t> nslots((size_t)G, 0);
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(16, G / 4));
  std::atomic<bool> too_big{false};
  auto chunk_walk = [&](const std::vector<CsEnt> &E, auto &&emit) {
    // chunks of C entries, closed early when the span would pass 65535
    int64_t i = 0, cnt_ = 0;
    const int64_t ne = (int64_t)E.size();
    while (i < ne) {
      const uint32_t c0 = E[(size_t)i].col;
      int64_t j = i;
      while (j < ne && j - i < C && E[(size_t)j].col - c0 <= 65535u) ++j;
      emit(cnt_, c0, i, j);
      ++cnt_;
      i = j;
    }
    return cnt_;
  };
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t]() {
        for (int64_t b = t; b < G; b += nt) {
          const int h = (int)(b % H);
          const int32_t r0 = wg_rows[(size_t)(2 * b)], r1 = wg_rows[(size_t)(2 * b + 1)];
          const int32_t nr = r1 - r0;
          auto &E = ents[(size_t)b];
          for (int32_t r = r0; r < r1; ++r) {
            if (rp[r + 1] - rp[r] > long_t) continue;
            for (int32_t k = rp[r]; k < rp[r + 1]; ++k)
              if (part_of(col[k]) == h) E.push_back({(uint32_t)col[k], (uint32_t)(r - r0), (uint32_t)k});
          }
          const auto &sl = wg_sl[(size_t)b];
          for (size_t v = 0; v < sl.size(); ++v)
            for (uint32_t k : slice_k[(size_t)sl[v]])
              E.push_back({(uint32_t)col[k], (uint32_t)(nr + (int32_t)v), k});
          std::sort(E.begin(), E.end());
          nslots[(size_t)b] = nr + (int32_t)sl.size() + 1;  // + the dummy slot
          if (nslots[(size_t)b] > 65536 || ((int64_t)nslots[(size_t)b] + 1) * slot_bytes > lds_max) too_big = true;
          nchunks[(size_t)b] = chunk_walk(E, [](int64_t, uint32_t, int64_t, int64_t) {});
        }
      });
    for (auto &x : th) x.join();
  }
  if (too_big) return HSPMV_OK;
  std::vector<int32_t> blk_c((size_t)G + 1, 0), blk_v((size_t)G + 1, 0), vslice;
  int64_t tot_chunks = 0;
  int32_t max_slots_used = 1;
  for (int64_t b = 0; b < G; ++b) {
    blk_c[(size_t)b] = (int32_t)tot_chunks;
    tot_chunks += nchunks[(size_t)b];
    blk_v[(size_t)b] = (int32_t)vslice.size();
    for (int32_t sl : wg_sl[(size_t)b]) vslice.push_back(sl);
    max_slots_used = std::max(max_slots_used, nslots[(size_t)b]);
  }
  blk_c[(size_t)G] = (int32_t)tot_chunks;
  blk_v[(size_t)G] = (int32_t)vslice.size();
  if (tot_chunks * C >= (int64_t)1 << 40 || tot_chunks >= INT32_MAX) return HSPMV_OK;
  const int64_t tot = tot_chunks * C;
  std::vector<int32_t> slice_row_of((size_t)n_slices, 0);
  for (size_t j = 0; j + 1 < lcs.size(); ++j)
    for (int32_t sl = lcs[j]; sl < lcs[j + 1]; ++sl) slice_row_of[(size_t)sl] = lrow[j];
  auto slice_row = [&](int32_t sl) -> int64_t { return slice_row_of[(size_t)sl]; };
  // pass 2: the device arrays
  std::vector<int32_t> cbase((size_t)std::max<int64_t>(tot_chunks, 1), 0);
  std::vector<uint32_t> idx;
  std::vector<uint64_t> rec;
  std::vector<double> val64;
  if (dtype == HSPMV_F32)
    rec.assign((size_t)tot, 0);
  else {
    idx.assign((size_t)tot, 0);
    val64.assign((size_t)tot, 0.0);
  }
  std::atomic<int64_t> n_seg{0};  // chunks stored slot-sorted (segmented)
  // diagnostic builds (Tuning.csort_trace): per workgroup {rows, slices,
  // chunks, entries, gather quad-sectors, gather sectors, segmented chunks,
  // 0} -- the cost terms the per-workgroup timelines are compared with
  constexpr int kWgStats = 8;
  const bool stats = tn.csort_trace == 1;
  std::vector<int64_t> wst(stats ? (size_t)(kWgStats * G) : 0, 0);
  const int sec_shift = dtype == HSPMV_F32 ? 3 : 2;  // x entries per 32-byte sector: 8 / 4
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t]() {
        for (int64_t b = t; b < G; b += nt) {
          auto &E = ents[(size_t)b];
          const uint32_t dummy = (uint32_t)(nslots[(size_t)b] - 1);
          const int32_t br0 = wg_rows[(size_t)(2 * b)], bnr = wg_rows[(size_t)(2 * b + 1)] - br0;
          const auto &bsl = wg_sl[(size_t)b];
          auto row_of = [&](uint32_t slot) -> int64_t {  // source row of a slot (fixed-point scale)
            return (int32_t)slot < bnr ? (int64_t)br0 + slot : slice_row(bsl[slot - bnr]);
          };
          const int64_t cfirst = blk_c[(size_t)b];
          // entry q of a chunk (lane q % 64, u = q / 64) is stored at q, or,
          // for 16-byte loads, interleaved so that one load brings the lane
          // entries u, u+1 (fp32 records, fp64 values) or u..u+3 (fp64 indices)
          auto at = [&](int64_t q, int per) -> int64_t {
            if (!wide) return q;
            const int64_t u = q / 64, lane = q % 64;
            return (u / per) * (64 * per) + lane * per + (u % per);
          };
          std::vector<CsEnt> tmp;
          uint32_t sl64[64];
          chunk_walk(E, [&](int64_t ci, uint32_t c0, int64_t i, int64_t j) {
            const int64_t ch = cfirst + ci;
            // Same-slot lanes in one instruction serialise the LDS atomics:
            // an RCM ordering puts a hub row's entries on contiguous columns,
            // so column order can give one instruction 64 lanes of one row
            // (RCM power-law: a few workgroups with ~100 K serialised lanes
            // set the launch's tail, 204 vs 108 us).  Such chunks are stored
            // sorted by slot instead and flagged (bit 31 of the base): the
            // kernel sums each instruction's runs first (segmented scan).
            const CsEnt *src = E.data() + i;
            bool seg = false;
            if (tn.csort_seg != 0) {
              int64_t extra = 0;
              for (int64_t g = i; g < j; g += 64) {
                const int64_t e = std::min(j, g + 64);
                for (int64_t t = g; t < e; ++t) sl64[t - g] = E[(size_t)t].slot;
                std::sort(sl64, sl64 + (e - g));
                int run = 1, mx = 1;
                for (int64_t t = 1; t < e - g; ++t) {
                  run = sl64[t] == sl64[t - 1] ? run + 1 : 1;
                  mx = std::max(mx, run);
                }
                extra += mx - 1;
              }
              const int64_t lim = tn.csort_seg_extra > 0 ? tn.csort_seg_extra : kCsortSegExtra;
              if (extra > lim || tn.csort_seg == 2) {
                // the crowded rows (>= kCsortSegHeavy entries in this chunk)
                // first, slot-sorted, in column order within each: their runs
                // are contiguous columns (coalesced gathers); the other
                // entries after them, still in column order
                std::vector<std::pair<uint32_t, int32_t>> cnt_s;
                cnt_s.reserve((size_t)(j - i));
                for (int64_t t = i; t < j; ++t) cnt_s.push_back({E[(size_t)t].slot, 0});
                std::sort(cnt_s.begin(), cnt_s.end());
                std::vector<uint32_t> heavy;
                for (size_t t = 0; t < cnt_s.size();) {
                  size_t e = t;
                  while (e < cnt_s.size() && cnt_s[e].first == cnt_s[t].first) ++e;
                  if ((int64_t)(e - t) >= kCsortSegHeavy || tn.csort_seg == 2) heavy.push_back(cnt_s[t].first);
                  t = e;
                }
                auto is_heavy = [&](uint32_t sl) { return std::binary_search(heavy.begin(), heavy.end(), sl); };
                tmp.clear();
                for (int64_t t = i; t < j; ++t)
                  if (is_heavy(E[(size_t)t].slot)) tmp.push_back(E[(size_t)t]);
                std::stable_sort(tmp.begin(), tmp.end(), [](const CsEnt &a, const CsEnt &b) { return a.slot < b.slot; });
                for (int64_t t = i; t < j; ++t)
                  if (!is_heavy(E[(size_t)t].slot)) tmp.push_back(E[(size_t)t]);
                src = tmp.data();
                seg = true;
                n_seg.fetch_add(1, std::memory_order_relaxed);
              }
            }
            cbase[(size_t)ch] = (int32_t)(c0 | (seg ? 0x80000000u : 0u));
            const int64_t ne = j - i;  // lanes >= ne: padding (gathers x[base])
            if (stats) {
              int64_t *w = wst.data() + kWgStats * b;
              w[2] += 1;
              w[3] += j - i;
              w[6] += seg ? 1 : 0;
              for (int64_t g = 0; g < C; g += 64) {  // one gather instruction
                uint32_t sec[64];
                for (int64_t q = 0; q < 64; ++q)
                  sec[q] = (g + q < ne ? src[g + q].col : c0) >> sec_shift;
                for (int64_t q = 0; q < 64; q += 4) {  // the L1 serves each quad on its own
                  int d = 1;
                  for (int t = 1; t < 4; ++t) {
                    bool seen = false;
                    for (int t2 = 0; t2 < t; ++t2) seen |= sec[q + t] == sec[q + t2];
                    d += seen ? 0 : 1;
                  }
                  w[4] += d;
                }
                std::sort(sec, sec + 64);
                w[5] += (int64_t)(std::unique(sec, sec + 64) - sec);
              }
            }
            for (int64_t q = 0; q < C; ++q) {
              const int64_t o = ch * C + at(q, dtype == HSPMV_F32 ? 2 : 4);
              const int64_t ov = ch * C + at(q, 2);
              uint32_t ix = dummy << 16;  // padding: 0 * x[base] into the dummy slot
              if (dtype == HSPMV_F32) {
                uint32_t vb = 0;
                if (q < ne) {
                  const CsEnt &e = src[q];
                  ix = (e.slot << 16) | (e.col - c0);
                  vb = value_f32(e.k, row_of(e.slot));
                }
                rec[(size_t)o] = ((uint64_t)vb << 32) | ix;
              } else {
                if (q < ne) {
                  const CsEnt &e = src[q];
                  ix = (e.slot << 16) | (e.col - c0);
                  val64[(size_t)ov] = value_f64(e.k, row_of(e.slot));
                }
                idx[(size_t)o] = ix;
              }
            }
          });
          std::vector<CsEnt>().swap(E);
        }
      });
    for (auto &x : th) x.join();
  }
  std::vector<uint32_t> mask;
  if (!lrow.empty()) {
    mask.assign((size_t)((m + 31) / 32), 0u);
    for (int32_t r : lrow) mask[(size_t)r >> 5] |= 1u << (r & 31);
  }
  int rc;
  auto up = [&](auto **d, const auto &h) -> int {
    using E = typename std::decay_t<decltype(h)>::value_type;
    const size_t bytes = sizeof(E) * std::max<size_t>(h.size(), 1);
    int r2 = dev_alloc(d, bytes, &s.bytes);
    if (r2) return r2;
    if (!h.empty()) HIP_TRY(hipMemcpy(*d, h.data(), sizeof(E) * h.size(), hipMemcpyHostToDevice));
    return HSPMV_OK;
  };
  if ((rc = up(&s.d_cs_blk_c, blk_c)) || (rc = up(&s.d_cs_blk_r, wg_rows)) ||
      (rc = up(&s.d_cs_blk_v, blk_v)) || (rc = up(&s.d_cs_vslice, vslice)) || (rc = up(&s.d_cs_cbase, cbase)))
    return rc;
  if (dtype == HSPMV_F32) {
    uint64_t *d = nullptr;
    if ((rc = up(&d, rec))) return rc;
    s.d_cs_ent = d;
  } else {
    uint32_t *di = nullptr;
    double *dv = nullptr;
    if ((rc = up(&di, idx))) return rc;
    s.d_cs_ent = di;
    if ((rc = up(&dv, val64))) return rc;
    s.d_cs_val = dv;
  }
  const bool direct = H == 1 && lrow.empty();
  // Row partials: fp32 for fp32 data (part32, the default since r06; the
  // LDS slots stay fp64 and the finishing pass adds in fp64): half of C5's
  // 64 MB of partial traffic, C5 98.2 -> 91.9 us, c5r 99.2 -> 94.5 (t_min,
  // one process, profiles/r05q1/ab_part32.jsonl).  y then rounds twice on
  // rows with entries in both column parts (the part's sum, then y):
  // |y - y64| <= 2^-24 (sum_h |p_h| + |y64|), inside omp_spmv's own fp32
  // error (len + 2) 2^-23 sum|a x| (tests/test_gpu_parity.py).  Tuning
  // csort_part32 = 0 keeps fp64 partials (A/B).
  const bool part32 = dtype == HSPMV_F32 && !slot32 && tn.csort_part32 != 0;
  const int64_t part_bytes = part32 ? 4 : slot_bytes;
  if (!direct) {
    if ((rc = dev_alloc(&s.d_cs_part, part_bytes * (size_t)H * (size_t)m, &s.bytes))) return rc;
    if ((rc = dev_alloc(&s.d_cs_spart, slot_bytes * (size_t)std::max<int64_t>(n_slices, 1), &s.bytes)))
      return rc;
  }
  if (!lrow.empty()) {
    if ((rc = up(&s.d_cs_mask, mask)) || (rc = up(&s.d_cs_long_row, lrow)) || (rc = up(&s.d_cs_long_cs, lcs)))
      return rc;
  }
  int32_t n_xexp = 0;
  if (fixed) {  // the x-exponent pre-pass: one block per 8192 entries of x, at most kCsortXexpBlocks
    if ((rc = up(&s.d_cs_rexp, rexp)) || (rc = up(&s.d_cs_sexp, sexp))) return rc;
    n_xexp = (int32_t)std::min<int64_t>(kCsortXexpBlocks,
                                        std::max<int64_t>(1, (n + kCsortXexpChunk - 1) / kCsortXexpChunk));
    if ((rc = dev_alloc(&s.d_cs_xexp, 4 * (size_t)n_xexp, &s.bytes))) return rc;
  }
  // (An in-launch combine -- write-through partials, an arrival counter per
  // row block, the last arriver adding the parts -- measured slower than
  // the finishing launch: C5 114.8 vs 107.3 us, profiles/r02s_*.)
  DevCsort &c = s.csort;
  c = DevCsort();
  c.n_wg = (int32_t)G;
  c.H = H;
  c.u = U;
  c.direct = direct ? 1 : 0;
  c.n_long = (int32_t)lrow.size();
  c.nontemporal = true;  // the entry stream is read once; keep x in the caches
  if (tn.csort_nt >= 0) c.nontemporal = tn.csort_nt != 0;  // A/B knobs
  c.prefetch = wide && dtype == HSPMV_F32;  // see `wide` above
  if (tn.csort_pf >= 0) c.prefetch = tn.csort_pf != 0;
  c.slot32 = slot32;
  c.part32 = part32;
  c.wide = wide;
  c.fin_rows = tn.csort_fin_rows;
  c.fixed = fixed;
  c.rexp = s.d_cs_rexp;
  c.sexp = s.d_cs_sexp;
  c.xexp_part = s.d_cs_xexp;
  c.n_xexp = n_xexp;
  c.n_x = n;
  // waves claim chunks from the workgroup's LDS queue: one process, 7
  // rounds (profiles/r05c/ab_csort_dyn.jsonl): C5 106.9 -> 101.9 us median,
  // c5r 107.3 -> 104.9, fp64 C5 flat (175.7 -> 174.7)
  c.dyn = tn.csort_dyn != 0;
  c.m = m;
  c.lds_bytes = (int32_t)(slot_bytes * max_slots_used);
  c.blk_c = s.d_cs_blk_c;
  c.blk_r = s.d_cs_blk_r;
  c.blk_v = s.d_cs_blk_v;
  c.row_blocks = (int32_t)NB;
  s.csort_seg_chunks = n_seg.load();
  if (stats) {
    for (int64_t b = 0; b < G; ++b) {
      wst[(size_t)(kWgStats * b)] = wg_rows[(size_t)(2 * b + 1)] - wg_rows[(size_t)(2 * b)];
      wst[(size_t)(kWgStats * b + 1)] = (int64_t)wg_sl[(size_t)b].size();
    }
    s.csort_wg_stats.swap(wst);
  }
  s.csort_chunks = tot_chunks;
  for (int h = 0; h < 4; ++h) s.csort_part_begin[h] = h < H ? pb[(size_t)h] : 0;
  if (tn.csort_trace == 1 && (rc = dev_alloc(&s.d_cs_trace, 8 * kCsortTraceSlots * (size_t)G, &s.bytes))) return rc;
  c.trace = s.d_cs_trace;
  c.vslice = s.d_cs_vslice;
  c.cbase = s.d_cs_cbase;
  c.ent = s.d_cs_ent;
  c.val = s.d_cs_val;
  c.part = s.d_cs_part;
  c.spart = s.d_cs_spart;
  c.long_mask = s.d_cs_mask;
  c.long_row = s.d_cs_long_row;
  c.long_cs = s.d_cs_long_cs;
  // bytes moved: the entry stream + chunk bases + x (distinct columns) + the
  // partial sums written and read back + y
  const double xb = (double)s.x_entries * (double)sv;
  const double part_traffic =
      direct ? 0.0
             : 2.0 * ((double)part_bytes * (double)H * (double)m + (double)slot_bytes * (double)n_slices);
  // (fixed-point: + the x exponent's read of x and the row scales)
  const double fix_traffic = fixed ? (double)n * (double)sv + 2.0 * (double)H * (double)m : 0.0;
  s.csort_format_bytes = (double)tot * (double)(4 + sv) + 4.0 * (double)tot_chunks + xb + part_traffic +
                         (double)sv * (double)m + fix_traffic;
  s.A.has_csort = true;
  return HSPMV_OK;
}

}  // namespace hspmv
