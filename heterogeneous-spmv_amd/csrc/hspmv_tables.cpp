// hspmv_tables.cpp -- host planner tables of a shard
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

// Number of distinct column indices in col[0..nnz) (< n): x entries read.
int64_t count_distinct_cols(const int32_t *col, int64_t nnz, int64_t n) {
  std::vector<uint64_t> bits((size_t)(n / 64 + 1), 0);
  for (int64_t k = 0; k < nnz; ++k) bits[(size_t)col[k] >> 6] |= 1ull << (col[k] & 63);
  int64_t c = 0;
  for (uint64_t w : bits) c += __builtin_popcountll(w);
  return c;
}

// 16-bit column offsets: per block of 2^kC16Shift nonzeros, base = the
// block's smallest column and col - base split into its low 16 bits (off16)
// and k high bits stored as k bit-planes of 64-bit words (bit k&63 of word
// k>>6), k = the fewest that cover every block's column span.  Used when
// k <= kMaxC16Planes and the shard streams from HBM.  One-process A/B
// runs (profiles/r01_ab_col16.jsonl): C4 (k = 0) -10 %, C3 (k = 1) -5 %;
// C5 (k = 5) +9 % and the Infinity-Cache-resident C2 +4 % slower, where the
// extra scalar loads and selects outweigh the bytes saved.
constexpr int kMaxC16Planes = 1;
constexpr int kMaxC16PlanesForced = 8;  // 3 index bytes: still fewer than 4

int build_col16(Shard &s, const int32_t *col, int64_t nnz, int64_t m, int64_t n, int dtype,
                unsigned flags, bool *used) {
  *used = false;
  if (nnz == 0) return HSPMV_OK;
  const bool forced = (flags & HSPMV_FLAG_COL16) != 0 && !(flags & HSPMV_FLAG_NO_COL16);
  const double sv = (double)dtype_size(dtype);
  if (!forced && (double)nnz * (sv + 4.0) + (double)m * (sv + 4.0) + (double)n * sv <= kMallResident)
    return HSPMV_OK;
  const int64_t B = int64_t(1) << kC16Shift;
  const int64_t nb = (nnz + B - 1) / B;
  std::vector<int32_t> base((size_t)nb + 1, 0);  // +1: kernels load bases in pairs
  std::vector<int32_t> span((size_t)nb, 0);
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(16, nb / 4096));
  auto par = [&](auto &&body) {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&, t]() { body(nb * t / nt, nb * (t + 1) / nt); });
    for (auto &x : th) x.join();
  };
  par([&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b) {
      const int64_t k0 = b * B, k1 = std::min(nnz, k0 + B);
      int32_t lo = col[k0], hi = col[k0];
      for (int64_t k = k0 + 1; k < k1; ++k) {
        lo = std::min(lo, col[k]);
        hi = std::max(hi, col[k]);
      }
      base[(size_t)b] = lo;
      span[(size_t)b] = hi - lo;
    }
  });
  int32_t maxspan = 0;
  for (int32_t v : span) maxspan = std::max(maxspan, v);
  int bits = 0;
  while (bits < 31 && (int64_t(1) << bits) <= maxspan) ++bits;
  s.A.col_span_bits = std::max(1, bits);  // the planner's gather-regularity hint
  if (flags & HSPMV_FLAG_NO_COL16) return HSPMV_OK;
  const int planes = std::max(0, bits - 16);
  if (planes > (forced ? kMaxC16PlanesForced : kMaxC16Planes)) return HSPMV_OK;
  const int64_t nw = (nnz + 63) / 64 + 1;  // +1: kernels load words in pairs
  std::vector<uint16_t> off((size_t)nnz);
  std::vector<uint64_t> pl((size_t)(planes * nw), 0);
  par([&](int64_t b0, int64_t b1) {
    // blocks are 4 words wide, so threads never share a plane word
    for (int64_t b = b0; b < b1; ++b) {
      const int64_t k0 = b * B, k1 = std::min(nnz, k0 + B);
      for (int64_t k = k0; k < k1; ++k) {
        const uint32_t d = (uint32_t)(col[k] - base[(size_t)b]);
        off[(size_t)k] = (uint16_t)d;
        for (int p = 0; p < planes; ++p)
          pl[(size_t)(p * nw + (k >> 6))] |= (uint64_t)((d >> (16 + p)) & 1u) << (k & 63);
      }
    }
  });
  int rc;
  if ((rc = dev_alloc(&s.d_c16, 2 * (size_t)nnz, &s.bytes))) return rc;
  if ((rc = dev_alloc(&s.d_cbase, 4 * (size_t)(nb + 1), &s.bytes))) return rc;
  HIP_TRY(hipMemcpy(s.d_c16, off.data(), 2 * (size_t)nnz, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s.d_cbase, base.data(), 4 * (size_t)(nb + 1), hipMemcpyHostToDevice));
  if (planes) {
    if ((rc = dev_alloc(&s.d_cplanes, 8 * pl.size(), &s.bytes))) return rc;
    HIP_TRY(hipMemcpy(s.d_cplanes, pl.data(), 8 * pl.size(), hipMemcpyHostToDevice));
  }
  s.A.col16 = s.d_c16;
  s.A.cbase = s.d_cbase;
  s.A.cplanes = s.d_cplanes;
  s.A.n_cplanes = planes;
  s.A.cplane_words = (int32_t)nw;
  *used = true;
  return HSPMV_OK;
}

// Group-base 16-bit column offsets (STREAM): when every 64-row group's
// columns span < 65536, col = base[g] + off16 with one int32 base per
// group -- 2 instead of 4 index bytes per nonzero for one scalar load per
// group and one add per element, none of the per-256-nonzero base pairs,
// selects and planes of build_col16.  Auto: Infinity-Cache-resident
// matrices (C2: 15.56 -> 15.12 us in one process, bench 724-732 -> 754
// GFLOP/s); HBM-resident ones keep build_col16's blocks (C4 53.0 vs 55.4
// us with group bases, c3h/l4k within 1 %; profiles/r01_ab_col16_group*.jsonl).
// Tuning.col16_group = -1 disables, 1 uses it whenever it fits.  Split rows (read
// by the split-row kernels from the 32-bit columns) get offset 0.
// Row groups: STREAM's 64-row groups (starts == nullptr) or the packed CSR3
// wave tasks [starts[g], starts[g+1]).
int build_col16g(Shard &s, const int32_t *rp, const int32_t *col, int64_t m, int64_t n, int dtype,
                 unsigned flags, const std::vector<int32_t> *starts, bool *used) {
  *used = false;
  const int mode = s.tune.col16_group;  // -1 off, 0 auto, 1 on whenever it fits
  const int64_t nnz = rp[m];
  if (mode < 0 || (flags & HSPMV_FLAG_NO_COL16) || nnz == 0) return HSPMV_OK;
  const double sv = (double)dtype_size(dtype);
  const bool forced = (flags & HSPMV_FLAG_COL16) != 0 || mode == 1;
  if (!forced && (double)nnz * (sv + 4.0) + (double)m * (sv + 4.0) + (double)n * sv > kMallResident)
    return HSPMV_OK;
  const int32_t long_t = (flags & HSPMV_FLAG_NO_SPLIT) ? INT32_MAX : kLongRow;
  const int64_t ng = starts ? (int64_t)starts->size() - 1 : (m + 63) / 64;
  if (ng <= 0) return HSPMV_OK;
  auto rows = [&](int64_t g, int64_t &r0, int64_t &r1) {
    r0 = starts ? (*starts)[(size_t)g] : 64 * g;
    r1 = starts ? (*starts)[(size_t)g + 1] : std::min(m, 64 * g + 64);
  };
  std::vector<int32_t> base((size_t)ng + 1, 0);  // +1: read by 8-byte scalar loads
  std::vector<int32_t> span((size_t)ng, 0);
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(16, ng / 4096));
  auto par = [&](auto &&body) {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&, t]() { body(ng * t / nt, ng * (t + 1) / nt); });
    for (auto &x : th) x.join();
  };
  par([&](int64_t g0, int64_t g1) {
    for (int64_t g = g0; g < g1; ++g) {
      int32_t lo = INT32_MAX, hi = -1;
      int64_t ra, rb;
      rows(g, ra, rb);
      for (int64_t r = ra; r < rb; ++r) {
        if (rp[r + 1] - rp[r] > long_t) continue;
        for (int32_t k = rp[r]; k < rp[r + 1]; ++k) {
          lo = std::min(lo, col[k]);
          hi = std::max(hi, col[k]);
        }
      }
      base[(size_t)g] = hi >= 0 ? lo : 0;
      span[(size_t)g] = hi >= 0 ? hi - lo : 0;
    }
  });
  int32_t maxspan = 0;
  for (int32_t v : span) maxspan = std::max(maxspan, v);
  if (maxspan > 65535) return HSPMV_OK;
  std::vector<uint16_t> off((size_t)nnz, 0);
  par([&](int64_t g0, int64_t g1) {
    for (int64_t g = g0; g < g1; ++g) {
      int64_t ra, rb;
      rows(g, ra, rb);
      for (int64_t r = ra; r < rb; ++r) {
        if (rp[r + 1] - rp[r] > long_t) continue;
        for (int32_t k = rp[r]; k < rp[r + 1]; ++k) off[(size_t)k] = (uint16_t)(col[k] - base[(size_t)g]);
      }
    }
  });
  int rc;
  if ((rc = dev_alloc(&s.d_c16, 2 * (size_t)nnz, &s.bytes))) return rc;
  if ((rc = dev_alloc(&s.d_cbase, 4 * base.size(), &s.bytes))) return rc;
  HIP_TRY(hipMemcpy(s.d_c16, off.data(), 2 * (size_t)nnz, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s.d_cbase, base.data(), 4 * base.size(), hipMemcpyHostToDevice));
  int bits = 0;
  while (bits < 31 && (int64_t(1) << bits) <= maxspan) ++bits;
  s.A.col_span_bits = std::max(1, bits);
  s.A.col16 = s.d_c16;
  s.A.cbase = s.d_cbase;
  s.A.cplanes = nullptr;
  s.A.n_cplanes = 0;
  s.A.c16_mode = 2;
  s.c16g_shape = starts ? kCsr3 : kStream;
  *used = true;
  return HSPMV_OK;
}

// CSR-3 task packing (the default CSR-3 plan): the super-rows of the inner
// map, in order, are packed into wave tasks of at most one 64-row group
// (the lanes of a wave's ordered sums); a super-row longer than 64 rows is
// cut at 64-row steps.  Four consecutive tasks form a workgroup, so a
// super-super-row spans as many waves as its rows need instead of a fixed W
// per launch (handCoarsen's super-super-rows vary ~10x in rows).
// Tuning.csr3_plan = HSPMV_CSR3_PLAN_SSR selects the workgroup-per-super-
// super-row plan (ssr_tasks).
bool csr3_packed(const Tuning &t) { return t.csr3_plan != HSPMV_CSR3_PLAN_SSR; }

// The workgroup-per-super-super-row plan (the reference's cuSpMV_3 mapping,
// csrk.cu:245-319): W = ssr_waves(mean rows per SSR) tasks per SSR, each
// SSR's super-rows split W ways by nonzeros -- wave w starts at the first
// super-row reaching w/W of the SSR's nonzeros, but strictly after wave
// w-1's start while super-rows remain: two waves never share a start (an
// empty task beside a doubled one was 15 % of the tasks on a 64-row
// grouping: 144 -> 129 us there).  Row-granular cuts capped at 64 rows per
// wave measured 7-30 % slower on C3's groupings (long tails where an SSR
// exceeds W*64 rows); profiles/r01_ab_csr3_tasks.jsonl.  Built with the
// other host tables (not at plan time) so the block x dictionaries of the
// packed plans apply to it: block b = SSR b.
void ssr_tasks(const int32_t *rp, int64_t m, const std::vector<int32_t> &o,
               const std::vector<int32_t> &in, int W, std::vector<int32_t> &ts) {
  const int64_t nssr = (int64_t)o.size() - 1;
  ts.assign((size_t)(nssr * W + 1), 0);
  for (int64_t b = 0; b < nssr; ++b) {
    const int32_t s0 = o[(size_t)b], s1 = o[(size_t)b + 1];
    const int64_t k0 = rp[in[(size_t)s0]], k1 = rp[in[(size_t)s1]];
    int32_t sr = s0, prev = s0 - 1;
    for (int w = 0; w < W; ++w) {
      const int64_t target = k0 + (k1 - k0) * w / W;
      while (sr < s1 && rp[in[(size_t)sr]] < target) ++sr;
      int32_t st = w == 0 ? s0 : sr;
      if (st <= prev) st = prev + 1;
      const int32_t latest = s1 - (W - w);  // leave one super-row per later wave
      if (st > latest) st = std::max(prev + 1, latest);
      if (st > s1) st = s1;
      ts[(size_t)(b * W + w)] = in[(size_t)st];
      prev = st;
      sr = std::max(sr, st);
    }
  }
  ts[(size_t)(nssr * W)] = (int32_t)m;
}

// The SSR plan's aligned cut (Tuning.ssr_align): the same one workgroup of W
// waves per super-super-row, but the waves take the SSR's 64-row ALIGNED
// pieces -- [R0, next multiple of 64), whole aligned groups, [last multiple,
// R1) -- instead of nonzero-balanced runs of whole super-rows, so a wave's
// y stores cover whole cache lines except at the SSR's two edges (the
// kernel's groups end on multiples of 64: DevPlan.task_align).  With more
// pieces than waves, the adjacent pair with the fewest nonzeros merges until
// W remain; with fewer, the last waves get empty tasks.
bool ssr_aligned(const Tuning &t) { return t.csr3_plan == HSPMV_CSR3_PLAN_SSR && t.ssr_align == 1; }

// The SSR plan's wave cut (Tuning.ssr_align): 2 (default) row-granular
// nonzero balance, 0 the super-row-granular cut (ssr_tasks), 1 aligned
// pieces (ssr_tasks_aligned).
int ssr_cut(const Tuning &t) { return t.ssr_align < 0 ? 2 : t.ssr_align; }

// ssr_align = 2, the default since r05: the SSR's rows split W ways by
// nonzeros at ROW granularity (wave w starts at the first row reaching w/W
// of the SSR's nonzeros), so the waves of a workgroup carry equal work
// whatever the super-rows' sizes -- the workgroup's LDS is held until its
// slowest wave ends; a wave may run more than 64 rows (several groups).
// One process (profiles/r05u/ab_ssr_rows.jsonl): C3 120.7 -> 118.2 us,
// the MI355X grouping (64, 4) 126.6 -> 121.3, fp32 71.8 -> 71.5.  (r01's
// row-granular cut capped waves at 64 rows and lost 7-30 % to long tails.)
void ssr_tasks_rows(const int32_t *rp, int64_t m, const std::vector<int32_t> &o,
                    const std::vector<int32_t> &in, int W, std::vector<int32_t> &ts) {
  const int64_t nssr = (int64_t)o.size() - 1;
  ts.assign((size_t)(nssr * W + 1), 0);
  for (int64_t b = 0; b < nssr; ++b) {
    const int32_t R0 = in[(size_t)o[(size_t)b]], R1 = in[(size_t)o[(size_t)b + 1]];
    const int64_t k0 = rp[R0], k1 = rp[R1];
    int32_t r = R0;
    for (int w = 0; w < W; ++w) {
      const int64_t target = k0 + (k1 - k0) * w / W;
      while (r < R1 && rp[r] < target) ++r;
      ts[(size_t)(b * W + w)] = w == 0 ? R0 : r;
    }
  }
  ts[(size_t)(nssr * W)] = (int32_t)m;
}

void ssr_tasks_aligned(const int32_t *rp, int64_t m, const std::vector<int32_t> &o,
                       const std::vector<int32_t> &in, int W, std::vector<int32_t> &ts) {
  const int64_t nssr = (int64_t)o.size() - 1;
  ts.assign((size_t)(nssr * W + 1), 0);
  std::vector<int32_t> cut;
  for (int64_t b = 0; b < nssr; ++b) {
    const int32_t R0 = in[(size_t)o[(size_t)b]], R1 = in[(size_t)o[(size_t)b + 1]];
    cut.clear();
    cut.push_back(R0);
    for (int32_t a = (R0 & ~63) + 64; a < R1; a += 64) cut.push_back(a);
    cut.push_back(R1);
    while ((int)cut.size() - 1 > W) {  // merge the lightest adjacent pair
      size_t best = 1;
      int64_t bn = INT64_MAX;
      for (size_t i = 1; i + 1 < cut.size(); ++i) {
        const int64_t nz = (int64_t)rp[cut[i + 1]] - rp[cut[i - 1]];
        if (nz < bn) {
          bn = nz;
          best = i;
        }
      }
      cut.erase(cut.begin() + (ptrdiff_t)best);
    }
    for (int w = 0; w < W; ++w)
      ts[(size_t)(b * W + w)] = w + 1 < (int)cut.size() ? cut[(size_t)w] : R1;
  }
  ts[(size_t)(nssr * W)] = (int32_t)m;
}

// Task cut of the packed CSR-3 plan: 64-row groups aligned to multiples of 64
// rows (default), or whole super-rows packed up to 64 rows
// (Tuning.csr3_plan = HSPMV_CSR3_PLAN_PACKED, pack_csr3_tasks).  The row sums are row-local, so y is
// the same bit for bit either way; what differs is the y stores: a wave's 64
// rows are 512 B (fp64) / 256 B (fp32) on cache-line boundaries, where C3's
// ten-row super-rows gave 60-row tasks whose stores split lines between two
// waves.  C3 fp64 111.0 -> 109.6 us and 110.2 -> 109.4 in two one-process
// A/Bs of the default configuration (profiles/r02ab_ab_c3_tasks.jsonl,
// r02ac/).  The super-super-rows still bound the shards of the multi-GPU
// split.
bool csr3_fill(const Tuning &t) { return t.csr3_plan != HSPMV_CSR3_PLAN_PACKED; }

void pack_csr3_tasks(const std::vector<int32_t> &in, int32_t m, std::vector<int32_t> &ts) {
  constexpr int32_t kTaskRows = 64;  // one wave's lanes
  ts.clear();
  ts.reserve((size_t)m / 32 + 2);
  int32_t start = 0;
  const int64_t nsr = (int64_t)in.size() - 1;
  for (int64_t sr = 0; sr < nsr; ++sr) {
    const int32_t r0 = in[(size_t)sr], r1 = in[(size_t)sr + 1];
    if (r1 - start <= kTaskRows) continue;  // the super-row joins the open task
    if (r0 > start) {                   // close the open task before it
      ts.push_back(start);
      start = r0;
    }
    while (r1 - start > kTaskRows) {  // a long super-row: 64-row steps
      ts.push_back(start);
      start += kTaskRows;
    }
  }
  while (m - start > kTaskRows) {  // rows past the maps (none for validated maps)
    ts.push_back(start);
    start += kTaskRows;
  }
  if (start < m || ts.empty()) ts.push_back(start);
  ts.push_back(m);
}

// Heavy tasks.  A wave's task is also capped at a nonzero budget (in-kernel
// rows only: split rows are summed elsewhere), cut at row boundaries: with
// 64 rows of 512-2048 nonzeros one wave would stream 32-128 K nonzeros and a
// 25 K-row matrix would fill only 381 waves (d2048: 3.9 ms against 120 us
// for a wave per row, profiles/r02z2_ab_vector.jsonl).  Tuning.task_nnz
// moves the budget.
constexpr int32_t kTaskNnz = 2048;

int32_t task_nnz_budget(const Tuning &t) { return t.task_nnz > 0 ? t.task_nnz : kTaskNnz; }

void cap_task_nnz(const int32_t *rp, int32_t long_t, int32_t budget, std::vector<int32_t> &ts) {
  std::vector<int32_t> out;
  out.reserve(ts.size());
  for (size_t t = 0; t + 1 < ts.size(); ++t) {
    const int32_t a = ts[t], b = ts[t + 1];
    out.push_back(a);
    int64_t acc = 0;
    for (int32_t r = a; r < b; ++r) {
      const int64_t len = rp[r + 1] - rp[r] > long_t ? 0 : rp[r + 1] - rp[r];
      if (r > out.back() && acc + len > budget) {
        out.push_back(r);
        acc = 0;
      }
      acc += len;
    }
  }
  out.push_back(ts.back());
  ts.swap(out);
}

// The wave tasks of a shard (empty: STREAM's fixed 64-row groups) and the
// tasks per workgroup (*waves).  CSR-3: 64-row aligned groups or packed
// super-rows, 4 per workgroup; or the SSR plan's W per super-super-row.
// CSR under the auto (or CSR3) kernel: when at least a quarter of the
// in-kernel nonzeros sit in 64-row groups over the budget, the 64-row groups
// with the heavy ones cut -- the CSR3 kernel then runs them (a CSR-2 with
// one-row super-rows).  All but the SSR tasks are capped at the budget.
void build_tasks(const int32_t *rp, int64_t m, const std::vector<int32_t> *inner,
                 const std::vector<int32_t> *outer, unsigned flags, const Tuning &tune,
                 std::vector<int32_t> &ts, int *waves) {
  ts.clear();
  *waves = 4;
  if (!csr3_packed(tune)) {
    if (!inner || !outer || outer->size() < 2) return;
    *waves = (tune.ssr_w == 1 || tune.ssr_w == 2 || tune.ssr_w == 4 || tune.ssr_w == 8)
                 ? tune.ssr_w  // A/B knob (diagnostic builds)
                 : ssr_waves((double)m / (double)(outer->size() - 1));
    if (ssr_aligned(tune))
      ssr_tasks_aligned(rp, m, *outer, *inner, *waves, ts);
    else if (ssr_cut(tune) == 2)
      ssr_tasks_rows(rp, m, *outer, *inner, *waves, ts);
    else
      ssr_tasks(rp, m, *outer, *inner, *waves, ts);
    return;
  }
  const int32_t long_t = (flags & HSPMV_FLAG_NO_SPLIT) ? INT32_MAX : kLongRow;
  const int32_t budget = task_nnz_budget(tune);
  if (inner && csr3_fill(tune)) {
    for (int64_t g = 0; g < m; g += 64) ts.push_back((int32_t)g);
    if (ts.empty()) ts.push_back(0);
    ts.push_back((int32_t)m);
  } else if (inner) {
    pack_csr3_tasks(*inner, (int32_t)m, ts);
  } else {
    const unsigned k = flags & 0xFu;
    if ((k != kAuto && k != kCsr3) || m == 0) return;
    int64_t heavy = 0, total = 0;
    for (int64_t g = 0; g < m; g += 64) {
      int64_t in = 0;
      for (int64_t r = g; r < std::min(m, g + 64); ++r) {
        const int64_t len = rp[r + 1] - rp[r];
        in += len > long_t ? 0 : len;
      }
      total += in;
      heavy += in > budget ? in : 0;
    }
    if (4 * heavy < total || heavy == 0) return;
    for (int64_t g = 0; g < m; g += 64) ts.push_back((int32_t)g);
    ts.push_back((int32_t)m);
  }
  cap_task_nnz(rp, long_t, budget, ts);
}

// x windows of row groups [starts[g], starts[g+1]) -- the 64-row groups of
// STREAM when starts is null, the packed CSR-3 tasks otherwise: {lo, w}
// when the group's columns span w <= kXWin entries, else {0, 0}.  Empty
// when fewer than half the groups fit (Tuning.x_windows = -1 disables).  Several
// windows per group (C2's Laplacian: three runs around r-1000, r, r+1000)
// were measured and dropped: 15.6 -> 17.2 us on C2, 210 -> 232 us on a
// 4000^2 Laplacian (profiles/r01_ab_xwin_multi.jsonl) -- the staging and
// its registers cost more than gathers that hit L2.
std::vector<int32_t> xwin_table(const int32_t *rp, const int32_t *col, int64_t m,
                                const std::vector<int32_t> *starts, const Tuning &tune) {
  std::vector<int32_t> tab;
  if (tune.x_windows < 0) return tab;
  const int64_t ng = starts ? (int64_t)starts->size() - 1 : (m + 63) / 64;
  if (ng <= 0) return tab;
  tab.assign((size_t)(2 * ng), 0);
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(16, ng / 4096));
  std::vector<int64_t> fit((size_t)nt, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t]() {
      for (int64_t g = ng * t / nt; g < ng * (t + 1) / nt; ++g) {
        const int64_t r0 = starts ? (*starts)[(size_t)g] : 64 * g;
        const int64_t r1 = starts ? (*starts)[(size_t)g + 1] : std::min(m, 64 * g + 64);
        const int64_t k0 = rp[r0], k1 = rp[r1];
        if (k1 <= k0) continue;
        int32_t lo = col[k0], hi = col[k0];
        for (int64_t k = k0 + 1; k < k1; ++k) {
          lo = std::min(lo, col[k]);
          hi = std::max(hi, col[k]);
        }
        if ((int64_t)hi - lo + 1 <= kXWin) {
          tab[(size_t)(2 * g)] = lo;
          tab[(size_t)(2 * g + 1)] = hi - lo + 1;
          ++fit[(size_t)t];
        }
      }
    });
  for (auto &x : th) x.join();
  int64_t nfit = 0;
  for (int64_t f : fit) nfit += f;
  if (2 * nfit < ng) tab.clear();
  return tab;
}

// x slabs.  When the gathers are irregular (a 64-row group's columns span
// more than an XCD's 4 MiB L2 of x) and x itself exceeds the L2, nearly
// every gather misses L2 and pulls a whole line from the Infinity Fabric
// for 4-8 useful bytes (C5, power-law with random columns: ~48 M such
// misses, 443 us for 400 MB of matrix).  Cutting the columns into slabs
// of <= kSlabBytes of x and running the row kernel once per slab over a
// slab-major copy keeps each pass's gathers inside one L2-resident slice;
// the price per extra pass is one more row-pointer array and a y read +
// write.  Pass b > 0 starts each row from the y of pass b-1, so a row's
// products are still added left to right from 0 (bit-identical to
// omp_spmv for rows of <= kSerialMax (40) nonzeros per slab segment) -- which needs the
// row's columns to be non-decreasing slab by slab (sorted rows; checked).
// Tuning.x_slabs = -1 disables, B > 0 forces B slabs; Tuning.xslab_bytes
// (A/B) moves the slab size.
// Irregular gathers: one gather instruction of the row kernels covers 64
// consecutive nonzeros; when those fall on mostly distinct x cache lines
// (random / power-law / wide-band columns) every lane is its own L2 request
// and the row kernels run at the L2 request rate, whatever x's span.  Mean
// distinct 128-byte lines per 64 consecutive nonzeros, sampled over <= 16 K
// such runs: C2 5.3, C3 11.1, honeycomb 4.6, C4 5.0, d48/d512 banded 6.9 /
// 8.9 -- against C5 62.1 and the mixed-length +-4000 band 49.5 (row kernel
// 210 us, csort 130 us; profiles/r02z5_ab_mix.jsonl).  Irregular: >= 32.
// (The earlier test -- the median 64-row group spans more than 4 MiB of x
// -- missed the band.)
bool irregular_gathers(const int32_t *rp, const int32_t *col, int64_t m, double sv) {
  const int64_t nnz = rp[m];
  const int64_t runs = nnz / 64;
  if (runs == 0) return false;
  const int64_t step = std::max<int64_t>(1, runs / 16384);
  const int32_t per_line = (int32_t)(128.0 / sv);
  int64_t lines = 0, sampled = 0;
  int32_t c[64];
  for (int64_t r = 0; r < runs; r += step) {
    for (int j = 0; j < 64; ++j) c[j] = col[r * 64 + j] / per_line;
    std::sort(c, c + 64);
    int d = 1;
    for (int j = 1; j < 64; ++j) d += c[j] != c[j - 1];
    lines += d;
    ++sampled;
  }
  return lines >= 32 * sampled;
}

// Median over (up to 16 K sampled) 64-row groups of the columns a group
// spans (max - min + 1; empty groups skipped).
double median_group_span(const int32_t *rp, const int32_t *col, int64_t m) {
  const int64_t groups = (m + 63) / 64;
  const int64_t step = std::max<int64_t>(1, groups / 16384);
  std::vector<int64_t> spans;
  for (int64_t g = 0; g < groups; g += step) {
    const int64_t r0 = g * 64, r1 = std::min(m, r0 + 64);
    int32_t lo = INT32_MAX, hi = -1;
    for (int64_t r = r0; r < r1; ++r)
      for (int32_t k = rp[r]; k < rp[r + 1]; ++k) {
        lo = std::min(lo, col[k]);
        hi = std::max(hi, col[k]);
      }
    if (hi >= lo) spans.push_back((int64_t)hi - lo + 1);
  }
  if (spans.empty()) return 0.0;
  std::nth_element(spans.begin(), spans.begin() + (ptrdiff_t)(spans.size() / 2), spans.end());
  return (double)spans[spans.size() / 2];
}

constexpr double kSlabBytes = 2.0 * 1024 * 1024;
constexpr int kMaxSlabs = 32;

int build_xslabs(Shard &s, const int32_t *rp, const int32_t *col, const void *val, int64_t m,
                 int64_t n, int dtype, unsigned flags) {
  s.n_slabs = 0;
  const int forced = s.tune.x_slabs < 0 ? 0 : (s.tune.x_slabs > 0 ? s.tune.x_slabs : -1);  // -1 auto, 0 off, B slabs
  if (forced == 0 || !val || m == 0 || n == 0 || (flags & 0xFu) == kVector) return HSPMV_OK;
  const int64_t nnz = rp[m];
  const double sv = (double)dtype_size(dtype);
  const double slab_bytes = s.tune.xslab_bytes > 0 ? std::max(4096.0, s.tune.xslab_bytes) : kSlabBytes;
  int B = forced > 0 ? forced : (int)std::ceil((double)n * sv / slab_bytes);
  B = (int)std::min<int64_t>(std::min(B, kMaxSlabs), n);
  if (B < 2) return HSPMV_OK;
  const int32_t long_t = (flags & HSPMV_FLAG_NO_SPLIT) ? INT32_MAX : kLongRow;
  const int64_t W = (n + B - 1) / B;  // columns per slab
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(16, m / 65536));
  auto par = [&](auto &&body) {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&, t]() { body(t); });
    for (auto &x : th) x.join();
  };
  if (forced < 0) {
    const double footprint = (double)nnz * (sv + 4.0) + (double)m * (sv + 4.0) + (double)n * sv;
    if (footprint <= kMallResident || (double)n * sv <= 4.0 * 1024 * 1024) return HSPMV_OK;
    // the passes must pay: every extra one re-reads a row-pointer array and
    // y and rewrites y (at most a quarter of the matrix stream in total),
    // and each pass must stream millions of nonzeros (a launch is ~2-5 us)
    const double extra = (double)(B - 1) * (4.0 * (double)(m + 1) + 2.0 * sv * (double)m);
    if (extra > 0.25 * (double)nnz * (sv + 4.0) || (double)nnz / B < 2.0e6) return HSPMV_OK;
    if (!irregular_gathers(rp, col, m, sv)) return HSPMV_OK;
    // ... and only when the x a row group gathers from is wider than an
    // XCD's L2 (median 64-row group column span > 4 MiB of x): scattered but
    // local gathers (a +-4000 band of random columns, `mix`) stay L2 hits
    // without slabs, and the extra passes only cost (deterministic handles
    // on mix: 284 us with four slabs vs 209 without; profiles/r04/
    // sweep_deterministic.jsonl)
    if (median_group_span(rp, col, m) * sv <= 4.0 * 1024 * 1024) return HSPMV_OK;
  }
  // per (slab, row) segment lengths; rows must be slab-monotone
  std::vector<int32_t> srp((size_t)B * (size_t)(m + 1), 0);
  std::atomic<bool> unsorted{false};
  par([&](int t) {
    for (int64_t r = m * t / nt; r < m * (t + 1) / nt; ++r) {
      const int32_t k0 = rp[r], k1 = rp[r + 1];
      if (k1 - k0 > long_t) continue;  // split rows: empty segments
      int64_t prev = 0;
      for (int32_t k = k0; k < k1; ++k) {
        const int64_t b = col[k] / W;
        if (b < prev) { unsorted = true; return; }
        prev = b;
        ++srp[(size_t)b * (size_t)(m + 1) + (size_t)r + 1];
      }
    }
  });
  if (unsorted) return HSPMV_OK;
  int64_t base = 0;  // slab-major offsets
  for (int b = 0; b < B; ++b) {
    int32_t *p = srp.data() + (size_t)b * (size_t)(m + 1);
    p[0] = (int32_t)base;
    for (int64_t r = 0; r < m; ++r) p[r + 1] += p[r];
    base = p[m];
  }
  const int64_t snnz = base;  // in-kernel nonzeros (split rows excluded)
  std::vector<int32_t> scol((size_t)std::max<int64_t>(snnz, 1));
  std::vector<char> sval((size_t)std::max<int64_t>(snnz, 1) * (size_t)sv);
  par([&](int t) {
    for (int64_t r = m * t / nt; r < m * (t + 1) / nt; ++r) {
      const int32_t k0 = rp[r], k1 = rp[r + 1];
      if (k1 - k0 > long_t) continue;
      int32_t k = k0;
      for (int b = 0; b < B; ++b) {
        const int32_t *p = srp.data() + (size_t)b * (size_t)(m + 1);
        for (int32_t o = p[r]; o < p[r + 1]; ++o, ++k) {
          scol[(size_t)o] = col[k];
          memcpy(sval.data() + (size_t)o * (size_t)sv, (const char *)val + (size_t)k * (size_t)sv,
                 (size_t)sv);
        }
      }
    }
  });
  int rc;
  if ((rc = dev_alloc(&s.d_slab_rp, 4 * srp.size(), &s.bytes))) return rc;
  if ((rc = dev_alloc(&s.d_slab_col, 4 * scol.size(), &s.bytes))) return rc;
  if ((rc = dev_alloc(&s.d_slab_val, sval.size(), &s.bytes))) return rc;
  HIP_TRY(hipMemcpy(s.d_slab_rp, srp.data(), 4 * srp.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s.d_slab_col, scol.data(), 4 * scol.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s.d_slab_val, sval.data(), sval.size(), hipMemcpyHostToDevice));
  s.n_slabs = B;
  return HSPMV_OK;
}

// Which row kernel streams the x-slab passes of a handle that has CSR-3
// tasks (irregular gathers from a wide x with the column-sorted kernel off:
// deterministic handles, csort = -1).  The CSR3 tasks are capped at 2048
// nonzeros, so they balance 64-row groups a power-law ordering makes heavy;
// where the groups are balanced anyway the task table only costs.  r04 zoo
// (DESIGN.md §10): C5's random row order -- 6.5 % of the nonzeros in heavy
// groups -- STREAM 263 vs CSR3 313 us; c5r, the same rows RCM-ordered --
// 19.2 % heavy, the largest group 61.6 K nonzeros -- CSR3 307 vs STREAM 435.
// The cut at 1/8 of the nonzeros separates the two.  A rule, not a timing
// trial: a deterministic handle's y must not depend on which kernel won a
// race at creation (the two kernels sum rows above kSerialMax nonzeros in
// different orders).
constexpr double kSlabHeavyShare = 0.125;

void slab_kernel_rule(Shard &s, const int32_t *rp, int64_t m, unsigned flags) {
  const int32_t long_t = (flags & HSPMV_FLAG_NO_SPLIT) ? INT32_MAX : kLongRow;
  int64_t heavy = 0, total = 0;
  for (int64_t g = 0; g < m; g += 64) {
    int64_t in = 0;
    for (int64_t r = g; r < std::min(m, g + 64); ++r) {
      const int64_t len = rp[r + 1] - rp[r];
      in += len > long_t ? 0 : len;
    }
    total += in;
    heavy += in > task_nnz_budget(s.tune) ? in : 0;
  }
  s.heavy_frac = total ? (double)heavy / (double)total : 0.0;
  s.A.slab_stream = s.heavy_frac < kSlabHeavyShare;
}

// Host-side tables that need the columns (built at upload, while they are
// at hand): the CSR-3 packed tasks, the block x dictionaries, and (without
// dictionaries) the 16-bit column offsets and the x windows of both row
// kernels.
int build_row_tables(Shard &s, const int32_t *rp, const int32_t *col, const void *val, int64_t m,
                     int64_t n, int dtype, unsigned flags) {
  // the typical serially summed row (median length of the rows of 1..40
  // nonzeros, spmv_device.cuh kSerialMax): the planner's LDS bank rule
  {
    constexpr int kSerial = kSerialMax;
    int64_t hist[kSerial + 1] = {0}, tot = 0;
    for (int64_t r = 0; r < m; ++r) {
      const int64_t len = rp[r + 1] - rp[r];
      if (len >= 1 && len <= kSerial) {
        ++hist[len];
        ++tot;
      }
    }
    int32_t med = 0;
    for (int64_t acc = 0; med < kSerial && 2 * acc < tot;) acc += hist[++med];
    s.A.serial_len = tot ? med : 0;
  }
  int waves = 4;
  build_tasks(rp, m, s.A.n_ssr > 0 ? &s.h_inner : nullptr, s.A.n_ssr > 0 ? &s.h_outer : nullptr,
              flags, s.tune, s.h_tasks, &waves);
  s.A.task_waves = waves;
  s.h_xwin.clear();
  s.h_xwin_t.clear();
  int rc;
  {
    const unsigned kf = flags & 0xFu;
    const int cm = s.tune.csort;  // -1 off, 0 auto, 1 whenever it can be built
    const double sv = (double)dtype_size(dtype);
    const double footprint = (double)rp[m] * (sv + 4.0) + (double)m * (sv + 4.0) + (double)n * sv;
    // an ordered or serial handle (deterministic = 1, 3) never builds the
    // csort tables: the planner would pick kCsort whenever they exist
    // (plan_launch); a reproducible one (2) builds them with fixed-point slots
    const bool ordered = s.tune.deterministic == 1 || s.tune.deterministic == 3;
    bool want = !ordered && (kf == kCsort || cm == 1);
    // Scattered gathers from an x the L1 cannot hold go to the L2 one line
    // per nonzero, at its request rate, whatever the L2's capacity: until r04
    // the rule also asked for x beyond an XCD's 4 MiB L2, which kept fp32
    // `mix` (x = 3.8 MiB, random columns within +-4000) on the CSR3 kernel
    // at 90.8 us against csort's 62.5 (profiles/r04/auto_regret_f32.jsonl);
    // x of a few L1s (the zoo's `tall`, 16-32 KiB) stays on the row kernels.
    if (!want && kf == kAuto && cm == 0 && !ordered && s.tune.x_slabs == 0 &&
        footprint > kMallResident && (double)n * sv > 256.0 * 1024)
      want = irregular_gathers(rp, col, m, sv);
    if (want) {
      if ((rc = build_csort(s, rp, col, val, m, n, dtype, flags))) return rc;
      if (s.A.has_csort) {
        s.A.col_span_bits = 31;
        return HSPMV_OK;
      }
    }
  }
  if ((rc = build_xslabs(s, rp, col, val, m, n, dtype, flags))) return rc;
  if (s.n_slabs) {  // slab passes read 32-bit columns from global x
    s.A.col_span_bits = 31;
    s.A.n_slabs = s.n_slabs;
    if (!s.h_tasks.empty()) slab_kernel_rule(s, rp, m, flags);
    return HSPMV_OK;
  }
  s.h_xwin = xwin_table(rp, col, m, nullptr, s.tune);
  s.h_xwin_t.clear();
  if (!s.h_tasks.empty()) s.h_xwin_t = xwin_table(rp, col, m, &s.h_tasks, s.tune);
  const int kern = kernel_for_tables(s.A.n_ssr, !s.h_tasks.empty(), flags);
  const bool have_xwin = kern == kCsr3 ? !s.h_xwin_t.empty() : !s.h_xwin.empty();
  if ((rc = build_xdict(s, rp, col, m, n, dtype, flags, have_xwin))) return rc;
  if (s.xd_shape) {  // col_span_bits: the planner's gather-regularity hint
    s.h_xwin.clear();
    s.h_xwin_t.clear();
    s.A.col_span_bits = 1;
    s.A.has_xdict = s.xd_shape == kStream;
    s.A.has_xdict_tasks = s.xd_shape == kCsr3;
    return HSPMV_OK;
  }
  s.A.has_xwin = !s.h_xwin.empty();
  bool c16 = false;
  if (kern == kStream && (rc = build_col16g(s, rp, col, m, n, dtype, flags, nullptr, &c16))) return rc;
  if (kern == kCsr3 && (rc = build_col16g(s, rp, col, m, n, dtype, flags, &s.h_tasks, &c16))) return rc;
  if (!c16 && (rc = build_col16(s, col, rp[m], m, n, dtype, flags, &c16))) return rc;
  return HSPMV_OK;
}

// Host planner tables for one shard (needs s.h_rp): split rows (rows longer
// than kLongRow, cut into kLongChunk pieces), and the device copies of the
// tables build_row_tables planned (wave tasks, x windows).
int build_plan_tables(Shard &s, int dtype, unsigned flags) {
  const std::vector<int32_t> &rp = s.h_rp;
  const int64_t m = s.A.m;
  s.dp = DevPlan();
  s.dp.serial_max = dtype == HSPMV_F32 ? kSerialMaxF32 : kSerialMax;
  if (s.tune.deterministic == HSPMV_DETERMINISTIC_SERIAL) {  // every row by one lane, in order
    if (s.plan.kernel != kStream && s.plan.kernel != kCsr3)
      return set_error(HSPMV_E_INVALID, "deterministic = 3 (serial order) needs the row kernels, and "
                                        "they cannot address this matrix (32-bit offsets)");
    s.dp.serial_max = INT32_MAX;
  } else if (s.tune.serial_max > 0) {
    s.dp.serial_max = s.tune.serial_max;  // A/B knob (HSPMV_SERIAL_MAX, diagnostic builds)
  }
  int64_t long_nnz = 0;
  if (s.plan.kernel == kCsort) {  // long rows are slices of the csort blocks
    s.dp.cs = s.csort;
    s.plan.blocks = s.csort.n_wg;
    s.plan.u = s.csort.u;
    const double alg = hspmv_alg_bytes(s.A.m, s.x_entries, s.A.nnz, dtype, 0, 0);
    s.c16_saved = alg - s.csort_format_bytes;
    return HSPMV_OK;
  }
  if (s.plan.kernel != kVector && !(flags & HSPMV_FLAG_NO_SPLIT)) {
    std::vector<int32_t> lrow, lcs(1, 0), ck;
    for (int64_t r = 0; r < m; ++r) {
      const int32_t b = rp[r], e = rp[r + 1];
      if (e - b <= kLongRow) continue;
      long_nnz += e - b;
      lrow.push_back((int32_t)r);
      for (int32_t k = b; k < e; k += kLongChunk) {
        ck.push_back(k);
        ck.push_back(e - k > kLongChunk ? k + kLongChunk : e);
      }
      lcs.push_back((int32_t)(ck.size() / 2));
    }
    if (!lrow.empty() && s.dp.serial_max == INT32_MAX) {  // serial order: one workgroup per row
      int rc;
      const int64_t nl = (int64_t)lrow.size();
      if ((rc = dev_alloc(&s.d_long_row, 4 * (size_t)nl, &s.bytes))) return rc;
      if ((rc = dev_alloc(&s.d_partials, dtype_size(dtype) * (size_t)nl, &s.bytes))) return rc;
      HIP_TRY(hipMemcpy(s.d_long_row, lrow.data(), 4 * (size_t)nl, hipMemcpyHostToDevice));
      s.dp.partials = s.d_partials;  // the rows' sums, scattered into y after the row kernel
      s.dp.long_t = kLongRow;
      s.dp.n_long = (int32_t)nl;
      s.dp.long_row = s.d_long_row;
      s.dp.long_serial = true;
      HIP_TRY(hipStreamCreateWithFlags(&s.long_stream, hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&s.long_fork, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&s.long_join, hipEventDisableTiming));
      s.dp.long_stream = s.long_stream;
      s.dp.long_fork = s.long_fork;
      s.dp.long_join = s.long_join;
    } else if (!lrow.empty()) {
      int rc;
      const int64_t nl = (int64_t)lrow.size(), nc = (int64_t)ck.size() / 2;
      if ((rc = dev_alloc(&s.d_long_row, 4 * (size_t)nl, &s.bytes))) return rc;
      if ((rc = dev_alloc(&s.d_long_cstart, 4 * (size_t)(nl + 1), &s.bytes))) return rc;
      if ((rc = dev_alloc(&s.d_chunk_k, 8 * (size_t)nc, &s.bytes))) return rc;
      if ((rc = dev_alloc(&s.d_partials, dtype_size(dtype) * (size_t)nc, &s.bytes))) return rc;
      HIP_TRY(hipMemcpy(s.d_long_row, lrow.data(), 4 * (size_t)nl, hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(s.d_long_cstart, lcs.data(), 4 * (size_t)(nl + 1), hipMemcpyHostToDevice));
      HIP_TRY(hipMemcpy(s.d_chunk_k, ck.data(), 8 * (size_t)nc, hipMemcpyHostToDevice));
      s.dp.long_t = kLongRow;
      s.dp.n_long = (int32_t)nl;
      s.dp.n_chunks = (int32_t)nc;
      s.dp.long_row = s.d_long_row;
      s.dp.long_cstart = s.d_long_cstart;
      s.dp.chunk_k = s.d_chunk_k;
      s.dp.partials = s.d_partials;
    }
  }
  if (s.plan.kernel == kVector) {
    s.A.col16 = nullptr;  // the vector kernel reads 32-bit columns
    s.A.cbase = nullptr;
    s.A.cplanes = nullptr;
    s.A.n_cplanes = 0;
  }
  if (s.xd_shape) {
    const bool fits = (s.xd_shape == kStream && s.plan.kernel == kStream && s.plan.groups == 1 &&
                       s.plan.waves_per_block == 4) ||
                      (s.xd_shape == kCsr3 && s.plan.kernel == kCsr3 && !s.h_tasks.empty() &&
                       s.plan.waves_per_block == s.A.task_waves);
    if (fits) {
      s.dp.xd_blk = s.d_xd_blk;
      s.dp.xd_runs = s.d_xd_runs;
      s.dp.xd_lds_bytes = s.xd_lds_bytes;
      // index bytes: 2 instead of 4 per in-kernel nonzero, plus the tables;
      // x: the staged entries instead of the distinct columns
      const double sv = (double)dtype_size(dtype);
      s.c16_saved = 2.0 * (double)(s.A.nnz - long_nnz) - 4.0 * (double)(s.xd_runs_n * 2) -
                    4.0 * (double)s.plan.blocks - sv * (double)(s.xd_entries - s.x_entries);
    } else {  // planned for another block shape: the kernels read the 32-bit columns
      s.A.col16 = nullptr;
    }
  } else if (s.A.col16 && s.A.c16_mode == 2 &&
             (s.plan.kernel != s.c16g_shape || (s.plan.kernel == kCsr3 && s.h_tasks.empty()))) {
    s.A.col16 = nullptr;  // group bases built for another row grouping: 32-bit columns
    s.A.cbase = nullptr;
  } else if (s.A.col16 && s.A.c16_mode == 2) {
    const int64_t ngb = s.plan.kernel == kCsr3 ? (int64_t)s.h_tasks.size() - 1 : (s.A.m + 63) / 64;
    s.c16_saved = 2.0 * (double)(s.A.nnz - long_nnz) - 4.0 * (double)ngb;
  } else if (s.A.col16) {
    const int64_t nb = (s.A.nnz + (int64_t(1) << kC16Shift) - 1) >> kC16Shift;
    s.c16_saved = 2.0 * (double)(s.A.nnz - long_nnz) - 4.0 * (double)nb -
                  (double)s.A.n_cplanes * (double)(s.A.nnz - long_nnz) / 8.0;
  }
  if (s.n_slabs && (s.plan.kernel == kStream || s.plan.kernel == kCsr3)) {
    s.dp.n_slabs = s.n_slabs;
    s.dp.slab_rp = s.d_slab_rp;
    s.dp.slab_col = s.d_slab_col;
    s.dp.slab_val = s.d_slab_val;
    // per extra pass: one more row-pointer array, and y read back + rewritten
    const double sv = (double)dtype_size(dtype);
    s.c16_saved = -(double)(s.n_slabs - 1) * (4.0 * (double)(m + 1) + 2.0 * sv * (double)m);
  }
  const std::vector<int32_t> &xw = s.plan.kernel == kStream ? s.h_xwin : s.h_xwin_t;
  if ((s.plan.kernel == kStream || (s.plan.kernel == kCsr3 && !s.h_tasks.empty())) && !xw.empty()) {
    int rc;
    if ((rc = dev_alloc(&s.d_xwin, 4 * xw.size(), &s.bytes))) return rc;
    HIP_TRY(hipMemcpy(s.d_xwin, xw.data(), 4 * xw.size(), hipMemcpyHostToDevice));
    s.dp.xwin = s.d_xwin;
  }
  std::vector<int32_t>().swap(s.h_xwin);
  std::vector<int32_t>().swap(s.h_xwin_t);
  if (s.plan.kernel == kCsr3 && !s.h_tasks.empty()) {
    int rc;
    if ((rc = dev_alloc(&s.d_task, 4 * s.h_tasks.size(), &s.bytes))) return rc;
    HIP_TRY(hipMemcpy(s.d_task, s.h_tasks.data(), 4 * s.h_tasks.size(), hipMemcpyHostToDevice));
    s.dp.task_start = s.d_task;
    s.dp.n_tasks = (int32_t)(s.h_tasks.size() - 1);
    s.dp.task_align = ssr_aligned(s.tune) ? 1 : 0;
  }
  return HSPMV_OK;
}

}  // namespace hspmv
