// hspmv_xdict.cpp -- block x dictionaries
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

// Block x dictionaries.  Per workgroup (STREAM: 256 consecutive rows; CSR3:
// four consecutive packed tasks) the distinct columns its in-kernel rows
// reference, as runs of consecutive columns (gaps of <= kXdGap unused
// entries are bridged, so a run is one contiguous load); the kernel stages
// them in LDS once per workgroup and every nonzero's column becomes a 16-bit
// position in that copy.  The gathers (one per nonzero, spread over many L2
// lines) become contiguous loads plus ds_reads, and the index stream is
// 2 B/nnz with no bases or planes.  On C3 (27-point RCM stencil) 256 rows
// reference ~1500 distinct x in ~4 runs, against ~6800 nonzeros.
// Auto: matrices that stream from HBM, whose largest dictionary fits
// kXdCapBytes of LDS and whose staged entries are <= half the nonzeros;
// Tuning.x_dict = -1/1 turns it off / on (on: whenever it fits the cap),
// Tuning.x_dict_cap (bytes) moves the cap.  Splits rows (> kLongRow) keep
// their 32-bit columns (split-row kernels).
constexpr int32_t kXdGap = 8;
constexpr int32_t kXdMaxRuns = 63;          // run records per block live in one wave's lanes
constexpr int32_t kXdCapBytes = 20 * 1024;  // + 8-12 KB of product staging: 6 blocks/CU

// Which row kernel the planner will pick (plan_launch) for a shard with
// n_ssr super-super-rows and (CSR-3) packed tasks.
int kernel_for_tables(int64_t n_ssr, bool have_tasks, unsigned flags) {
  const unsigned k = flags & 0xFu;
  if (k == kVector) return kVector;
  if ((k == kCsr3 || k == kAuto) && n_ssr > 0)
    return have_tasks ? kCsr3 : -1;
  if ((k == kCsr3 || k == kAuto) && have_tasks) return kCsr3;  // CSR with heavy groups
  return kStream;
}

// The dictionaries of the workgroups whose rows are [bs[b], bs[b+1]).
struct XdPlan {
  std::vector<int32_t> blk;  // nb + 1 record ranges
  std::vector<int32_t> rec;  // {x_start, lds_off} per run, sentinel {0, entries} per block
  std::vector<uint16_t> pos; // per nonzero: position in its block's staged x (0 for split rows)
  std::vector<int32_t> total;  // entries per block
  int64_t entries = 0, in_kernel_nnz = 0;
  int32_t tmax = 0;
};

// false when some block needs more than cap entries.
bool plan_xdict(const int32_t *rp, const int32_t *col, const std::vector<int32_t> &bs,
                int32_t long_t, int64_t cap, bool fill, XdPlan &P) {
  const int64_t nb = (int64_t)bs.size() - 1;
  const int64_t nnz = rp[bs.back()];
  std::vector<std::vector<int32_t>> runs((size_t)nb);  // per block: start, end (inclusive) pairs
  std::vector<int32_t> total((size_t)nb, 0);
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(16, nb / 256));
  std::atomic<bool> fail{false};
  auto par = [&](auto &&body) {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&, t]() { body(nb * t / nt, nb * (t + 1) / nt); });
    for (auto &x : th) x.join();
  };
  par([&](int64_t b0, int64_t b1) {
    std::vector<int32_t> c;
    for (int64_t b = b0; b < b1 && !fail.load(std::memory_order_relaxed); ++b) {
      c.clear();
      for (int32_t r = bs[(size_t)b]; r < bs[(size_t)b + 1]; ++r)
        if (rp[r + 1] - rp[r] <= long_t) c.insert(c.end(), col + rp[r], col + rp[r + 1]);
      std::sort(c.begin(), c.end());
      c.erase(std::unique(c.begin(), c.end()), c.end());
      std::vector<int32_t> &R = runs[(size_t)b];
      for (int64_t gap = kXdGap;; gap *= 2) {  // bridge wider gaps until the runs fit a wave
        R.clear();
        for (int32_t v : c) {
          if (!R.empty() && (int64_t)v - R.back() <= gap) {
            R.back() = v;
          } else {
            R.push_back(v);
            R.push_back(v);
          }
        }
        if ((int64_t)R.size() / 2 <= kXdMaxRuns) break;
      }
      int64_t tot = 0;
      for (size_t i = 0; i < R.size(); i += 2) tot += (int64_t)R[i + 1] - R[i] + 1;
      if (tot > cap) fail = true;
      total[(size_t)b] = (int32_t)std::min<int64_t>(tot, INT32_MAX);
    }
  });
  if (fail) return false;
  P.total = total;
  int64_t nrec = 0;
  P.blk.assign((size_t)nb + 1, 0);
  P.entries = 0;
  P.tmax = 0;
  for (int64_t b = 0; b < nb; ++b) {
    P.entries += total[(size_t)b];
    P.tmax = std::max(P.tmax, total[(size_t)b]);
    P.blk[(size_t)b] = (int32_t)nrec;
    nrec += (int64_t)runs[(size_t)b].size() / 2 + 1;
  }
  P.blk[(size_t)nb] = (int32_t)nrec;
  P.in_kernel_nnz = 0;
  for (int32_t r = bs.front(); r < bs.back(); ++r)
    if (rp[r + 1] - rp[r] <= long_t) P.in_kernel_nnz += rp[r + 1] - rp[r];
  if (!fill) return true;
  P.rec.assign((size_t)(2 * nrec), 0);
  P.pos.assign((size_t)nnz, 0);
  par([&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b) {
      const std::vector<int32_t> &R = runs[(size_t)b];
      const int64_t nr = (int64_t)R.size() / 2;
      int32_t *o = P.rec.data() + 2 * (size_t)P.blk[(size_t)b];
      int32_t off = 0;
      for (int64_t i = 0; i < nr; ++i) {
        o[2 * i] = R[2 * i];
        o[2 * i + 1] = off;
        off += R[2 * i + 1] - R[2 * i] + 1;
      }
      o[2 * nr] = 0;
      o[2 * nr + 1] = off;  // sentinel: entries of the block
      for (int32_t r = bs[(size_t)b]; r < bs[(size_t)b + 1]; ++r) {
        if (rp[r + 1] - rp[r] > long_t) continue;
        for (int32_t k = rp[r]; k < rp[r + 1]; ++k) {
          // last run starting at or before col[k] (runs sorted by start)
          int64_t lo = 0, hi = nr - 1;
          while (lo < hi) {
            const int64_t mid = (lo + hi + 1) / 2;
            if (R[2 * mid] <= col[k]) lo = mid; else hi = mid - 1;
          }
          P.pos[(size_t)k] = (uint16_t)(o[2 * lo + 1] + (col[k] - R[2 * lo]));
        }
      }
    }
  });
  return true;
}

// Workgroup row ranges of the row kernel `kern` (STREAM: 256 rows; CSR3:
// four packed tasks).
// Packed CSR3 tasks per dictionary workgroup: 4, or 8 with Tuning.xd_waves
// (A/B; 512 rows share one dictionary: fewer staged entries per row, half
// the barriers, twice the LDS per block).
int xd_task_waves(const Tuning &t) { return t.xd_waves == 8 ? 8 : 4; }

// Tasks per dictionary block of a CSR3 task table: the SSR plan's W tasks
// per super-super-row (one workgroup each), else xd_task_waves.
int xd_block_tasks(const Tuning &t, int task_waves) {
  return t.csr3_plan == HSPMV_CSR3_PLAN_SSR ? task_waves : xd_task_waves(t);
}

std::vector<int32_t> xdict_blocks(int kern, int64_t m, const std::vector<int32_t> &tasks, int W) {
  std::vector<int32_t> bs;
  if (kern == kStream) {
    for (int64_t r = 0; r < m; r += 256) bs.push_back((int32_t)r);
    bs.push_back((int32_t)m);
  } else {
    const int64_t nt = (int64_t)tasks.size() - 1;
    for (int64_t t = 0; t < nt; t += W) bs.push_back(tasks[(size_t)t]);
    bs.push_back(tasks[(size_t)nt]);
  }
  return bs;
}

int64_t xdict_cap_entries(int dtype, const Tuning &t) {
  const int64_t cap_bytes = t.x_dict_cap > 0 ? t.x_dict_cap : kXdCapBytes;
  // <= 64 KiB of LDS (and 16-bit positions) whatever x_dict_cap asks
  return std::min<int64_t>(std::min<int64_t>(cap_bytes, 64 * 1024) / (int64_t)dtype_size(dtype),
                           65536);
}

// Blocks per CU the CSR3 dictionary workgroups are sized for.  The LDS of a
// workgroup is its product staging (W x 64 x U values) plus its dictionary,
// allocated in 1 KiB granules (C3 fp64: 8 KiB + 18.8 KiB ran 5 workgroups per
// CU, tools/block_trace.py).  A block whose dictionary would not fit 160 KiB
// / kXdBlocksPerCu is cut into two half blocks (two tasks each, two empty
// task slots): C3 cuts 40 of its 7630 blocks for 6 per CU.
constexpr int kXdBlocksPerCu = 6;
constexpr int64_t kLdsPerCu = 160 * 1024, kLdsGranule = 1024;

int64_t xd_target_entries(int dtype, const Tuning &t) {
  const int bpc = t.xd_blocks_per_cu > 0 ? t.xd_blocks_per_cu : kXdBlocksPerCu;
  const int64_t sv = (int64_t)dtype_size(dtype);
  // product staging of the chunk plan_launch picks for >= 12 nonzeros per
  // row (pick_u: U = 4 fp64, 16 fp32), 4 waves (CSR3 product buffers are
  // never bank-padded: spmv_device.cuh wave_lds<U, false>)
  const int64_t staging = 4 * 64 * (sv == 8 ? 4 : 16) * sv + 16;
  const int64_t per_block = (kLdsPerCu / bpc) / kLdsGranule * kLdsGranule;
  return std::max<int64_t>(0, (per_block - staging) / sv);
}

// Cuts the 4-task blocks of `tasks` whose dictionary exceeds `target`
// entries into two 2-task blocks padded with empty tasks.  Returns the
// number of blocks cut.  (Cutting the launch's last blocks as well, so its
// drain runs on workgroups of half the life, measured slower: C3 108.0 ->
// 110.7 / 112.2 / 115.8 us for the last 768 / 1536 / 3072 blocks, fp32 62.1
// -> 64.0 / 66.6 / 70.9; profiles/r03/ab_c3_tail_cuts_negative.jsonl.)
int64_t split_xd_blocks(std::vector<int32_t> &tasks, const std::vector<int32_t> &total,
                        int64_t target) {
  const int64_t nt = (int64_t)tasks.size() - 1, W = 4;
  int64_t cut = 0;
  std::vector<int32_t> out;
  out.reserve(tasks.size() + 64);
  for (int64_t b = 0; b * W < nt; ++b) {
    const int64_t t0 = b * W, t1 = std::min(nt, t0 + W);
    if (total[(size_t)b] > target && t1 - t0 > 2) {
      ++cut;
      const int32_t mid = tasks[(size_t)t0 + 2];
      out.push_back(tasks[(size_t)t0]);
      out.push_back(tasks[(size_t)t0 + 1]);
      out.push_back(mid);
      out.push_back(mid);  // two empty tasks
      for (int64_t t = t0 + 2; t < t1; ++t) out.push_back(tasks[(size_t)t]);
      for (int64_t t = t1 - t0 - 2; t < W; ++t) out.push_back(tasks[(size_t)t1]);
    } else {
      for (int64_t t = t0; t < t1; ++t) out.push_back(tasks[(size_t)t]);
    }
  }
  out.push_back(tasks[(size_t)nt]);
  if (cut) tasks.swap(out);
  return cut;
}

// plan_xdict over the workgroups of `kern`; CSR3 task tables are first cut
// for occupancy (split_xd_blocks), so the plan is the one the kernel runs.
// (The SSR plan's blocks are its super-super-rows: never cut.)
bool plan_xdict_for(const int32_t *rp, const int32_t *col, int kern, int64_t m,
                    std::vector<int32_t> &tasks, int W, int32_t long_t, int64_t cap, int dtype,
                    const Tuning &tune, bool fill, XdPlan &P, int64_t *cut) {
  *cut = 0;
  const bool cuts = kern == kCsr3 && W == 4 && tune.csr3_plan != HSPMV_CSR3_PLAN_SSR &&
                    tune.xd_blocks_per_cu >= 0;
  if (!plan_xdict(rp, col, xdict_blocks(kern, m, tasks, W), long_t, cap, fill && !cuts, P))
    return false;
  if (!cuts) return true;
  *cut = split_xd_blocks(tasks, P.total, xd_target_entries(dtype, tune));
  if (*cut == 0 && !fill) return true;
  return plan_xdict(rp, col, xdict_blocks(kern, m, tasks, W), long_t, cap, fill, P);
}

// Auto mode also leaves banded matrices to the x windows (have_xwin: the
// row kernel's window table qualified): on C4's shard the per-wave windows
// need no block barrier and were 7 % faster than the dictionaries
// (53.8 vs 57.9 us, profiles/r01_ab_xdict.jsonl).
int build_xdict(Shard &s, const int32_t *rp, const int32_t *col, int64_t m, int64_t n, int dtype,
                unsigned flags, bool have_xwin) {
  s.xd_shape = 0;
  const int mode = s.tune.x_dict > 0 ? 1 : (s.tune.x_dict < 0 ? 0 : -1);  // -1 auto, 0 off, 1 on when it fits
  if (mode == 0 || (flags & HSPMV_FLAG_NO_COL16) || m == 0) return HSPMV_OK;
  if (mode < 0 && have_xwin) return HSPMV_OK;
  const int kern = kernel_for_tables(s.A.n_ssr, !s.h_tasks.empty(), flags);
  if (kern != kStream && kern != kCsr3) return HSPMV_OK;
  const int W = xd_block_tasks(s.tune, s.A.task_waves);
  if (kern == kCsr3 && W != 4 && W != 8) return HSPMV_OK;  // the XD kernels run 4 or 8 waves
  if (kern == kStream && ((flags >> 29) & 0x7u) > 1) return HSPMV_OK;  // groups != 1
  const double sv = (double)dtype_size(dtype);
  const int64_t nnz = rp[m];
  const double footprint = (double)nnz * (sv + 4.0) + (double)m * (sv + 4.0) + (double)n * sv;
  if (mode < 0 && footprint <= kMallResident) return HSPMV_OK;
  const int32_t long_t = (flags & HSPMV_FLAG_NO_SPLIT) ? INT32_MAX : kLongRow;
  XdPlan P;
  // (cuts the task table only when the dictionaries are taken)
  std::vector<int32_t> tasks = s.h_tasks;
  if (!plan_xdict_for(rp, col, kern, m, tasks, W, long_t, xdict_cap_entries(dtype, s.tune), dtype,
                      s.tune, true, P, &s.xd_cut))
    return HSPMV_OK;
  if (mode < 0 && 2 * P.entries > P.in_kernel_nnz) return HSPMV_OK;  // too little reuse to pay
  s.h_tasks.swap(tasks);
  int rc;
  if ((rc = dev_alloc(&s.d_c16, 2 * (size_t)std::max<int64_t>(nnz, 1), &s.bytes))) return rc;
  if ((rc = dev_alloc(&s.d_xd_blk, 4 * P.blk.size(), &s.bytes))) return rc;
  if ((rc = dev_alloc(&s.d_xd_runs, 4 * P.rec.size(), &s.bytes))) return rc;
  if (nnz) HIP_TRY(hipMemcpy(s.d_c16, P.pos.data(), 2 * (size_t)nnz, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s.d_xd_blk, P.blk.data(), 4 * P.blk.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s.d_xd_runs, P.rec.data(), 4 * P.rec.size(), hipMemcpyHostToDevice));
  s.A.col16 = s.d_c16;
  s.A.cbase = nullptr;
  s.A.cplanes = nullptr;
  s.A.n_cplanes = 0;
  s.xd_shape = kern;
  if (kern == kCsr3) s.A.task_waves = W;
  s.xd_lds_bytes = (int32_t)((int64_t)P.tmax * (int64_t)sv);
  s.xd_entries = P.entries;
  s.xd_runs_n = (int64_t)P.rec.size() / 2;
  return HSPMV_OK;
}

}  // namespace hspmv

using namespace hspmv;

extern "C" {

int hspmv_xdict_plan_ex(const hspmv_csr *A, const hspmv_csr3_maps *maps, const hspmv_options *opt,
                        int64_t cap_entries, int64_t *n_blocks, int64_t *n_records, int32_t *blk,
                        int32_t *runs, uint16_t *pos) {
  clear_error();
  if (!n_blocks || !n_records) return set_error(HSPMV_E_INVALID, "NULL output");
  *n_blocks = 0;
  *n_records = 0;
  int rc;
  Tuning tune;
  if ((rc = tuning_from_options(opt, &tune))) return rc;
  const unsigned flags = opt ? opt->flags : 0u;
  if ((rc = validate_host_csr(A, true))) return rc;
  if ((rc = validate_host_maps(maps, A->m))) return rc;
  std::vector<int32_t> tasks;
  const bool csr3 = maps && maps->n_ssr > 0;
  int waves = 4;
  if (csr3) {
    const std::vector<int32_t> inner(maps->inner, maps->inner + maps->n_sr + 1);
    const std::vector<int32_t> outer(maps->outer, maps->outer + maps->n_ssr + 1);
    build_tasks(A->row_ptr, A->m, &inner, &outer, flags, tune, tasks, &waves);
  } else {
    build_tasks(A->row_ptr, A->m, nullptr, nullptr, flags, tune, tasks, &waves);
  }
  const int W = xd_block_tasks(tune, waves);
  const int kern = kernel_for_tables(csr3 ? maps->n_ssr : 0, !tasks.empty(), flags);
  if ((kern != kStream && kern != kCsr3) || A->m == 0 || (kern == kCsr3 && W != 4 && W != 8))
    return HSPMV_OK;
  if (cap_entries <= 0) cap_entries = xdict_cap_entries(A->dtype, tune);
  XdPlan P;
  const int32_t long_t = (flags & HSPMV_FLAG_NO_SPLIT) ? INT32_MAX : kLongRow;
  const bool fill = blk || runs || pos;
  int64_t cut = 0;
  if (!plan_xdict_for(A->row_ptr, A->col_idx, kern, A->m, tasks, W, long_t,
                      std::min<int64_t>(cap_entries, 65536), A->dtype, tune, fill, P, &cut))
    return HSPMV_OK;  // some block exceeds the cap: no dictionary (n_blocks = 0)
  *n_blocks = (int64_t)P.blk.size() - 1;
  *n_records = (int64_t)P.blk.back();
  if (blk) memcpy(blk, P.blk.data(), 4 * P.blk.size());
  if (runs) memcpy(runs, P.rec.data(), 4 * P.rec.size());
  if (pos && A->nnz) memcpy(pos, P.pos.data(), 2 * (size_t)A->nnz);
  return HSPMV_OK;
}

int hspmv_xdict_plan(const hspmv_csr *A, const hspmv_csr3_maps *maps, unsigned flags,
                     int64_t cap_entries, int64_t *n_blocks, int64_t *n_records, int32_t *blk,
                     int32_t *runs, uint16_t *pos) {
  hspmv_options o;
  memset(&o, 0, sizeof(o));
  o.struct_size = sizeof(o);
  o.flags = flags;
  return hspmv_xdict_plan_ex(A, maps, &o, cap_entries, n_blocks, n_records, blk, runs, pos);
}

}  // extern "C"

namespace hspmv {

}  // namespace hspmv
