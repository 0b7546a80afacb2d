// hspmv_api.cpp -- device runtime behind the C ABI (include/hspmv.h):
// handles, uploads, launch planning, the reference timing protocol and the
// multi-GPU row-range partition with RCCL over xGMI.
//
// Replaces the CSRk_Graph device plumbing of the reference
// (cuda-spmv-csrk/hip/csrk.cu:92-113, 531-641, 722-870): device buffers are
// owned by a handle instead of process globals, every HIP/RCCL status is
// checked, and there is one stream per GPU instead of the default stream +
// hipDeviceSynchronize.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <cstddef>
#include <cmath>
#include <cstdlib>
#include <atomic>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>

#include "hspmv_common.h"
#include "hspmv_internal.h"

namespace hspmv {
namespace {

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess)                                                          \
      return set_error(HSPMV_E_HIP, "%s failed: %s (%s:%d)", #expr,                \
                       hipGetErrorString(_e), __FILE__, __LINE__);                 \
  } while (0)

// One row-range shard on one GPU.
struct Shard {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int64_t row0 = 0;  // first global row
  DevCSR A;          // device view (rows rebased to 0)
  LaunchPlan plan;
  double mean_rows_per_ssr = 0.0;
  // owned device memory
  int32_t *d_rp = nullptr, *d_ci = nullptr, *d_outer = nullptr, *d_inner = nullptr;
  uint16_t *d_c16 = nullptr;  // 16-bit column offsets (owned even for borrowed A)
  int32_t *d_cbase = nullptr;
  uint64_t *d_cplanes = nullptr;
  int32_t *d_xwin = nullptr;         // STREAM x windows {lo, w} per 64-row group
  int32_t *d_xd_blk = nullptr;       // block x dictionaries (build_xdict)
  int64_t xd_cut = 0;                // CSR3 dictionary blocks cut in two (split_xd_blocks)
  int32_t *d_xd_runs = nullptr;
  int32_t xd_lds_bytes = 0;
  int xd_shape = 0;                  // 0 none, kStream (256-row blocks), kCsr3 (4 packed tasks)
  int64_t xd_entries = 0;            // x entries staged per SpMV (all blocks)
  int64_t xd_runs_n = 0;             // run records incl. sentinels
  int32_t *d_slab_rp = nullptr;      // x slabs (build_xslabs): per-slab row pointers,
  int32_t *d_slab_col = nullptr;     // slab-major columns and values
  void *d_slab_val = nullptr;
  int32_t n_slabs = 0;
  // column-sorted row blocks (build_csort): owned tables, and the launch
  // description they form (copied into dp.cs when the planner picks kCsort)
  int32_t *d_cs_blk_c = nullptr, *d_cs_blk_r = nullptr, *d_cs_blk_v = nullptr,
          *d_cs_vslice = nullptr, *d_cs_cbase = nullptr, *d_cs_long_row = nullptr,
          *d_cs_long_cs = nullptr;
  uint32_t *d_cs_mask = nullptr;
  unsigned long long *d_cs_trace = nullptr;  // diagnostic builds: csort per-workgroup timestamps
  void *d_cs_ent = nullptr, *d_cs_val = nullptr;
  double *d_cs_part = nullptr, *d_cs_spart = nullptr;
  DevCsort csort;
  double csort_format_bytes = 0.0;   // bytes one csort SpMV moves
  int c16g_shape = 0;                // group-base columns built for kStream groups / kCsr3 tasks
  std::vector<int32_t> h_xwin;       // built at upload (host columns at hand)
  std::vector<int32_t> h_xwin_t;     // the same per packed CSR-3 task
  void *d_val = nullptr;
  void *d_x = nullptr;     // own x (n entries)
  void *d_y = nullptr;     // own y (m_shard entries) -- or a slice of d_yfull
  void *d_yfull = nullptr; // multi-GPU: padded all-gather buffer P*max_rows
  const void *x = nullptr; // x in use (own or bound)
  void *y = nullptr;       // y in use (own or bound)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  int64_t bytes = 0;
  int64_t x_entries = 0;   // distinct columns of this shard
  double c16_saved = 0.0;  // bytes per SpMV the 16-bit column offsets save
  // planner tables (owned): CSR-3 wave tasks and split-row chunks
  DevPlan dp;
  int32_t *d_task = nullptr, *d_long_row = nullptr, *d_long_cstart = nullptr,
          *d_chunk_k = nullptr;
  void *d_partials = nullptr;
  // host copies kept until the plan is built
  std::vector<int32_t> h_rp, h_outer, h_inner, h_tasks;
  // placement trials (place_shard): SpMV time of each array set, the kept one
  std::vector<double> place_us;
  int place_pick = 0;
  Tuning tune;  // the handle's planner choices (hspmv_options)
};

}  // namespace
}  // namespace hspmv

struct hspmv_handle {
  std::vector<hspmv::Shard> shards;
  int64_t m = 0, n = 0, nnz = 0;
  int dtype = HSPMV_F64;
  int64_t n_ssr = 0, n_sr = 0;
  unsigned flags = 0;
  bool x_set = false;
  bool borrowed = false;  // HSPMV_FLAG_DEVICE_PTRS: matrix arrays not owned
  int64_t max_rows = 0;   // multi-GPU padding for the y all-gather
  bool sharded = false;   // row-range partition (hspmv_create_sharded / num_gpus > 1)
  int64_t x_entries() const {
    int64_t t = 0;
    for (auto &s : shards) t += s.x_entries;
    return t;
  }
  std::vector<ncclComm_t> comms;
};

using namespace hspmv;

namespace {

// Planner options -> Tuning.  Fields past the caller's struct_size read as 0.
int tuning_from_options(const hspmv_options *o, Tuning *t) {
  *t = Tuning();
  if (!o) return HSPMV_OK;
  if (o->struct_size < offsetof(hspmv_options, csr3_plan))
    return set_error(HSPMV_E_INVALID, "hspmv_options.struct_size %u too small", o->struct_size);
  hspmv_options v;
  memset(&v, 0, sizeof(v));
  memcpy(&v, o, std::min<size_t>(o->struct_size, sizeof(v)));
  if (v.csr3_plan < 0 || v.csr3_plan > HSPMV_CSR3_PLAN_SSR)
    return set_error(HSPMV_E_INVALID, "csr3_plan %d unknown", v.csr3_plan);
  if ((v.csort_parts && v.csort_parts != 1 && v.csort_parts != 2 && v.csort_parts != 4) ||
      (v.csort_chunk_u && v.csort_chunk_u != 4 && v.csort_chunk_u != 8 && v.csort_chunk_u != 16) ||
      (v.stream_waves && v.stream_waves != 1 && v.stream_waves != 2 && v.stream_waves != 4) ||
      v.task_nnz < 0 || v.x_dict_cap < 0 || v.placement_trials < 0 || v.placement_trials > 8)
    return set_error(HSPMV_E_INVALID, "hspmv_options: value out of range");
  if (v.deterministic && (v.flags & 0xFu) == kCsort)
    return set_error(HSPMV_E_INVALID, "HSPMV_KERNEL_CSORT is not deterministic");
  t->csr3_plan = v.csr3_plan;
  t->task_nnz = v.task_nnz;
  t->x_windows = v.x_windows < 0 ? -1 : 0;
  t->x_dict = v.x_dict < 0 ? -1 : (v.x_dict > 0 ? 1 : 0);
  t->x_dict_cap = v.x_dict_cap;
  t->x_slabs = v.x_slabs < 0 ? -1 : v.x_slabs;
  t->col16_group = v.col16_group < 0 ? -1 : (v.col16_group > 0 ? 1 : 0);
  t->csort = v.csort < 0 ? -1 : (v.csort > 0 ? 1 : 0);
  t->csort_parts = v.csort_parts;
  t->csort_u = v.csort_chunk_u;
  t->stream_waves = v.stream_waves;
  t->deterministic = v.deterministic ? 1 : 0;
  t->placement_trials = v.placement_trials;
  return HSPMV_OK;
}

#ifdef HSPMV_ENV_KNOBS
// Diagnostic builds only (make diag-env): HSPMV_* environment variables
// override the options, for the A/B scripts under tools/.
void tuning_from_env(Tuning *t) {
  auto geti = [](const char *k, int *v) {
    if (const char *e = getenv(k)) *v = atoi(e);
  };
  if (const char *e = getenv("HSPMV_CSR3_PLAN"))
    t->csr3_plan = !strcmp(e, "ssr") ? HSPMV_CSR3_PLAN_SSR
                   : !strcmp(e, "packed") ? HSPMV_CSR3_PLAN_PACKED : HSPMV_CSR3_PLAN_ALIGNED;
  if (const char *e = getenv("HSPMV_TASK_FILL"))
    if (atoi(e) == 0) t->csr3_plan = HSPMV_CSR3_PLAN_PACKED;
  geti("HSPMV_TASK_NNZ", &t->task_nnz);
  if (const char *e = getenv("HSPMV_XWIN")) t->x_windows = atoi(e) == 0 ? -1 : 0;
  if (const char *e = getenv("HSPMV_XDICT")) t->x_dict = atoi(e) == 0 ? -1 : 1;
  geti("HSPMV_XDICT_CAP", &t->x_dict_cap);
  if (const char *e = getenv("HSPMV_XSLABS")) t->x_slabs = atoi(e) == 0 ? -1 : atoi(e);
  if (const char *e = getenv("HSPMV_XSLAB_BYTES")) t->xslab_bytes = atof(e);
  if (const char *e = getenv("HSPMV_COL16G")) t->col16_group = atoi(e) == 0 ? -1 : 1;
  if (const char *e = getenv("HSPMV_CSORT")) t->csort = atoi(e) == 0 ? -1 : 1;
  geti("HSPMV_CSORT_H", &t->csort_parts);
  geti("HSPMV_CSORT_U", &t->csort_u);
  geti("HSPMV_CSORT_NT", &t->csort_nt);
  geti("HSPMV_CSORT_PF", &t->csort_pf);
  geti("HSPMV_CSORT_BPC", &t->csort_blocks_per_cu);
  geti("HSPMV_CSORT_SLOT32", &t->csort_slot32);
  geti("HSPMV_CSORT_WIDE", &t->csort_wide);
  geti("HSPMV_CSORT_LDS", &t->csort_lds_cap);
  geti("HSPMV_CSORT_SEG", &t->csort_seg);
  geti("HSPMV_CSORT_SEG_EXTRA", &t->csort_seg_extra);
  geti("HSPMV_CSORT_TRACE", &t->csort_trace);
  geti("HSPMV_CSORT_LONG", &t->csort_long);
  geti("HSPMV_STREAM_W", &t->stream_waves);
  geti("HSPMV_PLACEMENT", &t->placement_trials);
  geti("HSPMV_CONTIG", &t->contig);
  geti("HSPMV_XD_WAVES", &t->xd_waves);
  geti("HSPMV_XD_BPC", &t->xd_blocks_per_cu);
  geti("HSPMV_PF", &t->pf);
  geti("HSPMV_YNT", &t->y_nt);
  geti("HSPMV_NT", &t->nt);
  geti("HSPMV_DYNLDS", &t->dyn_lds);
}
#else
void tuning_from_env(Tuning *) {}
#endif

// Tuning.contig (A/B, diagnostic builds): physically contiguous device
// allocations (hipDeviceMallocContiguous; plain hipMalloc when that fails).
// Set for the duration of one handle creation (creation is not re-entrant per
// thread).
thread_local bool t_contig = false;
bool contig_alloc() { return t_contig; }

template <typename T>
int dev_alloc(T **p, size_t bytes, int64_t *acc) {
  *p = nullptr;
  if (bytes == 0) bytes = 16;
  hipError_t e = hipErrorMemoryAllocation;
  if (contig_alloc()) {
    e = hipExtMallocWithFlags((void **)p, bytes, hipDeviceMallocContiguous);
    if (e != hipSuccess) (void)hipGetLastError();
  }
  if (e != hipSuccess) e = hipMalloc((void **)p, bytes);
  if (e != hipSuccess)
    return set_error(HSPMV_E_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  *acc += (int64_t)bytes;
  return HSPMV_OK;
}

void free_shard(Shard &s, bool borrowed) {
  (void)hipSetDevice(s.device);
  if (!borrowed) {
    (void)hipFree(s.d_rp);
    (void)hipFree(s.d_ci);
    (void)hipFree(s.d_val);
    (void)hipFree(s.d_outer);
    (void)hipFree(s.d_inner);
  }
  (void)hipFree(s.d_c16);
  (void)hipFree(s.d_cbase);
  (void)hipFree(s.d_cplanes);
  (void)hipFree(s.d_xwin);
  (void)hipFree(s.d_xd_blk);
  (void)hipFree(s.d_xd_runs);
  (void)hipFree(s.d_slab_rp);
  (void)hipFree(s.d_slab_col);
  (void)hipFree(s.d_slab_val);
  for (void *p : {(void *)s.d_cs_blk_c, (void *)s.d_cs_blk_r, (void *)s.d_cs_blk_v,
                  (void *)s.d_cs_vslice, (void *)s.d_cs_cbase, (void *)s.d_cs_long_row,
                  (void *)s.d_cs_long_cs, (void *)s.d_cs_mask, s.d_cs_ent, s.d_cs_val,
                  (void *)s.d_cs_part, (void *)s.d_cs_spart, (void *)s.d_cs_trace})
    (void)hipFree(p);
  (void)hipFree(s.d_task);
  (void)hipFree(s.d_long_row);
  (void)hipFree(s.d_long_cstart);
  (void)hipFree(s.d_chunk_k);
  (void)hipFree(s.d_partials);
  (void)hipFree(s.d_x);
  if (!s.d_yfull) (void)hipFree(s.d_y);
  (void)hipFree(s.d_yfull);
  if (s.ev0) (void)hipEventDestroy(s.ev0);
  if (s.ev1) (void)hipEventDestroy(s.ev1);
  if (s.own_stream && s.stream) (void)hipStreamDestroy(s.stream);
  s = Shard();
}

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
constexpr double kMallResident = 192.0 * 1024 * 1024;  // same bound as the XCD order

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

// x windows of the STREAM kernel's 64-row groups: {lo, w} with w = the
// group's column span when it is at most kXWin entries (its x slice is then
// staged in LDS and gathered from there), else 0.  Kept only when at least
// half of the groups qualify (banded matrices); Tuning.x_windows = -1 disables.
// CSR-3 task packing (the default CSR-3 plan): the super-rows of the inner
// map, in order, are packed into wave tasks of at most one 64-row group
// (the lanes of a wave's ordered sums); a super-row longer than 64 rows is
// cut at 64-row steps.  Four consecutive tasks form a workgroup, so a
// super-super-row spans as many waves as its rows need instead of a fixed W
// per launch (handCoarsen's super-super-rows vary ~10x in rows).
// Tuning.csr3_plan = HSPMV_CSR3_PLAN_SSR selects the workgroup-per-super-
// super-row plan.
bool csr3_packed(const Tuning &t) { return t.csr3_plan != HSPMV_CSR3_PLAN_SSR; }

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

// The wave tasks of a shard (empty: STREAM's fixed 64-row groups, or the
// workgroup-per-super-super-row CSR-3 plan).  CSR-3: the packed super-rows.
// CSR under the auto (or CSR3) kernel: when at least a quarter of the
// in-kernel nonzeros sit in 64-row groups over the budget, the 64-row groups
// with the heavy ones cut -- the CSR3 kernel then runs them (a CSR-2 with
// one-row super-rows).  Both are capped at the budget.
void build_tasks(const int32_t *rp, int64_t m, const std::vector<int32_t> *inner, unsigned flags,
                 const Tuning &tune, std::vector<int32_t> &ts) {
  ts.clear();
  if (!csr3_packed(tune)) return;
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
    return have_tasks ? kCsr3 : -1;  // workgroup-per-SSR plan: no dictionaries
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

std::vector<int32_t> xdict_blocks(int kern, int64_t m, const std::vector<int32_t> &tasks,
                                  const Tuning &tune) {
  std::vector<int32_t> bs;
  if (kern == kStream) {
    for (int64_t r = 0; r < m; r += 256) bs.push_back((int32_t)r);
    bs.push_back((int32_t)m);
  } else {
    const int64_t nt = (int64_t)tasks.size() - 1;
    for (int64_t t = 0; t < nt; t += xd_task_waves(tune)) bs.push_back(tasks[(size_t)t]);
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
  // row (pick_u: U = 4 fp64, 16 fp32), 4 waves
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
bool plan_xdict_for(const int32_t *rp, const int32_t *col, int kern, int64_t m,
                    std::vector<int32_t> &tasks, int32_t long_t, int64_t cap, int dtype,
                    const Tuning &tune, bool fill, XdPlan &P, int64_t *cut) {
  *cut = 0;
  const bool cuts = kern == kCsr3 && xd_task_waves(tune) == 4 && tune.xd_blocks_per_cu >= 0;
  if (!plan_xdict(rp, col, xdict_blocks(kern, m, tasks, tune), long_t, cap, fill && !cuts, P))
    return false;
  if (!cuts) return true;
  *cut = split_xd_blocks(tasks, P.total, xd_target_entries(dtype, tune));
  if (*cut == 0 && !fill) return true;
  return plan_xdict(rp, col, xdict_blocks(kern, m, tasks, tune), long_t, cap, fill, P);
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
  if (kern == kStream && ((flags >> 29) & 0x7u) > 1) return HSPMV_OK;  // groups != 1
  const double sv = (double)dtype_size(dtype);
  const int64_t nnz = rp[m];
  const double footprint = (double)nnz * (sv + 4.0) + (double)m * (sv + 4.0) + (double)n * sv;
  if (mode < 0 && footprint <= kMallResident) return HSPMV_OK;
  const int32_t long_t = (flags & HSPMV_FLAG_NO_SPLIT) ? INT32_MAX : kLongRow;
  XdPlan P;
  // (cuts the task table only when the dictionaries are taken)
  std::vector<int32_t> tasks = s.h_tasks;
  if (!plan_xdict_for(rp, col, kern, m, tasks, long_t, xdict_cap_entries(dtype, s.tune), dtype,
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
  if (kern == kCsr3) s.A.task_waves = xd_task_waves(s.tune);
  s.xd_lds_bytes = (int32_t)((int64_t)P.tmax * (int64_t)sv);
  s.xd_entries = P.entries;
  s.xd_runs_n = (int64_t)P.rec.size() / 2;
  return HSPMV_OK;
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
// Auto: HBM-resident matrices with irregular gathers and x beyond an XCD's
// L2 (the x-slab rule, which it replaces: C5 264 -> ~110 us), unless the
// handle asks for deterministic sums (the slots add in atomic order);
// HSPMV_KERNEL_CSORT forces it, Tuning.csort = -1 turns auto off,
// Tuning.csort_parts = 1/2/4 sets the column parts, csort_u = 4/8/16 the
// chunk.  The row blocks are capped by the device's LDS per workgroup.
constexpr int32_t kCsortSlice = 2048;
// a chunk whose instructions would serialise more than this many same-slot
// lanes in all is stored slot-sorted (segmented)
constexpr int64_t kCsortSegExtra = 128;
constexpr int64_t kCsortSegHeavy = 8;  // entries of one row in a chunk that make it a run

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
  lds_max = std::min(lds_max, kCsortMaxLds);
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
  auto part_of = [&](int64_t c) { return (int)((c * H) / n); };  // c in part floor(c*H/n)
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
  // Row blocks PER COLUMN PART.  Part h is a fixed slice of x,
  // [ceil(n h / H), ceil(n (h + 1) / H)), and workgroup j works on part
  // j % H: under round-robin dispatch (workgroup j on XCD j % 8;
  // tools/xcd_map_probe.hip records it per box) every XCD sweeps one slice,
  // which its 4 MiB L2 keeps for all its CUs.  Each part has its OWN row
  // partition, balanced on the nonzeros that fall in that part and capped in
  // rows (the LDS slots), so the parts' workgroups carry equal work whatever
  // the ordering: with one row partition for all parts an RCM-ordered
  // power-law matrix put ~90 % of a block's entries in one part (322 us vs
  // 108 us on the same matrix unordered), and quantile splits per block, which
  // balance the work but let every XCD sweep all of x, still took 205 us.
  const int64_t nb0 = std::max<int64_t>(1, (int64_t)cus * bpc / H);
  const int64_t reserve = n_slices / nb0 + 2;
  const int64_t row_cap = max_slots - 1 - reserve;
  if (row_cap < 64) return HSPMV_OK;  // too many slices for the LDS: not this path
  std::vector<int32_t> cnt((size_t)(H * m), 0);  // [h][r]: row r's in-kernel nonzeros in part h
  {
    const int ntc = (int)std::max<int64_t>(1, std::min<int64_t>(16, m / 65536));
    std::vector<std::thread> th;
    for (int t = 0; t < ntc; ++t)
      th.emplace_back([&, t]() {
        for (int64_t r = m * t / ntc; r < m * (t + 1) / ntc; ++r) {
          if (rp[r + 1] - rp[r] > long_t) continue;
          for (int32_t k = rp[r]; k < rp[r + 1]; ++k) ++cnt[(size_t)(part_of(col[k]) * m + r)];
        }
      });
    for (auto &x : th) x.join();
  }
  // Greedy cuts at `target` nonzeros or row_cap rows; the target is the
  // smallest that yields at most nb0 blocks (one block more would run a
  // second round of workgroups on one CU and double the launch).
  auto cut = [&](int h, int64_t target, std::vector<int32_t> *out) -> int64_t {
    const int32_t *c = cnt.data() + (size_t)h * (size_t)m;
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
  std::vector<std::vector<int32_t>> brh((size_t)H);
  int64_t NB = 0;
  for (int h = 0; h < H; ++h) {
    int64_t tot_h = 0;
    for (int64_t r = 0; r < m; ++r) tot_h += cnt[(size_t)(h * m + r)];
    int64_t lo = std::max<int64_t>(1, (tot_h + nb0 - 1) / nb0), hi = std::max<int64_t>(lo, tot_h + 1);
    if (cut(h, lo, nullptr) > nb0) {
      if (cut(h, hi, nullptr) > nb0) lo = hi;  // the row cap alone needs more blocks
      while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (cut(h, mid, nullptr) <= nb0) hi = mid; else lo = mid + 1;
      }
    }
    cut(h, lo, &brh[(size_t)h]);
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
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t]() {
        for (int64_t b = t; b < G; b += nt) {
          auto &E = ents[(size_t)b];
          const uint32_t dummy = (uint32_t)(nslots[(size_t)b] - 1);
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
              }
            }
            cbase[(size_t)ch] = (int32_t)(c0 | (seg ? 0x80000000u : 0u));
            for (int64_t q = 0; q < C; ++q) {
              const int64_t o = ch * C + at(q, dtype == HSPMV_F32 ? 2 : 4);
              const int64_t ov = ch * C + at(q, 2);
              uint32_t ix = dummy << 16;  // padding: 0 * x[base] into the dummy slot
              const void *vp = nullptr;
              if (i + q < j) {
                const CsEnt &e = src[q];
                ix = (e.slot << 16) | (e.col - c0);
                vp = (const char *)val + sv * (size_t)e.k;
              }
              if (dtype == HSPMV_F32) {
                uint32_t vb = 0;
                if (vp) memcpy(&vb, vp, 4);
                rec[(size_t)o] = ((uint64_t)vb << 32) | ix;
              } else {
                idx[(size_t)o] = ix;
                if (vp) memcpy(&val64[(size_t)ov], vp, 8);
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
  if (!direct) {  // partial sums in the slot type
    if ((rc = dev_alloc(&s.d_cs_part, slot_bytes * (size_t)H * (size_t)m, &s.bytes))) return rc;
    if ((rc = dev_alloc(&s.d_cs_spart, slot_bytes * (size_t)std::max<int64_t>(n_slices, 1), &s.bytes)))
      return rc;
  }
  if (!lrow.empty()) {
    if ((rc = up(&s.d_cs_mask, mask)) || (rc = up(&s.d_cs_long_row, lrow)) || (rc = up(&s.d_cs_long_cs, lcs)))
      return rc;
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
  c.wide = wide;
  c.m = m;
  c.lds_bytes = (int32_t)(slot_bytes * max_slots_used);
  c.blk_c = s.d_cs_blk_c;
  c.blk_r = s.d_cs_blk_r;
  c.blk_v = s.d_cs_blk_v;
  c.row_blocks = (int32_t)NB;
  if (tn.csort_trace == 1 && (rc = dev_alloc(&s.d_cs_trace, 24 * (size_t)G, &s.bytes))) return rc;
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
  s.csort_format_bytes = (double)tot * (double)(4 + sv) + 4.0 * (double)tot_chunks + xb +
                         (direct ? 0.0 : 2.0 * (double)slot_bytes * ((double)H * (double)m + (double)n_slices)) +
                         (double)sv * (double)m;
  s.A.has_csort = true;
  return HSPMV_OK;
}


// Host-side tables that need the columns (built at upload, while they are
// at hand): the CSR-3 packed tasks, the block x dictionaries, and (without
// dictionaries) the 16-bit column offsets and the x windows of both row
// kernels.
int build_row_tables(Shard &s, const int32_t *rp, const int32_t *col, const void *val, int64_t m,
                     int64_t n, int dtype, unsigned flags) {
  build_tasks(rp, m, s.A.n_ssr > 0 ? &s.h_inner : nullptr, flags, s.tune, s.h_tasks);
  s.h_xwin.clear();
  s.h_xwin_t.clear();
  int rc;
  {
    const unsigned kf = flags & 0xFu;
    const int cm = s.tune.csort;  // -1 off, 0 auto, 1 whenever it can be built
    const double sv = (double)dtype_size(dtype);
    const double footprint = (double)rp[m] * (sv + 4.0) + (double)m * (sv + 4.0) + (double)n * sv;
    bool want = kf == kCsort || cm == 1;
    if (!want && kf == kAuto && cm == 0 && !s.tune.deterministic && s.tune.x_slabs == 0 &&
        footprint > kMallResident && (double)n * sv > 4.0 * 1024 * 1024)
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

// Uploads rows [r0, r1) of A (and the matching slice of the maps) to shard s.
int upload_shard(Shard &s, const hspmv_csr *A, const hspmv_csr3_maps *mp, int64_t r0, int64_t r1,
                 int64_t ssr0, int64_t ssr1, int64_t y_rows_alloc, unsigned flags) {
  const size_t sv = dtype_size(A->dtype);
  const int64_t m = r1 - r0;
  const int64_t k0 = A->row_ptr[r0], k1 = A->row_ptr[r1];
  const int64_t nnz = k1 - k0;
  HIP_TRY(hipSetDevice(s.device));
  s.row0 = r0;
  int rc;
  if ((rc = dev_alloc(&s.d_rp, 4 * (size_t)(m + 1), &s.bytes))) return rc;
  if ((rc = dev_alloc(&s.d_ci, 4 * (size_t)nnz, &s.bytes))) return rc;
  if ((rc = dev_alloc(&s.d_val, sv * (size_t)nnz, &s.bytes))) return rc;
  if ((rc = dev_alloc(&s.d_x, sv * (size_t)A->n, &s.bytes))) return rc;
  if (y_rows_alloc > 0) {
    if ((rc = dev_alloc(&s.d_y, sv * (size_t)y_rows_alloc, &s.bytes))) return rc;
  }
  std::vector<int32_t> &rp = s.h_rp;
  rp.resize((size_t)(m + 1));
  for (int64_t i = 0; i <= m; ++i) rp[i] = (int32_t)(A->row_ptr[r0 + i] - k0);
  HIP_TRY(hipMemcpy(s.d_rp, rp.data(), 4 * (size_t)(m + 1), hipMemcpyHostToDevice));
  s.x_entries = count_distinct_cols(A->col_idx + k0, nnz, A->n);
  if (nnz) {
    HIP_TRY(hipMemcpy(s.d_ci, A->col_idx + k0, 4 * (size_t)nnz, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s.d_val, (const char *)A->val + sv * k0, sv * (size_t)nnz,
                      hipMemcpyHostToDevice));
  }
  s.A.m = (int32_t)m;
  s.A.n = A->n;
  s.A.nnz = nnz;
  s.A.row_ptr = s.d_rp;
  s.A.col_idx = s.d_ci;
  s.A.val = s.d_val;
  if (mp && mp->n_ssr > 0) {
    const int64_t nssr = ssr1 - ssr0;
    const int64_t sr0 = mp->outer[ssr0], sr1 = mp->outer[ssr1];
    const int64_t nsr = sr1 - sr0;
    std::vector<int32_t> &o = s.h_outer, &in = s.h_inner;
    o.resize((size_t)(nssr + 1));
    in.resize((size_t)(nsr + 1));
    for (int64_t i = 0; i <= nssr; ++i) o[i] = (int32_t)(mp->outer[ssr0 + i] - sr0);
    for (int64_t i = 0; i <= nsr; ++i) in[i] = (int32_t)(mp->inner[sr0 + i] - r0);
    if ((rc = dev_alloc(&s.d_outer, 4 * (size_t)(nssr + 1), &s.bytes))) return rc;
    if ((rc = dev_alloc(&s.d_inner, 4 * (size_t)(nsr + 1), &s.bytes))) return rc;
    HIP_TRY(hipMemcpy(s.d_outer, o.data(), 4 * (size_t)(nssr + 1), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s.d_inner, in.data(), 4 * (size_t)(nsr + 1), hipMemcpyHostToDevice));
    s.A.n_ssr = (int32_t)nssr;
    s.A.n_sr = (int32_t)nsr;
    s.A.outer = s.d_outer;
    s.A.inner = s.d_inner;
    s.mean_rows_per_ssr = nssr ? (double)m / (double)nssr : 0.0;
  }
  return build_row_tables(s, rp.data(), A->col_idx + k0, (const char *)A->val + sv * k0, m, A->n,
                          A->dtype, flags);
}

// Host planner tables for one shard (needs s.h_rp, and s.h_outer/h_inner for
// CSR-3):
//  * split rows: rows longer than kLongRow, cut into kLongChunk pieces;
//  * CSR-3 wave tasks: each super-super-row's super-rows split into
//    waves_per_block contiguous ranges with ~equal nonzeros -- the first
//    super-row s with rp[inner[s]] >= k0 + (k1-k0)*w/W starts wave w.
int build_plan_tables(Shard &s, int dtype, unsigned flags) {
  const std::vector<int32_t> &rp = s.h_rp;
  const int64_t m = s.A.m;
  s.dp = DevPlan();
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
    if (!lrow.empty()) {
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
  } else if (s.plan.kernel == kCsr3) {
    const std::vector<int32_t> &o = s.h_outer, &in = s.h_inner;
    const int64_t nssr = s.A.n_ssr;
    const int W = s.plan.waves_per_block;
    std::vector<int32_t> ts((size_t)(nssr * W + 1));
    for (int64_t b = 0; b < nssr; ++b) {
      const int32_t s0 = o[b], s1 = o[b + 1];
      const int64_t k0 = rp[in[s0]], k1 = rp[in[s1]];
      // wave w starts at the first super-row reaching w/W of the nonzeros,
      // but strictly after wave w-1's start while super-rows remain: two
      // waves never share a start (an empty task beside a doubled one was
      // 15 % of the tasks on a 64-row grouping: 144 -> 129 us there).
      // Row-granular cuts capped at 64 rows per wave measured 7-30 % slower
      // on C3's groupings (long tails where an SSR exceeds W*64 rows);
      // profiles/r01_ab_csr3_tasks.jsonl.
      int32_t sr = s0, prev = s0 - 1;
      for (int w = 0; w < W; ++w) {
        const int64_t target = k0 + (k1 - k0) * w / W;
        while (sr < s1 && rp[in[sr]] < target) ++sr;
        int32_t st = w == 0 ? s0 : sr;
        if (st <= prev) st = prev + 1;
        const int32_t latest = s1 - (W - w);  // leave one super-row per later wave
        if (st > latest) st = std::max(prev + 1, latest);
        if (st > s1) st = s1;
        ts[(size_t)(b * W + w)] = in[st];
        prev = st;
        sr = std::max(sr, st);
      }
    }
    ts[(size_t)(nssr * W)] = (int32_t)m;
    int rc;
    if ((rc = dev_alloc(&s.d_task, 4 * ts.size(), &s.bytes))) return rc;
    HIP_TRY(hipMemcpy(s.d_task, ts.data(), 4 * ts.size(), hipMemcpyHostToDevice));
    s.dp.task_start = s.d_task;
    s.dp.n_tasks = (int32_t)(nssr * W);
  }
  return HSPMV_OK;
}

int finish_shard(Shard &s, int dtype, unsigned flags, void *stream) {
  HIP_TRY(hipSetDevice(s.device));
  if (stream) {
    s.stream = (hipStream_t)stream;
    s.own_stream = false;
  } else {
    HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    s.own_stream = true;
  }
  HIP_TRY(hipEventCreate(&s.ev0));
  HIP_TRY(hipEventCreate(&s.ev1));
  // CSR-3 block size from the mean rows per super-super-row (sizing on the
  // 90th percentile doubled C3's waves for a 7-12 % loss, r01_ab_csr3_tasks)
  const double ssr_rows = s.mean_rows_per_ssr;
  s.plan = plan_launch(s.A, dtype, flags, ssr_rows,
                       s.h_tasks.empty() ? 0 : (int64_t)s.h_tasks.size() - 1, s.tune);
  int rc = build_plan_tables(s, dtype, flags);
  if (rc) return rc;
  s.x = s.d_x;
  s.y = s.d_y;
  std::vector<int32_t>().swap(s.h_rp);
  std::vector<int32_t>().swap(s.h_outer);
  std::vector<int32_t>().swap(s.h_inner);
  return HSPMV_OK;
}

int check_handle(hspmv_handle *h) {
  if (!h || h->shards.empty()) return set_error(HSPMV_E_INVALID, "invalid handle");
  return HSPMV_OK;
}

// Mean SpMV time (us) of the shard's current arrays: 2 warm-up launches, then
// the best of 3 event-timed runs of 5 launches.  < 0 on a launch error.
double time_shard(Shard &s, int dtype) {
  for (int i = 0; i < 2; ++i)
    if (launch_spmv(s.A, s.dp, dtype, s.plan, s.x, s.y, s.stream) != hipSuccess) return -1.0;
  double best = 1e30;
  for (int r = 0; r < 3; ++r) {
    if (hipEventRecord(s.ev0, s.stream) != hipSuccess) return -1.0;
    for (int i = 0; i < 5; ++i)
      if (launch_spmv(s.A, s.dp, dtype, s.plan, s.x, s.y, s.stream) != hipSuccess) return -1.0;
    float ms = 0.0f;
    if (hipEventRecord(s.ev1, s.stream) != hipSuccess || hipEventSynchronize(s.ev1) != hipSuccess ||
        hipEventElapsedTime(&ms, s.ev0, s.ev1) != hipSuccess)
      return -1.0;
    best = std::min(best, 1000.0 * (double)ms / 5.0);
  }
  return best;
}

// Placement trials.  Where a handle's streamed arrays land in HBM moves the
// HBM-bound row kernels by up to ~10 %: identical C3 handles created one
// after another in one process ran 101.0, 105.4 and 110.8 us, each stable
// over its own rounds (profiles/r02ad_ab_placement.jsonl).  So the shard's
// streamed arrays -- row pointers, the column stream the kernel reads (16-bit
// positions/offsets or 32-bit columns), values, x and y -- are copied into
// trials-1 fresh allocations in turn (all held until the end, so each lands
// elsewhere), every set is timed over a few SpMVs, and the fastest is kept;
// the others are freed.  The kernel, its tables and every bit of y are the
// same for all sets.  Single-GPU handles with owned arrays whose row kernel
// (STREAM / CSR3) streams from HBM; Tuning.placement_trials = K sets the number of sets
// (0 or 1 = off); memory for the extra sets must be free, else fewer are
// tried.  Off by default: with 4 sets per handle no faster placement turned
// up on C3 (the first set won 8 of 8 handles; the trial sets ran 111-117 us
// against 109-111) and C4's picks did not carry over to the steady state
// (49.5 vs 49.4 us without trials; profiles/r02ae_ab_placement_trials.jsonl),
// so what made some handles fast in r02ad is not the placement of these
// arrays alone.
constexpr int kPlacementTrials = 0;

int place_shard(Shard &s, int64_t n, int dtype) {
  int trials = s.tune.placement_trials > 0 ? std::min(8, s.tune.placement_trials) : kPlacementTrials;
  if (trials <= 1 || (s.plan.kernel != kStream && s.plan.kernel != kCsr3) || s.A.m == 0) return HSPMV_OK;
  const size_t sv = dtype_size(dtype);
  const int64_t m = s.A.m, nnz = s.A.nnz;
  if ((double)nnz * (double)(sv + 4) + (double)m * (double)(sv + 4) + (double)n * (double)sv <=
      kMallResident)
    return HSPMV_OK;  // served from the Infinity Cache: placement does not matter
  struct Arr { void **slot; size_t bytes; };
  std::vector<Arr> arrs = {{(void **)&s.d_rp, 4 * (size_t)(m + 1)},
                           {(void **)&s.d_val, sv * (size_t)nnz},
                           {(void **)&s.d_x, sv * (size_t)n},
                           {(void **)&s.d_y, sv * (size_t)m}};
  if (s.A.col16)
    arrs.push_back({(void **)&s.d_c16, 2 * (size_t)nnz});
  else
    arrs.push_back({(void **)&s.d_ci, 4 * (size_t)nnz});
  size_t set_bytes = 0;
  for (auto &a : arrs) set_bytes += a.bytes;
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  const size_t margin = (size_t)1 << 30;
  const int fit = free_b > margin ? (int)std::min<size_t>(8, (free_b - margin) / set_bytes) : 0;
  trials = std::min(trials, 1 + fit);
  if (trials <= 1) return HSPMV_OK;
  auto point = [&]() {
    s.A.row_ptr = s.d_rp;
    s.A.col_idx = s.d_ci;
    s.A.val = s.d_val;
    if (s.A.col16) s.A.col16 = s.d_c16;
    s.x = s.d_x;
    s.y = s.d_y;
  };
  HIP_TRY(hipMemsetAsync(s.d_x, 0, sv * (size_t)n, s.stream));
  std::vector<std::vector<void *>> sets(1);
  for (auto &a : arrs) sets[0].push_back(*a.slot);
  s.place_us.assign(1, time_shard(s, dtype));
  if (s.place_us[0] < 0) return set_error(HSPMV_E_HIP, "placement trial: launch failed");
  int rc = HSPMV_OK;
  for (int k = 1; k < trials && rc == HSPMV_OK; ++k) {
    std::vector<void *> set;
    for (auto &a : arrs) {
      void *p = nullptr;
      if (hipMalloc(&p, a.bytes) != hipSuccess) break;
      set.push_back(p);
      if (hipMemcpyAsync(p, *a.slot, a.bytes, hipMemcpyDeviceToDevice, s.stream) != hipSuccess) {
        rc = set_error(HSPMV_E_HIP, "placement trial: copy failed");
        break;
      }
    }
    if (rc != HSPMV_OK || set.size() != arrs.size()) {  // out of memory or a failed copy: stop
      (void)hipStreamSynchronize(s.stream);
      for (void *p : set) (void)hipFree(p);
      (void)hipGetLastError();
      break;
    }
    for (size_t i = 0; i < arrs.size(); ++i) *arrs[i].slot = set[i];
    point();
    const double t = time_shard(s, dtype);
    sets.push_back(set);
    s.place_us.push_back(t);
    if (t < 0) rc = set_error(HSPMV_E_HIP, "placement trial: launch failed");
  }
  HIP_TRY(hipStreamSynchronize(s.stream));
  int pick = 0;
  for (int k = 1; k < (int)sets.size(); ++k)
    if (s.place_us[(size_t)k] >= 0 && s.place_us[(size_t)k] < s.place_us[(size_t)pick]) pick = k;
  for (int k = 0; k < (int)sets.size(); ++k)
    if (k != pick)
      for (void *p : sets[(size_t)k]) (void)hipFree(p);
  for (size_t i = 0; i < arrs.size(); ++i) *arrs[i].slot = sets[(size_t)pick][i];
  point();
  s.place_pick = pick;
  return rc;
}

}  // namespace

extern "C" {

int hspmv_device_count(int *count) {
  clear_error();
  if (!count) return set_error(HSPMV_E_INVALID, "NULL argument");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    return set_error(HSPMV_E_NODEV, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *count = c;
  return HSPMV_OK;
}

}  // extern "C"

namespace {

// Sets the allocation mode of one handle creation (Tuning.contig) and
// restores it on every return path.
struct ContigScope {
  explicit ContigScope(const Tuning &t) { t_contig = t.contig == 1; }
  ~ContigScope() { t_contig = false; }
};

int create_single(hspmv_handle **hp, const hspmv_csr *A, const hspmv_csr3_maps *maps, int device,
                  void *stream, unsigned flags, const Tuning &tune) {
  ContigScope contig(tune);
  const bool devptrs = (flags & HSPMV_FLAG_DEVICE_PTRS) != 0;
  if (!A) return set_error(HSPMV_E_INVALID, "matrix is NULL");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
    return set_error(HSPMV_E_NODEV, "no HIP device available");
  if (device < 0 || device >= ndev)
    return set_error(HSPMV_E_NODEV, "device %d out of range (have %d)", device, ndev);
  std::unique_ptr<hspmv_handle> h(new hspmv_handle());
  h->m = A->m; h->n = A->n; h->nnz = A->nnz; h->dtype = A->dtype; h->flags = flags;
  h->shards.resize(1);
  Shard &s = h->shards[0];
  s.device = device;
  s.tune = tune;
  int rc;
  if (!devptrs) {
    if ((rc = validate_host_csr(A, true))) return rc;
    if ((rc = validate_host_maps(maps, A->m))) return rc;
    if (maps && maps->n_ssr > 0) { h->n_ssr = maps->n_ssr; h->n_sr = maps->n_sr; }
    if ((rc = upload_shard(s, A, maps, 0, A->m, 0, maps ? maps->n_ssr : 0, A->m, flags))) {
      free_shard(s, false);
      return rc;
    }
  } else {
    // Borrowed device arrays: validate what the kernels index with (row_ptr
    // and the maps) on the host before the first launch.
    h->borrowed = true;
    if (A->m < 0 || A->n < 0 || A->nnz < 0 || A->m >= INT32_MAX || A->nnz >= INT32_MAX ||
        (A->dtype != HSPMV_F32 && A->dtype != HSPMV_F64) || !A->row_ptr)
      return set_error(HSPMV_E_INVALID, "bad device matrix description");
    HIP_TRY(hipSetDevice(device));
    std::vector<int32_t> &rp = s.h_rp;
    rp.resize((size_t)(A->m + 1));
    HIP_TRY(hipMemcpy(rp.data(), A->row_ptr, 4 * (size_t)(A->m + 1), hipMemcpyDeviceToHost));
    hspmv_csr view = *A;  // device col/val are only null-checked, never read here
    view.row_ptr = rp.data();
    if ((rc = validate_host_csr(&view, false)) != HSPMV_OK) return rc;
    s.A.m = (int32_t)A->m; s.A.n = A->n; s.A.nnz = A->nnz;
    s.A.row_ptr = A->row_ptr; s.A.col_idx = A->col_idx; s.A.val = A->val;
    std::vector<int32_t> cols((size_t)A->nnz);  // host copy until the row tables are built
    {
      if (A->nnz)
        HIP_TRY(hipMemcpy(cols.data(), A->col_idx, 4 * (size_t)A->nnz, hipMemcpyDeviceToHost));
      for (int32_t c : cols)
        if (c < 0 || c >= A->n) return set_error(HSPMV_E_INVALID, "device col_idx %d out of [0, %lld)", c, (long long)A->n);
      s.x_entries = count_distinct_cols(cols.data(), A->nnz, A->n);
    }
    if (maps && maps->n_ssr > 0) {
      std::vector<int32_t> &o = s.h_outer, &in = s.h_inner;
      o.resize((size_t)(maps->n_ssr + 1));
      in.resize((size_t)(maps->n_sr + 1));
      HIP_TRY(hipMemcpy(o.data(), maps->outer, 4 * o.size(), hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(in.data(), maps->inner, 4 * in.size(), hipMemcpyDeviceToHost));
      hspmv_csr3_maps mv = {maps->n_ssr, maps->n_sr, o.data(), in.data()};
      if ((rc = validate_host_maps(&mv, A->m))) return rc;
      s.A.n_ssr = (int32_t)maps->n_ssr; s.A.n_sr = (int32_t)maps->n_sr;
      s.A.outer = maps->outer; s.A.inner = maps->inner;
      s.mean_rows_per_ssr = (double)A->m / (double)maps->n_ssr;
      h->n_ssr = maps->n_ssr; h->n_sr = maps->n_sr;
    }
    // the values come back to the host too: the x slabs copy them slab-major
    std::vector<char> vals(dtype_size(A->dtype) * (size_t)A->nnz);
    if (A->nnz) HIP_TRY(hipMemcpy(vals.data(), A->val, vals.size(), hipMemcpyDeviceToHost));
    // from here on the shard owns device memory: every error path frees it
    if ((rc = build_row_tables(s, rp.data(), cols.data(), vals.data(), A->m, A->n, A->dtype, flags))) {
      free_shard(s, true);
      return rc;
    }
    std::vector<char>().swap(vals);
    std::vector<int32_t>().swap(cols);
    const size_t sv = dtype_size(A->dtype);
    if ((rc = dev_alloc(&s.d_x, sv * (size_t)A->n, &s.bytes)) ||
        (rc = dev_alloc(&s.d_y, sv * (size_t)A->m, &s.bytes))) {
      free_shard(s, true);
      return rc;
    }
  }
  if ((rc = finish_shard(s, A->dtype, flags, stream))) {
    free_shard(s, h->borrowed);
    return rc;
  }
  if (!devptrs && (rc = place_shard(s, A->n, A->dtype))) {
    free_shard(s, h->borrowed);
    return rc;
  }
  *hp = h.release();
  return HSPMV_OK;
}

// The row-range partition over the devices devs[0..P) (one shard each; a
// device may appear more than once).  Distinct devices exchange x and y with
// RCCL (one communicator per shard, ncclCommInitAll); a list that repeats a
// device exchanges by device-to-device copies instead (RCCL allows one rank
// per device), which is how the partition, the padded y all-gather and the
// unpadding are exercised on a one-GPU box.
int create_sharded(hspmv_handle **hp, const hspmv_csr *A, const hspmv_csr3_maps *maps,
                   const std::vector<int> &devs, unsigned flags, const Tuning &tune) {
  ContigScope contig(tune);
  const int num_gpus = (int)devs.size();
  int rc;
  if ((rc = validate_host_csr(A, true))) return rc;
  if ((rc = validate_host_maps(maps, A->m))) return rc;
  const bool csr3 = maps && maps->n_ssr > 0;
  std::unique_ptr<hspmv_handle> h(new hspmv_handle());
  h->m = A->m; h->n = A->n; h->nnz = A->nnz; h->dtype = A->dtype; h->flags = flags;
  if (csr3) { h->n_ssr = maps->n_ssr; h->n_sr = maps->n_sr; }
  std::vector<int64_t> splits((size_t)num_gpus + 1);
  if ((rc = hspmv_partition_rows(A->m, A->row_ptr, csr3 ? maps : nullptr, num_gpus, splits.data())))
    return rc;
  // super-super-row index of each split (CSR-3 partitions on SSR boundaries)
  std::vector<int64_t> ssr_split((size_t)num_gpus + 1, 0);
  if (csr3) {
    int64_t s = 0;
    for (int p = 0; p <= num_gpus; ++p) {
      while (s < maps->n_ssr && maps->inner[maps->outer[s]] < splits[p]) ++s;
      ssr_split[p] = s;
    }
    ssr_split[num_gpus] = maps->n_ssr;
  }
  int64_t max_rows = 0;
  for (int p = 0; p < num_gpus; ++p) max_rows = std::max(max_rows, splits[p + 1] - splits[p]);
  h->max_rows = max_rows;
  h->shards.resize((size_t)num_gpus);
  const size_t sv = dtype_size(A->dtype);
  auto cleanup = [&]() {
    for (auto &s : h->shards) free_shard(s, false);
  };
  for (int p = 0; p < num_gpus; ++p) {
    Shard &s = h->shards[p];
    s.device = devs[(size_t)p];
    s.tune = tune;
    if ((rc = upload_shard(s, A, maps, splits[p], splits[p + 1], ssr_split[p], ssr_split[p + 1], 0,
                           flags))) {
      cleanup();
      return rc;
    }
    // y lives in this GPU's slot of a padded [P][max_rows] all-gather buffer
    if ((rc = dev_alloc(&s.d_yfull, sv * (size_t)(max_rows * num_gpus), &s.bytes))) {
      cleanup();
      return rc;
    }
    s.d_y = (char *)s.d_yfull + sv * (size_t)(max_rows * p);
    if ((rc = finish_shard(s, A->dtype, flags, nullptr))) {
      cleanup();
      return rc;
    }
  }
  std::vector<int> sorted(devs);
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  if (distinct) {
    h->comms.resize((size_t)num_gpus);
    std::vector<int> dl(devs);
    ncclResult_t r = ncclCommInitAll(h->comms.data(), num_gpus, dl.data());
    if (r != ncclSuccess) {
      cleanup();
      h->comms.clear();
      return set_error(HSPMV_E_RCCL, "ncclCommInitAll: %s", ncclGetErrorString(r));
    }
  }
  h->sharded = true;
  *hp = h.release();
  return HSPMV_OK;
}

int check_devices(const int *devices, int n, int *ndev_out) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
    return set_error(HSPMV_E_NODEV, "no HIP device available");
  *ndev_out = ndev;
  for (int p = 0; devices && p < n; ++p)
    if (devices[p] < 0 || devices[p] >= ndev)
      return set_error(HSPMV_E_NODEV, "device %d out of range (have %d)", devices[p], ndev);
  return HSPMV_OK;
}

Tuning default_tuning() {
  Tuning t;
  tuning_from_env(&t);  // no-op outside diagnostic builds
  return t;
}

}  // namespace

extern "C" {

int hspmv_create_on_device(hspmv_handle **hp, const hspmv_csr *A, const hspmv_csr3_maps *maps,
                           int device, void *stream, unsigned flags) {
  clear_error();
  if (!hp) return set_error(HSPMV_E_INVALID, "NULL handle pointer");
  *hp = nullptr;
  return create_single(hp, A, maps, device, stream, flags, default_tuning());
}

int hspmv_create_ex(hspmv_handle **hp, const hspmv_csr *A, const hspmv_csr3_maps *maps,
                    const hspmv_options *opt) {
  clear_error();
  if (!hp) return set_error(HSPMV_E_INVALID, "NULL handle pointer");
  *hp = nullptr;
  Tuning t;
  int rc;
  if ((rc = tuning_from_options(opt, &t))) return rc;
  tuning_from_env(&t);  // diagnostic builds only
  const unsigned flags = opt ? opt->flags : 0u;
  if (opt && opt->devices) {
    if (flags & HSPMV_FLAG_DEVICE_PTRS)
      return set_error(HSPMV_E_INVALID, "device pointers need a single-device handle");
    if (opt->n_devices < 1) return set_error(HSPMV_E_INVALID, "need n_devices >= 1");
    int ndev = 0;
    if ((rc = check_devices(opt->devices, opt->n_devices, &ndev))) return rc;
    return create_sharded(hp, A, maps, std::vector<int>(opt->devices, opt->devices + opt->n_devices),
                          flags, t);
  }
  return create_single(hp, A, maps, opt ? opt->device : 0, opt ? opt->stream : nullptr, flags, t);
}

int hspmv_create(hspmv_handle **hp, const hspmv_csr *A, const hspmv_csr3_maps *maps, int num_gpus,
                 unsigned flags) {
  clear_error();
  if (!hp) return set_error(HSPMV_E_INVALID, "NULL handle pointer");
  *hp = nullptr;
  if (flags & HSPMV_FLAG_DEVICE_PTRS)
    return set_error(HSPMV_E_INVALID, "device pointers need hspmv_create_on_device");
  int ndev = 0, rc;
  if ((rc = check_devices(nullptr, 0, &ndev))) return rc;
  if (num_gpus <= 0) num_gpus = ndev;
  if (num_gpus > ndev)
    return set_error(HSPMV_E_NODEV, "%d GPUs requested, %d visible", num_gpus, ndev);
  if (num_gpus == 1) return create_single(hp, A, maps, 0, nullptr, flags, default_tuning());
  std::vector<int> devs((size_t)num_gpus);
  for (int p = 0; p < num_gpus; ++p) devs[(size_t)p] = p;
  return create_sharded(hp, A, maps, devs, flags, default_tuning());
}

int hspmv_create_sharded(hspmv_handle **hp, const hspmv_csr *A, const hspmv_csr3_maps *maps,
                         const int *devices, int n_shards, unsigned flags) {
  clear_error();
  if (!hp) return set_error(HSPMV_E_INVALID, "NULL handle pointer");
  *hp = nullptr;
  if (flags & HSPMV_FLAG_DEVICE_PTRS)
    return set_error(HSPMV_E_INVALID, "device pointers need hspmv_create_on_device");
  if (!devices || n_shards < 1) return set_error(HSPMV_E_INVALID, "need n_shards >= 1 devices");
  int ndev = 0, rc;
  if ((rc = check_devices(devices, n_shards, &ndev))) return rc;
  return create_sharded(hp, A, maps, std::vector<int>(devices, devices + n_shards), flags,
                        default_tuning());
}

// Shards that share a device (no communicators): the same exchanges as
// device-to-device copies on each destination shard's stream, after the
// source shard's stream has reached them.
static int copy_exchange(hspmv_handle *h, bool x_bcast) {
  const size_t sv = dtype_size(h->dtype);
  const size_t P = h->shards.size();
  std::vector<hipEvent_t> done(P, nullptr);
  int rc = HSPMV_OK;
  for (size_t p = 0; p < P && rc == HSPMV_OK; ++p) {
    Shard &s = h->shards[p];
    if (hipSetDevice(s.device) != hipSuccess ||
        hipEventCreateWithFlags(&done[p], hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(done[p], s.stream) != hipSuccess)
      rc = set_error(HSPMV_E_HIP, "exchange: event setup on GPU %d failed", s.device);
  }
  for (size_t q = 0; q < P && rc == HSPMV_OK; ++q) {
    Shard &d = h->shards[q];
    if (hipSetDevice(d.device) != hipSuccess) {
      rc = set_error(HSPMV_E_HIP, "hipSetDevice(%d) failed", d.device);
      break;
    }
    for (size_t p = 0; p < P && rc == HSPMV_OK; ++p) {
      const Shard &src = h->shards[x_bcast ? 0 : p];
      if (x_bcast && q == 0) break;
      if (hipStreamWaitEvent(d.stream, done[x_bcast ? 0 : p], 0) != hipSuccess) {
        rc = set_error(HSPMV_E_HIP, "exchange: stream wait failed");
        break;
      }
      hipError_t e;
      if (x_bcast) {
        e = hipMemcpyPeerAsync(d.d_x, d.device, src.d_x, src.device, sv * (size_t)h->n, d.stream);
      } else {
        char *dst = (char *)d.d_yfull + sv * (size_t)(h->max_rows * (int64_t)p);
        e = dst == src.d_y ? hipSuccess
                           : hipMemcpyPeerAsync(dst, d.device, src.d_y, src.device,
                                                sv * (size_t)src.A.m, d.stream);
      }
      if (e != hipSuccess) rc = set_error(HSPMV_E_HIP, "exchange copy failed: %s", hipGetErrorString(e));
      if (x_bcast) break;
    }
  }
  for (size_t p = 0; p < P; ++p)
    if (done[p]) (void)hipEventDestroy(done[p]);
  return rc;
}

}  // extern "C"

// One RCCL group over every shard's communicator: op(p) enqueues shard p's
// part.  The group is always closed (ncclGroupEnd) before returning, also
// when an enqueue fails -- an open group would swallow the calling thread's
// next RCCL calls.
template <typename Op>
static int rccl_group(hspmv_handle *h, const char *what, Op op) {
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return set_error(HSPMV_E_RCCL, "ncclGroupStart: %s", ncclGetErrorString(r));
  ncclResult_t first = ncclSuccess;
  for (size_t p = 0; p < h->shards.size() && first == ncclSuccess; ++p) first = op(p);
  r = ncclGroupEnd();
  if (first != ncclSuccess) return set_error(HSPMV_E_RCCL, "%s: %s", what, ncclGetErrorString(first));
  if (r != ncclSuccess) return set_error(HSPMV_E_RCCL, "%s (ncclGroupEnd): %s", what, ncclGetErrorString(r));
  return HSPMV_OK;
}

extern "C" {

static int bcast_x(hspmv_handle *h) {
  if (!h->sharded) return HSPMV_OK;
  if (h->comms.empty()) return copy_exchange(h, true);
  const ncclDataType_t dt = h->dtype == HSPMV_F64 ? ncclFloat64 : ncclFloat32;
  return rccl_group(h, "ncclBroadcast(x)", [&](size_t p) {
    Shard &s = h->shards[p];
    return ncclBroadcast(h->shards[0].d_x, s.d_x, (size_t)h->n, dt, 0, h->comms[p], s.stream);
  });
}

static int gather_y(hspmv_handle *h) {
  if (!h->sharded) return HSPMV_OK;
  if (h->comms.empty()) return copy_exchange(h, false);
  const ncclDataType_t dt = h->dtype == HSPMV_F64 ? ncclFloat64 : ncclFloat32;
  return rccl_group(h, "ncclAllGather(y)", [&](size_t p) {
    Shard &s = h->shards[p];
    return ncclAllGather(s.d_y, s.d_yfull, (size_t)h->max_rows, dt, h->comms[p], s.stream);
  });
}

int hspmv_set_x(hspmv_handle *h, const void *x_host) {
  clear_error();
  int rc;
  if ((rc = check_handle(h))) return rc;
  if (!x_host && h->n > 0) return set_error(HSPMV_E_INVALID, "x is NULL");
  const size_t bytes = dtype_size(h->dtype) * (size_t)h->n;
  Shard &s0 = h->shards[0];
  HIP_TRY(hipSetDevice(s0.device));
  if (bytes) {
    HIP_TRY(hipMemcpyAsync(s0.d_x, x_host, bytes, hipMemcpyHostToDevice, s0.stream));
    HIP_TRY(hipStreamSynchronize(s0.stream));
  }
  if ((rc = bcast_x(h))) return rc;
  for (auto &s : h->shards) {
    HIP_TRY(hipSetDevice(s.device));
    HIP_TRY(hipStreamSynchronize(s.stream));
    s.x = s.d_x;
  }
  h->x_set = true;
  return HSPMV_OK;
}

int hspmv_bind_x_device(hspmv_handle *h, const void *x_dev) {
  clear_error();
  int rc;
  if ((rc = check_handle(h))) return rc;
  if (h->sharded) return set_error(HSPMV_E_STATE, "bind needs a single-device handle");
  h->shards[0].x = x_dev ? x_dev : h->shards[0].d_x;
  h->x_set = x_dev != nullptr || h->x_set;
  return HSPMV_OK;
}

int hspmv_bind_y_device(hspmv_handle *h, void *y_dev) {
  clear_error();
  int rc;
  if ((rc = check_handle(h))) return rc;
  if (h->sharded) return set_error(HSPMV_E_STATE, "bind needs a single-device handle");
  h->shards[0].y = y_dev ? y_dev : h->shards[0].d_y;
  return HSPMV_OK;
}

void *hspmv_x_device(hspmv_handle *h, int gpu) {
  if (!h || gpu < 0 || gpu >= (int)h->shards.size()) return nullptr;
  return (void *)h->shards[gpu].x;
}

void *hspmv_y_device(hspmv_handle *h, int gpu) {
  if (!h || gpu < 0 || gpu >= (int)h->shards.size()) return nullptr;
  return h->shards[gpu].y;
}

int hspmv_spmv(hspmv_handle *h) {
  int rc;
  if ((rc = check_handle(h))) return rc;
  if (!h->x_set) return set_error(HSPMV_E_STATE, "x not set (hspmv_set_x / hspmv_bind_x_device)");
  for (auto &s : h->shards) {
    HIP_TRY(hipSetDevice(s.device));
    hipError_t e = launch_spmv(s.A, s.dp, h->dtype, s.plan, s.x, s.y, s.stream);
    if (e != hipSuccess)
      return set_error(HSPMV_E_HIP, "SpMV launch on GPU %d failed: %s", s.device, hipGetErrorString(e));
  }
  return HSPMV_OK;
}

int hspmv_synchronize(hspmv_handle *h) {
  clear_error();
  int rc;
  if ((rc = check_handle(h))) return rc;
  for (auto &s : h->shards) {
    HIP_TRY(hipSetDevice(s.device));
    HIP_TRY(hipStreamSynchronize(s.stream));
  }
  return HSPMV_OK;
}

int hspmv_run(hspmv_handle *h, int warmup, int iters, hspmv_timing *out) {
  clear_error();
  int rc;
  if ((rc = check_handle(h))) return rc;
  if (!out || iters < 1 || warmup < 0) return set_error(HSPMV_E_INVALID, "bad arguments");
  for (int i = 0; i < warmup; ++i) {
    if ((rc = hspmv_spmv(h))) return rc;
    if ((rc = hspmv_synchronize(h))) return rc;
  }
  double tmin = 1e30, tmax = 0, tsum = 0, wmin = 1e30, wmax = 0, wsum = 0;
  for (int i = 0; i < iters; ++i) {
    auto tic = std::chrono::steady_clock::now();
    for (auto &s : h->shards) {
      HIP_TRY(hipSetDevice(s.device));
      HIP_TRY(hipEventRecord(s.ev0, s.stream));
      hipError_t e = launch_spmv(s.A, s.dp, h->dtype, s.plan, s.x, s.y, s.stream);
      if (e != hipSuccess)
        return set_error(HSPMV_E_HIP, "SpMV launch failed: %s", hipGetErrorString(e));
      HIP_TRY(hipEventRecord(s.ev1, s.stream));
    }
    double dev = 0.0;
    for (auto &s : h->shards) {
      HIP_TRY(hipSetDevice(s.device));
      HIP_TRY(hipEventSynchronize(s.ev1));
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, s.ev0, s.ev1));
      dev = std::max(dev, (double)ms * 1e-3);
    }
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - tic).count();
    tmin = std::min(tmin, dev); tmax = std::max(tmax, dev); tsum += dev;
    wmin = std::min(wmin, wall); wmax = std::max(wmax, wall); wsum += wall;
  }
  memset(out, 0, sizeof(*out));
  out->t_min = tmin; out->t_max = tmax; out->t_avg = tsum / iters;
  out->wall_min = wmin; out->wall_max = wmax; out->wall_avg = wsum / iters;
  out->gflops = tmin > 0 ? 2.0 * (double)h->nnz / tmin * 1e-9 : 0.0;
  out->gbps_alg = tmin > 0 ? hspmv_alg_bytes(h->m, h->x_entries(), h->nnz, h->dtype, h->n_ssr, h->n_sr) / tmin * 1e-9 : 0.0;
  out->iters = iters;
  out->num_gpus = (int32_t)h->shards.size();
  return HSPMV_OK;
}

int hspmv_get_y(hspmv_handle *h, void *y_host) {
  clear_error();
  int rc;
  if ((rc = check_handle(h))) return rc;
  if (!y_host && h->m > 0) return set_error(HSPMV_E_INVALID, "y is NULL");
  const size_t sv = dtype_size(h->dtype);
  if (!h->sharded) {
    Shard &s = h->shards[0];
    HIP_TRY(hipSetDevice(s.device));
    if (h->m) HIP_TRY(hipMemcpyAsync(y_host, s.y, sv * (size_t)h->m, hipMemcpyDeviceToHost, s.stream));
    HIP_TRY(hipStreamSynchronize(s.stream));
    return HSPMV_OK;
  }
  // RCCL all-gather of the padded shards, then unpad GPU 0's copy.
  if ((rc = gather_y(h))) return rc;
  if ((rc = hspmv_synchronize(h))) return rc;
  Shard &s0 = h->shards[0];
  HIP_TRY(hipSetDevice(s0.device));
  std::vector<char> full(sv * (size_t)(h->max_rows * (int64_t)h->shards.size()));
  HIP_TRY(hipMemcpy(full.data(), s0.d_yfull, full.size(), hipMemcpyDeviceToHost));
  for (size_t p = 0; p < h->shards.size(); ++p) {
    const Shard &s = h->shards[p];
    memcpy((char *)y_host + sv * (size_t)s.row0, full.data() + sv * (size_t)(h->max_rows * (int64_t)p),
           sv * (size_t)s.A.m);
  }
  return HSPMV_OK;
}

int hspmv_exchange(hspmv_handle *h, double *bcast_s, double *gather_s) {
  clear_error();
  int rc;
  if ((rc = check_handle(h))) return rc;
  if (bcast_s) {
    if ((rc = hspmv_synchronize(h))) return rc;
    auto tic = std::chrono::steady_clock::now();
    if ((rc = bcast_x(h))) return rc;
    if ((rc = hspmv_synchronize(h))) return rc;
    *bcast_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tic).count();
  }
  if (gather_s) {
    if ((rc = hspmv_synchronize(h))) return rc;
    auto tic = std::chrono::steady_clock::now();
    if ((rc = gather_y(h))) return rc;
    if ((rc = hspmv_synchronize(h))) return rc;
    *gather_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tic).count();
  }
  return HSPMV_OK;
}

int hspmv_get_info(hspmv_handle *h, hspmv_info *out) {
  clear_error();
  int rc;
  if ((rc = check_handle(h))) return rc;
  if (!out) return set_error(HSPMV_E_INVALID, "NULL output");
  memset(out, 0, sizeof(*out));
  const Shard &s = h->shards[0];
  out->kernel = s.plan.kernel;
  out->lanes = s.plan.lanes;
  out->waves_per_block = s.plan.waves_per_block;
  out->num_gpus = (int32_t)h->shards.size();
  out->blocks = s.plan.blocks;
  out->x_entries = h->x_entries();
  out->alg_bytes = hspmv_alg_bytes(h->m, out->x_entries, h->nnz, h->dtype, h->n_ssr, h->n_sr);
  out->flops = 2.0 * (double)h->nnz;
  for (auto &sh : h->shards) out->device_bytes += sh.bytes;
  out->chunk_u = s.plan.u;
  out->n_split_rows = s.dp.n_long;
  out->xcd_remap = s.plan.xcd_chunk;
  out->groups_per_wave = s.plan.kernel == kStream ? s.plan.groups : 1;
  out->format_bytes = out->alg_bytes;
  for (auto &sh : h->shards) out->format_bytes -= sh.c16_saved;
  out->col16 = s.A.col16 ? 1 + s.A.n_cplanes : 0;
  out->wave_tasks = s.plan.kernel == kCsr3 ? s.dp.n_tasks : 0;
  out->x_windows = s.dp.xwin ? 1 : 0;
  out->x_dict = s.dp.xd_blk ? 1 : 0;
  out->x_slabs = s.dp.n_slabs;
  out->col16_group = (s.A.col16 && s.A.c16_mode == 2) ? 1 : 0;
  out->csort_parts = s.plan.kernel == kCsort ? s.dp.cs.H : 0;
  out->n_split_rows = s.plan.kernel == kCsort ? s.dp.cs.n_long : out->n_split_rows;
  for (auto &sh : h->shards) out->x_dict_entries += sh.dp.xd_blk ? sh.xd_entries : 0;
  out->placement_trials = (int32_t)s.place_us.size();
  out->placement_pick = s.place_pick;
  for (size_t k = 0; k < s.place_us.size() && k < 8; ++k) out->placement_us[k] = s.place_us[k];
  out->deterministic = 1;
  for (auto &sh : h->shards) out->deterministic &= sh.plan.kernel == kCsort ? 0 : 1;
  out->csr3_plan = s.plan.kernel != kCsr3 ? 0
                   : s.h_tasks.empty() ? HSPMV_CSR3_PLAN_SSR
                   : csr3_fill(s.tune) ? HSPMV_CSR3_PLAN_ALIGNED : HSPMV_CSR3_PLAN_PACKED;
  out->csort_slot_bytes = s.plan.kernel == kCsort ? (s.dp.cs.slot32 ? 4 : 8) : 0;
  out->csort_row_blocks = s.plan.kernel == kCsort ? s.dp.cs.row_blocks : 0;
  return HSPMV_OK;
}

#ifdef HSPMV_ENV_KNOBS
// Diagnostic builds only (not in hspmv.h): the last csort launch's
// per-workgroup {start, end, XCC_ID | HW_ID << 32} (s_memrealtime ticks),
// when the handle was created with HSPMV_CSORT_TRACE=1.  Returns the
// workgroup count (0: no trace).
int hspmv_diag_csort_trace(hspmv_handle *h, unsigned long long *out, int max_wg) {
  if (!h || h->shards.empty()) return 0;
  const Shard &s = h->shards[0];
  if (s.plan.kernel != kCsort || !s.dp.cs.trace) return 0;
  const int n = std::min(max_wg, s.dp.cs.n_wg);
  if (hipSetDevice(s.device) != hipSuccess || hipStreamSynchronize(s.stream) != hipSuccess ||
      hipMemcpy(out, s.dp.cs.trace, 24 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return n;
}
#endif

int hspmv_get_info_sized(hspmv_handle *h, hspmv_info *out, uint32_t out_size) {
  clear_error();
  if (!out) return set_error(HSPMV_E_INVALID, "NULL output");
  hspmv_info full;
  int rc = hspmv_get_info(h, &full);
  if (rc) return rc;
  memcpy(out, &full, std::min<size_t>(out_size, sizeof(full)));
  return HSPMV_OK;
}

int hspmv_xdict_plan(const hspmv_csr *A, const hspmv_csr3_maps *maps, const hspmv_options *opt,
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
  if (csr3) {
    const std::vector<int32_t> inner(maps->inner, maps->inner + maps->n_sr + 1);
    build_tasks(A->row_ptr, A->m, &inner, flags, tune, tasks);
  } else {
    build_tasks(A->row_ptr, A->m, nullptr, flags, tune, tasks);
  }
  const int kern = kernel_for_tables(csr3 ? maps->n_ssr : 0, !tasks.empty(), flags);
  if ((kern != kStream && kern != kCsr3) || A->m == 0) return HSPMV_OK;
  if (cap_entries <= 0) cap_entries = xdict_cap_entries(A->dtype, tune);
  XdPlan P;
  const int32_t long_t = (flags & HSPMV_FLAG_NO_SPLIT) ? INT32_MAX : kLongRow;
  const bool fill = blk || runs || pos;
  int64_t cut = 0;
  if (!plan_xdict_for(A->row_ptr, A->col_idx, kern, A->m, tasks, long_t,
                      std::min<int64_t>(cap_entries, 65536), A->dtype, tune, fill, P, &cut))
    return HSPMV_OK;  // some block exceeds the cap: no dictionary (n_blocks = 0)
  *n_blocks = (int64_t)P.blk.size() - 1;
  *n_records = (int64_t)P.blk.back();
  if (blk) memcpy(blk, P.blk.data(), 4 * P.blk.size());
  if (runs) memcpy(runs, P.rec.data(), 4 * P.rec.size());
  if (pos && A->nnz) memcpy(pos, P.pos.data(), 2 * (size_t)A->nnz);
  return HSPMV_OK;
}

void hspmv_destroy(hspmv_handle *h) {
  if (!h) return;
  for (auto &s : h->shards) {
    (void)hipSetDevice(s.device);
    if (s.stream) (void)hipStreamSynchronize(s.stream);
  }
  for (auto c : h->comms) (void)ncclCommDestroy(c);
  for (auto &s : h->shards) free_shard(s, h->borrowed);
  delete h;
}

}  // extern "C"
