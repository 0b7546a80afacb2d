// hspmv_runtime.h -- the host runtime's internal state and the functions its
// units share (not part of the C ABI).  The runtime is split by concern:
//   hspmv_options.cpp      hspmv_options -> Tuning (+ diagnostic env knobs)
//   hspmv_shard.cpp        device allocation, upload, launch-plan finish,
//                          placement trials of one row-range shard
//   hspmv_tables.cpp       host planner tables: 16-bit columns, wave tasks,
//                          x windows, x slabs, split rows, CSR-3 SSR tasks
//   hspmv_xdict.cpp        block x dictionaries (+ hspmv_xdict_plan)
//   hspmv_csort_build.cpp  column-sorted row blocks (csort.hip's tables)
//   hspmv_multi.cpp        the row-range partition over devices, RCCL
//   hspmv_api.cpp          the C ABI entry points
//
// Replaces the CSRk_Graph device plumbing of the reference
// (cuda-spmv-csrk/hip/csrk.cu:92-113, 531-641, 722-870): device buffers are
// owned by a handle instead of process globals, every HIP/RCCL status is
// checked, and there is one stream per GPU instead of the default stream +
// hipDeviceSynchronize.
#pragma once
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <vector>

#include "hspmv_common.h"
#include "hspmv_internal.h"

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess)                                                          \
      return set_error(HSPMV_E_HIP, "%s failed: %s (%s:%d)", #expr,                \
                       hipGetErrorString(_e), __FILE__, __LINE__);                 \
  } while (0)

namespace hspmv {

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
  int16_t *d_cs_rexp = nullptr, *d_cs_sexp = nullptr;  // reproducible csort: value scales
  int32_t *d_cs_xexp = nullptr;                        // reproducible csort: x exponent pre-pass
  DevCsort csort;
  double csort_format_bytes = 0.0;   // bytes one csort SpMV moves
  int64_t csort_chunks = 0, csort_seg_chunks = 0;  // chunks, and those stored slot-sorted
  std::vector<int64_t> csort_wg_stats;  // diagnostic builds: 8 cost terms per workgroup
  int64_t csort_part_begin[4] = {0, 0, 0, 0};  // first column of each column part
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
  hipStream_t long_stream = nullptr;  // serial order: the long-row kernel's stream
  hipEvent_t long_fork = nullptr, long_join = nullptr;
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
  double heavy_frac = -1.0;  // x-slab handles with CSR3 tasks: nonzeros in heavy 64-row groups (slab_kernel_rule)
  Tuning tune;  // the handle's planner choices (hspmv_options)
};

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
  int rccl_version = 0;   // ncclGetVersion of the RCCL this process resolved
};

namespace hspmv {

// A matrix whose bytes stay under this is served from the 256 MiB Infinity
// Cache across back-to-back SpMVs (the planner's "resident" test).
constexpr double kMallResident = 192.0 * 1024 * 1024;

// ---- hspmv_options.cpp
int tuning_from_options(const hspmv_options *o, Tuning *t);
void tuning_from_env(Tuning *t);
Tuning default_tuning();
int check_deterministic(unsigned flags, const Tuning &t);

// ---- hspmv_shard.cpp
extern thread_local bool t_contig;
// Sets the allocation mode of one handle creation (Tuning.contig) and
// restores it on every return path.
struct ContigScope {
  explicit ContigScope(const Tuning &t) { t_contig = t.contig == 1; }
  ~ContigScope() { t_contig = false; }
};

int dev_alloc_bytes(void **p, size_t bytes, int64_t *acc);
template <typename T>
inline int dev_alloc(T **p, size_t bytes, int64_t *acc) {
  return dev_alloc_bytes((void **)p, bytes, acc);
}
void free_shard(Shard &s, bool borrowed);
int upload_shard(Shard &s, const hspmv_csr *A, const hspmv_csr3_maps *mp, int64_t r0, int64_t r1,
                 int64_t ssr0, int64_t ssr1, int64_t y_rows_alloc, unsigned flags);
int finish_shard(Shard &s, int dtype, unsigned flags, void *stream);
int place_shard(Shard &s, int64_t n, int dtype);

// ---- hspmv_tables.cpp
int64_t count_distinct_cols(const int32_t *col, int64_t nnz, int64_t n);
bool csr3_packed(const Tuning &t);
bool csr3_fill(const Tuning &t);
void build_tasks(const int32_t *rp, int64_t m, const std::vector<int32_t> *inner,
                 const std::vector<int32_t> *outer, unsigned flags, const Tuning &tune,
                 std::vector<int32_t> &ts, int *waves);
bool irregular_gathers(const int32_t *rp, const int32_t *col, int64_t m, double sv);
int build_row_tables(Shard &s, const int32_t *rp, const int32_t *col, const void *val, int64_t m,
                     int64_t n, int dtype, unsigned flags);
int build_plan_tables(Shard &s, int dtype, unsigned flags);

// ---- hspmv_xdict.cpp
// Which row kernel the planner will pick for a shard with n_ssr
// super-super-rows and (CSR-3) wave tasks.
int kernel_for_tables(int64_t n_ssr, bool have_tasks, unsigned flags);
int build_xdict(Shard &s, const int32_t *rp, const int32_t *col, int64_t m, int64_t n, int dtype,
                unsigned flags, bool have_xwin);

// ---- hspmv_csort_build.cpp
int build_csort(Shard &s, const int32_t *rp, const int32_t *col, const void *val, int64_t m,
                int64_t n, int dtype, unsigned flags);

// ---- hspmv_multi.cpp
int create_sharded(hspmv_handle **hp, const hspmv_csr *A, const hspmv_csr3_maps *maps,
                   const std::vector<int> &devs, unsigned flags, const Tuning &tune);
int bcast_x(hspmv_handle *h);
int gather_y(hspmv_handle *h);

}  // namespace hspmv
