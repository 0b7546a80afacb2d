// hspmv_shard.cpp -- one row-range shard: allocation, upload, plan finish, placement
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

// Tuning.contig (A/B, diagnostic builds): physically contiguous device
// allocations (hipDeviceMallocContiguous; plain hipMalloc when that fails).
// Set for the duration of one handle creation (creation is not re-entrant per
// thread).
thread_local bool t_contig = false;

int dev_alloc_bytes(void **p, size_t bytes, int64_t *acc) {
  *p = nullptr;
  if (bytes == 0) bytes = 16;
  hipError_t e = hipErrorMemoryAllocation;
  if (t_contig) {
    e = hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous);
    if (e != hipSuccess) (void)hipGetLastError();
  }
  if (e != hipSuccess) e = hipMalloc(p, bytes);
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
                  (void *)s.d_cs_part, (void *)s.d_cs_spart, (void *)s.d_cs_trace, (void *)s.d_cs_rexp,
                  (void *)s.d_cs_sexp, (void *)s.d_cs_xexp})
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
  if (s.long_fork) (void)hipEventDestroy(s.long_fork);
  if (s.long_join) (void)hipEventDestroy(s.long_join);
  if (s.long_stream) (void)hipStreamDestroy(s.long_stream);
  s = Shard();
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

// Mean SpMV time (us) of the shard's current arrays: 2 warm-up launches, then
// the best of 3 event-timed runs of 5 launches.  < 0 on a launch error.
static double time_shard(Shard &s, int dtype) {
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
static constexpr int kPlacementTrials = 0;

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

}  // namespace hspmv
