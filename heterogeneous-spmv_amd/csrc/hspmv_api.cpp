// hspmv_api.cpp -- the C ABI entry points (include/hspmv.h): handle
// creation, x/y binding, the SpMV launch, the reference timing protocol,
// y gathering and the handle report.  The runtime behind them is in the
// other hspmv_*.cpp units (hspmv_runtime.h).
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <memory>
#include <vector>

#include "hspmv_runtime.h"

using namespace hspmv;

namespace {

int check_handle(hspmv_handle *h) {
  if (!h || h->shards.empty()) return set_error(HSPMV_E_INVALID, "invalid handle");
  return HSPMV_OK;
}

int create_single(hspmv_handle **hp, const hspmv_csr *A, const hspmv_csr3_maps *maps, int device,
                  void *stream, unsigned flags, const Tuning &tune) {
  ContigScope contig(tune);
  if (int rc0 = check_deterministic(flags, tune)) return rc0;
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
  (void)ncclGetVersion(&h->rccl_version);
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

}  // namespace

extern "C" {

int hspmv_rccl_version(int *version) {
  clear_error();
  if (!version) return set_error(HSPMV_E_INVALID, "NULL argument");
  *version = 0;
  ncclResult_t r = ncclGetVersion(version);
  if (r != ncclSuccess) return set_error(HSPMV_E_RCCL, "ncclGetVersion: %s", ncclGetErrorString(r));
  return HSPMV_OK;
}

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

}  // extern "C"

// The full report (this header's hspmv_info).
static int fill_info(hspmv_handle *h, hspmv_info *out) {
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
  for (auto &sh : h->shards) out->deterministic &= (sh.plan.kernel == kCsort && !sh.dp.cs.fixed) ? 0 : 1;
  // the maps-driven plans need maps; a CSR matrix whose heavy 64-row groups
  // sent it to the CSR3 kernel runs build_tasks' row groups
  out->csr3_plan = s.plan.kernel != kCsr3 ? 0
                   : s.A.n_ssr == 0 ? HSPMV_CSR3_PLAN_ROW_GROUPS
                   : s.tune.csr3_plan == HSPMV_CSR3_PLAN_SSR ? HSPMV_CSR3_PLAN_SSR
                   : csr3_fill(s.tune) ? HSPMV_CSR3_PLAN_ALIGNED : HSPMV_CSR3_PLAN_PACKED;
  out->csort_slot_bytes = s.plan.kernel == kCsort ? (s.dp.cs.slot32 ? 4 : 8) : 0;
  out->csort_row_blocks = s.plan.kernel == kCsort ? s.dp.cs.row_blocks : 0;
  out->rccl_version = h->rccl_version;
  out->slab_kernel_rule = s.heavy_frac < 0 ? 0 : (s.A.slab_stream ? 2 : 1);
  out->heavy_group_frac = s.heavy_frac < 0 ? 0.0 : s.heavy_frac;
  out->lds_pad = s.plan.lds_pad ? 1 : 0;
  out->csort_fixed_point = s.plan.kernel == kCsort && s.dp.cs.fixed ? 1 : 0;
  out->serial_order = 1;
  for (auto &sh : h->shards) out->serial_order &= sh.dp.serial_max == INT32_MAX ? 1 : 0;
  if (s.plan.kernel == kCsort)
    for (int hh = 0; hh < 4; ++hh) out->csort_part_begin[hh] = s.csort_part_begin[hh];
  for (auto &sh : h->shards)
    if (sh.plan.kernel == kCsort) {
      out->csort_chunks += sh.csort_chunks;
      out->csort_seg_chunks += sh.csort_seg_chunks;
    }
  return HSPMV_OK;
}

extern "C" {

// The 1.0 layout only (HSPMV_INFO_SIZE_1_0 bytes, frozen for major 1): a
// 1.0 caller's struct is that large whatever this library's hspmv_info is.
static_assert(sizeof(hspmv_info) >= HSPMV_INFO_SIZE_1_0, "hspmv_info shrank below its 1.0 layout");
static_assert(offsetof(hspmv_info, heavy_group_frac) + sizeof(double) == HSPMV_INFO_SIZE_1_0,
              "HSPMV_INFO_SIZE_1_0 must end at the last 1.0 field");

int hspmv_get_info(hspmv_handle *h, hspmv_info *out) {
  clear_error();
  if (!out) return set_error(HSPMV_E_INVALID, "NULL output");
  hspmv_info full;
  const int rc = fill_info(h, &full);
  if (rc) return rc;
  memcpy(out, &full, HSPMV_INFO_SIZE_1_0);
  return HSPMV_OK;
}

#ifdef HSPMV_ENV_KNOBS
// Diagnostic builds only (not in hspmv.h): the last csort launch's
// per-workgroup trace (kCsortTraceSlots u64 each, hspmv_internal.h),
// when the handle was created with HSPMV_CSORT_TRACE=1.  Returns the
// workgroup count (0: no trace).
int hspmv_diag_csort_trace(hspmv_handle *h, unsigned long long *out, int max_wg) {
  if (!h || h->shards.empty()) return 0;
  const Shard &s = h->shards[0];
  if (s.plan.kernel != kCsort || !s.dp.cs.trace) return 0;
  const int n = std::min(max_wg, s.dp.cs.n_wg);
  if (hipSetDevice(s.device) != hipSuccess || hipStreamSynchronize(s.stream) != hipSuccess ||
      hipMemcpy(out, s.dp.cs.trace, 8 * kCsortTraceSlots * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return n;
}

// Diagnostic builds only: build_csort's per-workgroup cost terms {rows,
// slices, chunks, entries, gather quad-sectors, gather sectors, segmented
// chunks, 0} (8 int64 per workgroup).  Returns the workgroup count.
int hspmv_diag_csort_stats(hspmv_handle *h, long long *out, int max_wg) {
  if (!h || h->shards.empty()) return 0;
  const Shard &s = h->shards[0];
  const int n = std::min<int>(max_wg, (int)(s.csort_wg_stats.size() / 8));
  memcpy(out, s.csort_wg_stats.data(), 8 * 8 * (size_t)n);
  return n;
}
#endif

int hspmv_get_info_sized(hspmv_handle *h, hspmv_info *out, uint32_t out_size) {
  clear_error();
  if (!out) return set_error(HSPMV_E_INVALID, "NULL output");
  hspmv_info full;
  int rc = fill_info(h, &full);
  if (rc) return rc;
  memcpy(out, &full, std::min<size_t>(out_size, sizeof(full)));
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
