// hspmv_multi.cpp -- row-range partition over devices; x broadcast / y all-gather (RCCL)
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
  if ((rc = check_deterministic(flags, tune))) return rc;
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
  (void)ncclGetVersion(&h->rccl_version);
  *hp = h.release();
  return HSPMV_OK;
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


int bcast_x(hspmv_handle *h) {
  if (!h->sharded) return HSPMV_OK;
  if (h->comms.empty()) return copy_exchange(h, true);
  const ncclDataType_t dt = h->dtype == HSPMV_F64 ? ncclFloat64 : ncclFloat32;
  return rccl_group(h, "ncclBroadcast(x)", [&](size_t p) {
    Shard &s = h->shards[p];
    return ncclBroadcast(h->shards[0].d_x, s.d_x, (size_t)h->n, dt, 0, h->comms[p], s.stream);
  });
}

int gather_y(hspmv_handle *h) {
  if (!h->sharded) return HSPMV_OK;
  if (h->comms.empty()) return copy_exchange(h, false);
  const ncclDataType_t dt = h->dtype == HSPMV_F64 ? ncclFloat64 : ncclFloat32;
  return rccl_group(h, "ncclAllGather(y)", [&](size_t p) {
    Shard &s = h->shards[p];
    return ncclAllGather(s.d_y, s.d_yfull, (size_t)h->max_rows, dt, h->comms[p], s.stream);
  });
}

}  // namespace hspmv
