// Internal interfaces shared by the host runtime (hspmv_api.cpp) and the
// HIP kernels (spmv_kernels.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace hspmv {

// Device view of one CSR shard (rows [0, m) of the shard; global columns).
struct DevCSR {
  int32_t m = 0;
  int64_t n = 0;
  int64_t nnz = 0;
  const int32_t *row_ptr = nullptr;
  const int32_t *col_idx = nullptr;
  const void *val = nullptr;
  int32_t n_ssr = 0, n_sr = 0;          // CSR-3 maps (0 = none)
  const int32_t *outer = nullptr;
  const int32_t *inner = nullptr;
};

enum Kernel : int { kAuto = 0, kVector = 1, kStream = 2, kCsr3 = 3 };

struct LaunchPlan {
  int kernel = kStream;
  int lanes = 64;          // VECTOR: lanes per row; STREAM: rows per task
  int waves_per_block = 4; // CSR3: waves per super-super-row workgroup
  bool nontemporal = false;
  int64_t blocks = 0;
};

// Chooses kernel / lanes / block shape for a shard (host-side heuristic).
LaunchPlan plan_launch(const DevCSR &A, int dtype, unsigned flags,
                       double max_ssr_rows_mean);

// Enqueues one y = A*x.  Returns hipSuccess or the launch error.
hipError_t launch_spmv(const DevCSR &A, int dtype, const LaunchPlan &plan,
                       const void *x, void *y, hipStream_t stream);

}  // namespace hspmv
