// bw_probe3.hip -- calibration microbenchmark (not product code): which of
// the SpMV's side streams costs HBM efficiency.  Base = bw_probe2's shape
// (one wave per segment of SEG nonzeros, narrow U=4 chunks of col + fp64
// val).  Variants add, one at a time, what the STREAM kernel does besides:
//   +rp : each wave first loads 65 row pointers (4 B/row, 64 rows per wave)
//         and waits for them before its col/val loads (the dependent start)
//   +y  : each wave stores 64 doubles at its end (the y rows)
//   +ynt: same stores, nontemporal
//   +x  : a dependent gather x[col] per element, col = row +- 32 band
//         (the C4 pattern) from an x of m doubles
//   all : +rp +x +y
// Reported as "effective" GB/s = (col+val+rp+y+x-distinct bytes) / time.
//
//   hipcc -O3 --offload-arch=gfx950 bw_probe3.hip -o bw_probe3 && ./bw_probe3
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                        \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

enum { RP = 1, Y = 2, YNT = 4, X = 8, YSMALL = 16, XIND = 32, XPF = 64 };

template <int MODE, int G = 1>
__global__ __launch_bounds__(256) void probe(const int *__restrict__ col,
                                             const double *__restrict__ val,
                                             const int *__restrict__ rp,
                                             const double *__restrict__ x,
                                             double *__restrict__ y, long nnz, int per_row,
                                             double *__restrict__ out) {
  constexpr int U = 4;
  const int lane = threadIdx.x & 63;
  const long seg = 64L * per_row;
  for (int gi = 0; gi < G; ++gi) {
  const long w = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * G + gi;
  long s0 = w * seg;
  if (s0 >= nnz) return;
  if constexpr ((MODE & RP) != 0) {
    // dependent start: the segment base comes from the loaded row pointer
    const int b = rp[w * 64 + lane];
    s0 = __builtin_amdgcn_readfirstlane(__shfl(b, 0, 64));
  }
  const long s1 = std::min(s0 + seg, nnz);
  double s = 0.0;
  if constexpr ((MODE & XPF) != 0) {
    // software-pipelined: chunk k+1's col/val issued before chunk k's gather
    int cv[U], cn[U];
    double vv[U], vn[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = std::min(s0 + u * 64 + lane, nnz - 1);
      cv[u] = col[j];
      vv[u] = val[j];
    }
    for (long c = s0; c < s1; c += 64 * U) {
      double xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xv[u] = x[cv[u]];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long j = std::min(c + 64 * U + u * 64 + lane, nnz - 1);
        cn[u] = col[j];
        vn[u] = val[j];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) s += vv[u] * xv[u];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        cv[u] = cn[u];
        vv[u] = vn[u];
      }
    }
  } else
  for (long c = s0; c < s1; c += 64 * U) {
    int cv[U];
    double vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = std::min(c + u * 64 + lane, nnz - 1);
      cv[u] = col[j];
      vv[u] = val[j];
    }
    if constexpr ((MODE & XIND) != 0) {
      // same gather bytes, address independent of the loaded col
      double xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xv[u] = x[std::min(c / per_row + ((u * 64 + lane) * 7) % 96 - 32 + 64, (long)(nnz / per_row) - 1)];
#pragma unroll
      for (int u = 0; u < U; ++u) s += vv[u] * xv[u] + cv[u];
    } else if constexpr ((MODE & X) != 0) {
      double xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xv[u] = x[cv[u]];
#pragma unroll
      for (int u = 0; u < U; ++u) s += vv[u] * xv[u];
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) s += vv[u] * (double)cv[u];
    }
  }
  if constexpr ((MODE & YSMALL) != 0) {
    y[(w * 64 + lane) & 0x1FFFF] = s;  // 1 MiB of y lines: stays in L2
  } else if constexpr ((MODE & (Y | YNT)) != 0) {
    const long r = w * 64 + lane;
    if constexpr ((MODE & YNT) != 0)
      __builtin_nontemporal_store(s, y + r);
    else
      y[r] = s;
  } else {
    if (s == 12345.678) out[0] = s;
  }
  }
}

template <typename F>
float time_ms(F launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  std::vector<float> t;
  for (int r = 0; r < reps + 3; ++r) {
    (void)hipEventRecord(a);
    launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r >= 3) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[0];
}

int main(int argc, char **argv) {
  const int per_row = argc > 1 ? atoi(argv[1]) : 10;  // 10 ~ C4, 27 ~ C3
  const long m = 25L << 20;                            // rows (C4 shard ~2.5M is 10x smaller; keep HBM-resident)
  const long nnz = m * per_row;
  std::vector<int> hcol(nnz), hrp(m + 1);
  unsigned long long st = 12345;
  for (long r = 0; r < m; ++r) {
    hrp[r] = (int)(r * per_row);
    for (int k = 0; k < per_row; ++k) {
      st = st * 6364136223846793005ULL + 1442695040888963407ULL;
      long c = r + (long)((st >> 33) % 65) - 32;
      hcol[r * per_row + k] = (int)std::min(std::max(c, 0L), m - 1);
    }
  }
  hrp[m] = (int)nnz;
  int *col, *rp;
  double *val, *x, *y, *out;
  CK(hipMalloc(&col, nnz * 4));
  CK(hipMalloc(&val, nnz * 8));
  CK(hipMalloc(&rp, (m + 1) * 4));
  CK(hipMalloc(&x, m * 8));
  CK(hipMalloc(&y, m * 8));
  CK(hipMalloc(&out, 64));
  CK(hipMemcpy(col, hcol.data(), nnz * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(rp, hrp.data(), (m + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemset(val, 0, nnz * 8));
  CK(hipMemset(x, 0, m * 8));
  const unsigned grid = (unsigned)((m / 64 + 3) / 4);
  const double base = (double)nnz * 12;
  auto run = [&](auto kern, double bytes, const char *name, int G = 1) {
    const unsigned g = (grid + G - 1) / G;
    const float ms = time_ms([&] { hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, col, val, rp, x, y, nnz, per_row, out); }, 10);
    printf("{\"per_row\": %d, \"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.0f}\n", per_row, name, ms,
           bytes / ms * 1e-6);
    fflush(stdout);
  };
  run(probe<0>, base, "base");
  run(probe<RP>, base + m * 4.0, "+rp");
  run(probe<Y>, base + m * 8.0, "+y");
  run(probe<YNT>, base + m * 8.0, "+ynt");
  run(probe<X>, base + m * 8.0, "+x");
  run(probe<RP | X | Y>, base + m * 20.0, "all");
  run(probe<0>, base, "base");
  run(probe<X>, base + m * 8.0, "+x");
  run(probe<XIND>, base + m * 8.0, "+x-independent");
  run(probe<XPF>, base + m * 8.0, "+x-pipelined");
  run(probe<0>, base, "base");
  CK(hipGetLastError());
  return 0;
}
