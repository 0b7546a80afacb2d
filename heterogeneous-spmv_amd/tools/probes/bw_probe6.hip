// bw_probe6.hip -- calibration microbenchmark (not product code): where the
// cost of the y stores in a streaming SpMV comes from, and which store
// pattern avoids it.  Stream = C3's shape: 64-row wave segments of PER
// nonzeros per row, 16-bit positions + fp64 values (10 B per nonzero), U = 4
// chunks, one sum per row written as y (8 B per row).  Variants:
//   base      : no y stores (a never-taken store keeps the sums live)
//   y.wave    : each wave stores its 64 y values when done (the SpMV kernels)
//   y.l2      : the same stores into a 1 MiB window (stay in L2: the store
//               instructions without the DRAM writes)
//   y.block   : the 4 waves' y through LDS, stored as one 2 KiB run after a
//               block barrier
//   y.nt      : y.wave with nontemporal stores
//   y.x4      : 32 lanes store two rows each (dwordx4)
//   y.block.x4: the block's 256 y through LDS, one wave stores 32 B a lane
//   y.lane0   : one lane per wave stores 8 B (cost per store instruction
//               vs per byte)
//   base+ykern: base, then a second kernel that writes the whole y (two
//               launches timed together: reads and writes never overlap)
//   <v> G=k   : each workgroup takes k consecutive 256-row segments in turn
//               (a wave's y store overlaps its next segment's loads)
//   y.xchg    : the store as a no-return 64-bit atomic exchange
//   y.agent   : a relaxed atomic store at agent scope
//   y.reg G=k : each wave keeps its k segments' sums in registers and stores
//               them after the last one (no store between a wave's loads)
//   y.defer   : persistent grid (256 CUs x 4 blocks), each block keeps its
//               rows' y in LDS and stores them all after its last segment
//   regp (mode 3): persistent grid of 1024-4096 blocks (what the CUs hold
//               at once), block b takes segments b, b + grid, ..., keeps the
//               sums in registers, stores y after its last segment
// Reported: ms (min of 10) and effective GB/s over the stream + y bytes.
//
//   hipcc -O3 --offload-arch=gfx950 bw_probe6.hip -o bw_probe6 && ./bw_probe6 [PER]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
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

enum { Y_NONE = 0, Y_WAVE = 1, Y_L2 = 2, Y_BLOCK = 3, Y_NT = 4, Y_X4 = 5, Y_BX4 = 6, Y_LANE0 = 7, Y_REG = 8, Y_XCHG = 9, Y_SC = 10 };
constexpr int U = 4;

// one wave's 64 rows: returns this lane's row sum
template <int U = ::U>
__device__ __forceinline__ double segment(const uint16_t *__restrict__ pos,
                                          const double *__restrict__ val, long s0, long s1,
                                          int lane, double *lds) {
  double acc = 0.0;
  for (long c = s0; c < s1; c += 64 * U) {
    uint16_t p[U];
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = std::min(c + u * 64 + lane, s1 - 1);
      p[u] = pos[j];
      v[u] = val[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) lds[u * 64 + lane] = v[u] * (double)(p[u] & 7);
    __builtin_amdgcn_wave_barrier();
    // every lane sums 4 of the chunk's products (stands in for the row sums)
#pragma unroll
    for (int u = 0; u < U; ++u) acc += lds[((lane * 4 + u) & (64 * U - 1))];
    __builtin_amdgcn_wave_barrier();
  }
  return acc;
}

template <int MODE, int G = 1, int UU = U>
__global__ __launch_bounds__(256) void probe(const uint16_t *__restrict__ pos,
                                             const double *__restrict__ val, double *__restrict__ y,
                                             long m, int per, double *__restrict__ out) {
  __shared__ double lds[4 * 64 * UU];
  __shared__ double ys[256];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double keep[G];
  for (int gi = 0; gi < G; ++gi) {
  const long w = ((long)blockIdx.x * G + gi) * 4 + wid;
  const long r = w * 64 + lane;
  const long nnz = m * per;
  const long s0 = std::min(w * 64 * per, nnz), s1 = std::min(s0 + 64L * per, nnz);
  const double s = segment<UU>(pos, val, s0, s1, lane, lds + wid * 64 * UU);
  if constexpr (MODE == Y_NONE) {
    if (s == 12345.678) out[0] = s;
  } else if constexpr (MODE == Y_WAVE) {
    if (r < m) y[r] = s;
  } else if constexpr (MODE == Y_L2) {
    if (r < m) y[r & 0x1FFFF] = s;
  } else if constexpr (MODE == Y_NT) {
    if (r < m) __builtin_nontemporal_store(s, y + r);
  } else if constexpr (MODE == Y_X4) {
    // 32 lanes store two rows each (16 B): half the store instructions' lanes
    const double o = __shfl_down(s, 1, 64);
    const long r2 = w * 64 + 2 * (lane & 31);
    if (lane < 32 && r2 + 1 < m) {
      const double e = __shfl(s, 2 * lane, 64), f = __shfl(s, 2 * lane + 1, 64);
      (void)o;
      *reinterpret_cast<double2 *>(y + r2) = make_double2(e, f);
    }
  } else if constexpr (MODE == Y_BX4) {
    ys[threadIdx.x] = s;
    __syncthreads();
    const long rb = (long)blockIdx.x * 256;
    if (wid == 0 && rb + 256 <= m) {  // one wave: 64 lanes x 32 B
      const double4 t = *reinterpret_cast<const double4 *>(ys + 4 * lane);
      *reinterpret_cast<double2 *>(y + rb + 4 * lane) = make_double2(t.x, t.y);
      *reinterpret_cast<double2 *>(y + rb + 4 * lane + 2) = make_double2(t.z, t.w);
    }
  } else if constexpr (MODE == Y_XCHG) {
    // the y store as a no-return atomic exchange (processed at the L2)
    if (r < m) (void)__hip_atomic_exchange(reinterpret_cast<unsigned long long *>(y + r),
                                          (unsigned long long)__builtin_bit_cast(long long, s),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (MODE == Y_SC) {
    // the y store with device scope (sc1): written through to L2 at once
    if (r < m) __hip_atomic_store(y + r, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (MODE == Y_REG) {
    keep[gi] = s;  // stored after the last segment
  } else if constexpr (MODE == Y_LANE0) {
    if (lane == 0 && r < m) y[r] = s;  // 8 B per wave: one store, one lane
  } else if constexpr (MODE == Y_BLOCK) {
    ys[threadIdx.x] = s;
    __syncthreads();
    const long rb = (long)blockIdx.x * 256;
    if (rb + threadIdx.x < m) y[rb + threadIdx.x] = ys[threadIdx.x];
  }
  }
  if constexpr (MODE == Y_REG) {
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const long r = (((long)blockIdx.x * G + gi) * 4 + wid) * 64 + lane;
      if (r < m) y[r] = keep[gi];
    }
  }
}

// A wave takes G consecutive 64-row segments as one chunk stream with the
// next chunk's loads issued before the current chunk's products (PF); a
// segment's y is stored right after the loads of the following segment's
// first chunk, so the store's completion overlaps those loads instead of
// ending the wave (YS = 0: no y stores, same loop).
template <int G, bool YS>
__global__ __launch_bounds__(256) void probe_pipe(const uint16_t *__restrict__ pos,
                                                  const double *__restrict__ val,
                                                  double *__restrict__ y, long m, int per,
                                                  double *__restrict__ out) {
  __shared__ double ldsa[4 * 64 * U];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double *lds = ldsa + wid * 64 * U;
  const long nnz = m * per;
  const long w0 = ((long)blockIdx.x * 4 + wid) * G;  // this wave's first segment
  auto sb = [&](int g) { return std::min((w0 + g) * 64 * per, nnz); };
  auto se = [&](int g) { return std::min((w0 + g + 1) * 64 * per, nnz); };
  int seg = 0;
  long c = sb(0);
  if (c >= se(0)) return;
  uint16_t p[U], pn[U];
  double v[U], vn[U];
  auto load = [&](long c0, long c1, uint16_t *pp, double *vv) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = std::min(c0 + u * 64 + lane, c1 - 1);
      pp[u] = pos[j];
      vv[u] = val[j];
    }
  };
  load(c, se(0), p, v);
  double acc = 0.0;
  while (true) {
    long cn = c + 64 * U;
    int sn = seg;
    if (cn >= se(seg)) {
      sn = seg + 1;
      cn = sb(sn);
    }
    const bool more = sn < G && cn < se(sn);
    __builtin_amdgcn_sched_barrier(0);
    if (more) load(cn, se(sn), pn, vn);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) lds[u * 64 + lane] = v[u] * (double)(p[u] & 7);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < U; ++u) acc += lds[((lane * 4 + u) & (64 * U - 1))];
    __builtin_amdgcn_wave_barrier();
    if (sn != seg) {
      const long r = (w0 + seg) * 64 + lane;
      if constexpr (YS) {
        if (r < m) y[r] = acc;
      } else {
        if (acc == 12345.678) out[0] = acc;
      }
      acc = 0.0;
    }
    if (!more) break;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      p[u] = pn[u];
      v[u] = vn[u];
    }
    c = cn;
    seg = sn;
  }
}

// Same, branch-free: every step loads chunk k+1 (clamped to the last), uses
// chunk k, and stores a finished segment's y after those loads; the chunk
// registers ping-pong (unrolled by two), so the use of chunk k waits only for
// its own loads (vmcnt counts the younger loads and the store).
template <int G, bool YS>
__global__ __launch_bounds__(256) void probe_pipe2(const uint16_t *__restrict__ pos,
                                                   const double *__restrict__ val,
                                                   double *__restrict__ y, long m, int per,
                                                   double *__restrict__ out) {
  __shared__ double ldsa[4 * 64 * U];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double *lds = ldsa + wid * 64 * U;
  const long nnz = m * per;
  const long w0 = ((long)blockIdx.x * 4 + wid) * G;
  const int nc = (64 * per + 64 * U - 1) / (64 * U);  // chunks per segment
  const int T = G * nc;
  if (w0 * 64 >= m) return;
  struct Ch {
    uint16_t p[U];
    double v[U];
  };
  auto load = [&](int k, Ch &ch) {
    k = min(k, T - 1);
    const long sg = w0 + k / nc;
    const long b = std::min(sg * 64 * per, nnz), e = std::min(b + 64L * per, nnz);
    const long c = b + (long)(k % nc) * 64 * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = std::max(std::min(c + u * 64 + lane, e - 1), 0L);
      ch.p[u] = pos[j];
      ch.v[u] = val[j];
    }
  };
  double acc = 0.0;
  auto use = [&](int k, const Ch &ch) {
#pragma unroll
    for (int u = 0; u < U; ++u) lds[u * 64 + lane] = ch.v[u] * (double)(ch.p[u] & 7);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < U; ++u) acc += lds[((lane * 4 + u) & (64 * U - 1))];
    __builtin_amdgcn_wave_barrier();
    if (k % nc == nc - 1) {
      const long r = (w0 + k / nc) * 64 + lane;
      if constexpr (YS) {
        if (r < m) y[r] = acc;
      } else {
        if (acc == 12345.678) out[0] = acc;
      }
      acc = 0.0;
    }
  };
  Ch a, b;
  load(0, a);
  for (int k = 0; k < T; k += 2) {
    __builtin_amdgcn_sched_barrier(0);
    load(k + 1, b);
    __builtin_amdgcn_sched_barrier(0);
    use(k, a);
    if (k + 1 >= T) break;
    __builtin_amdgcn_sched_barrier(0);
    load(k + 2, a);
    __builtin_amdgcn_sched_barrier(0);
    use(k + 1, b);
  }
}

__global__ __launch_bounds__(256) void ykern(double *__restrict__ y, long m) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < m) y[i] = (double)(i & 15);
}

// persistent: block b takes segments (4 waves each) b, b + G, ... and keeps
// their y in LDS (up to KEEP rows per block), storing them at the end
template <int KEEP>
__global__ __launch_bounds__(256) void probe_defer(const uint16_t *__restrict__ pos,
                                                   const double *__restrict__ val,
                                                   double *__restrict__ y, long m, int per) {
  __shared__ double lds[4 * 64 * U];
  __shared__ double ys[KEEP];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long nnz = m * per;
  const long nseg = (m + 255) / 256;
  int k = 0;
  for (long b = blockIdx.x; b < nseg; b += gridDim.x, ++k) {
    const long w = b * 4 + wid;
    const long s0 = std::min(w * 64 * per, nnz), s1 = std::min(s0 + 64L * per, nnz);
    ys[k * 256 + threadIdx.x] = segment(pos, val, s0, s1, lane, lds + wid * 64 * U);
  }
  __syncthreads();
  k = 0;
  for (long b = blockIdx.x; b < nseg; b += gridDim.x, ++k)
    if (b * 256 + threadIdx.x < m) y[b * 256 + threadIdx.x] = ys[k * 256 + threadIdx.x];
}

// persistent at full occupancy: the grid is what the CUs hold at once
// (gridDim.x blocks), block b takes segments b, b + G, ... (at most K, so
// the blocks in flight read neighbouring rows), keeps each segment's sums
// in registers and stores them all after its last segment (YS = 0: no y)
template <int K, bool YS, int YM = 0>
__global__ __launch_bounds__(256) void probe_regp(const uint16_t *__restrict__ pos,
                                                  const double *__restrict__ val,
                                                  double *__restrict__ y, long m, int per,
                                                  double *__restrict__ out) {
  __shared__ double lds[4 * 64 * U];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long nnz = m * per;
  const long nseg = (m + 255) / 256;
  double keep[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const long b = blockIdx.x + (long)k * gridDim.x;
    keep[k] = 0.0;
    if (b < nseg) {
      const long w = b * 4 + wid;
      const long s0 = std::min(w * 64 * per, nnz), s1 = std::min(s0 + 64L * per, nnz);
      keep[k] = segment(pos, val, s0, s1, lane, lds + wid * 64 * U);
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const long r = (blockIdx.x + (long)k * gridDim.x) * 256 + threadIdx.x;
    if constexpr (YS && YM == 0) {
      if (r < m) y[r] = keep[k];
    } else if constexpr (YS && YM == 1) {  // into a 1 MiB window (stays in L2)
      if (r < m) y[r & 0x1FFFF] = keep[k];
    } else if constexpr (YS && YM == 2) {  // one lane per wave (8 B)
      if (lane == 0 && r < m) y[r] = keep[k];
    } else {
      if (keep[k] == 12345.678) out[0] = keep[k];
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
  const int per = argc > 1 ? atoi(argv[1]) : 27;
  const long m = argc > 2 ? atol(argv[2]) : (2L << 20);
  const long nnz = m * per;
  uint16_t *pos;
  double *val, *y, *out;
  CK(hipMalloc(&pos, nnz * 2));
  CK(hipMalloc(&val, nnz * 8));
  CK(hipMalloc(&y, m * 8));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(pos, 1, nnz * 2));
  CK(hipMemset(val, 0, nnz * 8));
  CK(hipMemset(y, 0, m * 8));
  const unsigned grid = (unsigned)((m + 255) / 256);
  const double sb = (double)nnz * 10, yb = (double)m * 8;
  auto report = [&](const char *name, float ms, double bytes) {
    printf("{\"per_row\": %d, \"m\": %ld, \"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.0f}\n", per, m,
           name, ms, bytes / ms * 1e-6);
    fflush(stdout);
  };
  auto run = [&](auto kern, const char *name, double bytes, int G = 1) {
    const unsigned g = (grid + G - 1) / G;
    const float ms = time_ms([&] { hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, pos, val, y, m, per, out); }, 10);
    report(name, ms, bytes);
  };
  if (argc > 3 && atoi(argv[3]) == 3) {  // persistent register-deferred y vs the plain grid
    auto runp = [&](auto kern, const char *name, double bytes, unsigned g) {
      const float ms = time_ms([&] { hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, pos, val, y, m, per, out); }, 10);
      report(name, ms, bytes);
    };
    const long nseg = (m + 255) / 256;
    for (int rep = 0; rep < 2; ++rep) {
      run(probe<Y_NONE>, "base", sb);
      run(probe<Y_WAVE>, "y.wave", sb + yb);
      if (nseg <= 8L * 2048) {
        runp(probe_regp<8, false>, "regp base 1024 blocks", sb, 1024);
        runp(probe_regp<8, true>, "regp y 1024 blocks", sb + yb, 1024);
      }
      if (nseg <= 4L * 2048) {
        runp(probe_regp<4, false>, "regp base 2048 blocks", sb, 2048);
        runp(probe_regp<4, true>, "regp y 2048 blocks", sb + yb, 2048);
        runp(probe_regp<4, true, 1>, "regp y.l2 2048 blocks", sb + yb, 2048);
        runp(probe_regp<4, true, 2>, "regp y.lane0 2048 blocks", sb + yb, 2048);
      }
      if (nseg <= 8L * 1024) {
        runp(probe_regp<8, true, 1>, "regp y.l2 1024 blocks", sb + yb, 1024);
        runp(probe_regp<8, true, 2>, "regp y.lane0 1024 blocks", sb + yb, 1024);
      }
      if (nseg <= 6L * 1280) {
        runp(probe_regp<6, false>, "regp base 1280 blocks", sb, 1280);
        runp(probe_regp<6, true>, "regp y 1280 blocks", sb + yb, 1280);
      }
      if (nseg <= 2L * 4096) {
        runp(probe_regp<2, false>, "regp base 4096 blocks", sb, 4096);
        runp(probe_regp<2, true>, "regp y 4096 blocks", sb + yb, 4096);
      }
    }
    return 0;
  }
  const bool reg_only = argc > 3 && atoi(argv[3]) == 1;
  if (argc > 3 && atoi(argv[3]) == 2) {
    for (int rep = 0; rep < 2; ++rep) {
      run(probe<Y_NONE>, "base", sb);
      run(probe<Y_WAVE>, "y.wave", sb + yb);
      run(probe<Y_XCHG>, "y.xchg", sb + yb);
      run(probe<Y_SC>, "y.agent", sb + yb);
      run(probe<Y_NT>, "y.nt", sb + yb);
    }
    return 0;
  }
  for (int rep = 0; rep < 2 && reg_only; ++rep) {
    run(probe<Y_NONE>, "base", sb);
    run(probe<Y_WAVE>, "y.wave", sb + yb);
    run(probe<Y_NONE, 2>, "base G=2", sb, 2);
    run(probe<Y_REG, 2>, "y.reg G=2", sb + yb, 2);
    run(probe<Y_WAVE, 2>, "y.wave G=2", sb + yb, 2);
    run(probe<Y_NONE, 4>, "base G=4", sb, 4);
    run(probe<Y_REG, 4>, "y.reg G=4", sb + yb, 4);
    run(probe<Y_NONE, 8>, "base G=8", sb, 8);
    run(probe<Y_REG, 8>, "y.reg G=8", sb + yb, 8);
  }
  for (int rep = 0; rep < 2 && !reg_only; ++rep) {
    run(probe<Y_NONE>, "base", sb);
    run(probe<Y_WAVE>, "y.wave", sb + yb);
    run(probe<Y_L2>, "y.l2", sb + yb);
    run(probe<Y_BLOCK>, "y.block", sb + yb);
    run(probe<Y_NT>, "y.nt", sb + yb);
    run(probe<Y_NONE, 1, 8>, "base U=8", sb);
    run(probe<Y_WAVE, 1, 8>, "y.wave U=8", sb + yb);
    run(probe<Y_NONE, 1, 2>, "base U=2", sb);
    run(probe<Y_WAVE, 1, 2>, "y.wave U=2", sb + yb);
    run(probe<Y_X4>, "y.x4 (32 lanes x 16 B)", sb + yb);
    run(probe<Y_BX4>, "y.block.x4 (1 wave x 32 B)", sb + yb);
    run(probe<Y_LANE0>, "y.lane0 (8 B per wave)", sb + yb);
    run(probe<Y_NONE, 2>, "base G=2", sb, 2);
    run(probe<Y_WAVE, 2>, "y.wave G=2", sb + yb, 2);
    run(probe<Y_NONE, 4>, "base G=4", sb, 4);
    run(probe<Y_WAVE, 4>, "y.wave G=4", sb + yb, 4);
    run(probe<Y_L2, 4>, "y.l2 G=4", sb + yb, 4);
    run(probe<Y_WAVE, 8>, "y.wave G=8", sb + yb, 8);
    run(probe_pipe2<1, false>, "pipe2 base G=1", sb, 1);
    run(probe_pipe2<1, true>, "pipe2 y G=1", sb + yb, 1);
    run(probe_pipe2<2, false>, "pipe2 base G=2", sb, 2);
    run(probe_pipe2<2, true>, "pipe2 y G=2", sb + yb, 2);
    run(probe_pipe2<4, false>, "pipe2 base G=4", sb, 4);
    run(probe_pipe2<4, true>, "pipe2 y G=4", sb + yb, 4);
    run(probe_pipe2<8, true>, "pipe2 y G=8", sb + yb, 8);
    {
      const float ms = time_ms([&] {
        hipLaunchKernelGGL(probe<Y_NONE>, dim3(grid), dim3(256), 0, 0, pos, val, y, m, per, out);
        hipLaunchKernelGGL(ykern, dim3(grid), dim3(256), 0, 0, y, m);
      }, 10);
      report("base+ykern", ms, sb + yb);
    }
    {
      const float ms = time_ms([&] { hipLaunchKernelGGL(ykern, dim3(grid), dim3(256), 0, 0, y, m); }, 10);
      report("ykern only", ms, yb);
    }
    {
      constexpr int KEEP = 16 * 256;  // 32 KiB of y per block
      const unsigned g = 256 * 4;
      if ((long)g * KEEP >= m) {
        const float ms = time_ms([&] { hipLaunchKernelGGL(probe_defer<KEEP>, dim3(g), dim3(256), 0, 0, pos, val, y, m, per); }, 10);
        report("y.defer (1024 blocks, 32 KiB y each)", ms, sb + yb);
      }
    }
  }
  CK(hipGetLastError());
  return 0;
}
