// csort_proto.hip -- design probe for irregular (power-law, random-column)
// matrices: each workgroup owns a nnz-balanced row block and walks ITS
// nonzeros in COLUMN order, so the 64 lanes of a gather fall on a few x
// lines (coalesced in L1/TA) and all CUs of an XCD sweep x together (L2
// hits), instead of one L2 request per nonzero.  Row sums accumulate in an
// LDS array (one slot per row of the block) with LDS atomic adds.
//
// Not part of the product: a timing probe.  Checks its y against a host
// CSR loop (fp64 reference of the fp32 data) and prints JSON lines.
//   build/csort_proto [m] [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__);   \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int kLong = 4096;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------ kernels

// Variant A: per-entry 32-bit column, 16-bit block-local row, fp32 value.
template <typename Acc, int U, int NTH>
__global__ __launch_bounds__(NTH) void csort_kernel(const int64_t *__restrict__ blk_k,
                                                    const int32_t *__restrict__ blk_r,
                                                    const int32_t *__restrict__ col,
                                                    const uint16_t *__restrict__ rowl,
                                                    const float *__restrict__ val,
                                                    const float *__restrict__ x,
                                                    float *__restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Acc *acc = reinterpret_cast<Acc *>(smem);
  const int b = blockIdx.x;
  const int64_t k0 = blk_k[b], k1 = blk_k[b + 1];
  const int32_t r0 = blk_r[b], r1 = blk_r[b + 1];
  const int nr = r1 - r0;
  for (int i = threadIdx.x; i < nr; i += NTH) acc[i] = Acc(0);
  __syncthreads();
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int NW = NTH / 64;
  for (int64_t c = k0 + (int64_t)wid * 64 * U; c < k1; c += (int64_t)NW * 64 * U) {
    int32_t cc[U];
    uint16_t rr[U];
    float vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = min(c + u * 64 + lane, k1 - 1);
      cc[u] = col[k];
      rr[u] = rowl[k];
      vv[u] = val[k];
    }
    float xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = x[cc[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = c + u * 64 + lane;
      if (k < k1) atomicAdd(&acc[rr[u]], (Acc)(vv[u] * xv[u]));
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nr; i += NTH) y[r0 + i] = (float)acc[i];
}

// Variant B: 16-bit column offset from a per-64U-chunk base (chunks never
// span more than 65535 columns: the host pads), 16-bit row, fp32 value:
// 8 B/nnz like CSR fp32.
template <typename Acc, int U, int NTH>
__global__ __launch_bounds__(NTH) void csort16_kernel(const int64_t *__restrict__ blk_k,
                                                      const int32_t *__restrict__ blk_r,
                                                      const int32_t *__restrict__ cbase,
                                                      const uint16_t *__restrict__ coff,
                                                      const uint16_t *__restrict__ rowl,
                                                      const float *__restrict__ val,
                                                      const float *__restrict__ x,
                                                      float *__restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Acc *acc = reinterpret_cast<Acc *>(smem);
  const int b = blockIdx.x;
  const int64_t k0 = blk_k[b], k1 = blk_k[b + 1];
  const int32_t r0 = blk_r[b], r1 = blk_r[b + 1];
  const int nr = r1 - r0;
  for (int i = threadIdx.x; i < nr; i += NTH) acc[i] = Acc(0);
  __syncthreads();
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int NW = NTH / 64;
  for (int64_t c = k0 + (int64_t)wid * 64 * U; c < k1; c += (int64_t)NW * 64 * U) {
    const int32_t base = cbase[c / (64 * U)];
    uint16_t oo[U], rr[U];
    float vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = c + u * 64 + lane;  // blocks padded to whole chunks
      oo[u] = coff[k];
      rr[u] = rowl[k];
      vv[u] = val[k];
    }
    float xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = x[base + oo[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) atomicAdd(&acc[rr[u]], (Acc)(vv[u] * xv[u]));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nr; i += NTH) y[r0 + i] = (float)acc[i];
}

// Variant C: generic padded form.  PACK 0: coff/rowl/val arrays; 1: packed
// uint32 (row << 16 | coff) + val; 2: AoS {uint32 idx, float val} as one
// 8-byte load.  NT: nontemporal stream loads.  DIAG 1: no LDS atomics
// (per-lane register sums, wrong y); 2: no x gather (x := 1, wrong y).
template <typename Acc, int U, int NTH, int PACK, bool NT, int DIAG>
__global__ __launch_bounds__(NTH) void csortg_kernel(const int64_t *__restrict__ blk_k,
                                                     const int32_t *__restrict__ blk_r,
                                                     const int32_t *__restrict__ cbase,
                                                     const uint16_t *__restrict__ coff,
                                                     const uint16_t *__restrict__ rowl,
                                                     const uint32_t *__restrict__ pidx,
                                                     const float *__restrict__ val,
                                                     const u32x2 *__restrict__ aos,
                                                     const float *__restrict__ x,
                                                     float *__restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Acc *acc = reinterpret_cast<Acc *>(smem);
  const int b = blockIdx.x;
  const int64_t k0 = blk_k[b], k1 = blk_k[b + 1];
  const int32_t r0 = blk_r[b], r1 = blk_r[b + 1];
  const int nr = r1 - r0;
  for (int i = threadIdx.x; i < nr; i += NTH) acc[i] = Acc(0);
  __syncthreads();
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int NW = NTH / 64;
  Acc dsum = Acc(0);
  for (int64_t c = k0 + (int64_t)wid * 64 * U; c < k1; c += (int64_t)NW * 64 * U) {
    const int32_t base = cbase[c / (64 * U)];
    uint32_t oo[U], rr[U];
    float vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = c + u * 64 + lane;
      if constexpr (PACK == 0) {
        oo[u] = NT ? __builtin_nontemporal_load(coff + k) : coff[k];
        rr[u] = NT ? __builtin_nontemporal_load(rowl + k) : rowl[k];
        vv[u] = NT ? __builtin_nontemporal_load(val + k) : val[k];
      } else if constexpr (PACK == 1) {
        const uint32_t p = NT ? __builtin_nontemporal_load(pidx + k) : pidx[k];
        oo[u] = p & 0xffffu;
        rr[u] = p >> 16;
        vv[u] = NT ? __builtin_nontemporal_load(val + k) : val[k];
      } else {
        const u32x2 p = NT ? __builtin_nontemporal_load(aos + k) : aos[k];
        oo[u] = p.x & 0xffffu;
        rr[u] = p.x >> 16;
        vv[u] = __uint_as_float(p.y);
      }
    }
    float xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = DIAG == 2 ? 1.0f : x[base + oo[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (DIAG == 1)
        dsum += (Acc)(vv[u] * xv[u]) * (Acc)(rr[u] + 1);
      else
        atomicAdd(&acc[rr[u]], (Acc)(vv[u] * xv[u]));
    }
  }
  if constexpr (DIAG == 1) acc[threadIdx.x % (nr > 0 ? nr : 1)] = dsum;
  __syncthreads();
  for (int i = threadIdx.x; i < nr; i += NTH) y[r0 + i] = (float)acc[i];
}

// Variant H: 2-D split.  Workgroup b handles row block b / H and column
// part h = b % H (x[h*N/H, (h+1)*N/H)); its fp64 row sums go to
// part[h*m + row]; csort_finish adds the H partials per row (fixed order).
template <int U, int NTH, bool NT, int H, typename Acc = double>
__global__ __launch_bounds__(NTH) void csorth_kernel(const int64_t *__restrict__ blk_k,
                                                     const int32_t *__restrict__ blk_r,
                                                     const int32_t *__restrict__ cbase,
                                                     const u32x2 *__restrict__ aos,
                                                     const float *__restrict__ x, int64_t m,
                                                     double *__restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Acc *acc = reinterpret_cast<Acc *>(smem);
  const int b = blockIdx.x;
  const int rb = b / H, h = b % H;
  const int64_t k0 = blk_k[b], k1 = blk_k[b + 1];
  const int32_t r0 = blk_r[rb], r1 = blk_r[rb + 1];
  const int nr = r1 - r0;
  for (int i = threadIdx.x; i < nr; i += NTH) acc[i] = Acc(0);
  __syncthreads();
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int NW = NTH / 64;
  for (int64_t c = k0 + (int64_t)wid * 64 * U; c < k1; c += (int64_t)NW * 64 * U) {
    const int32_t base = cbase[c / (64 * U)];
    uint32_t oo[U], rr[U];
    float vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = c + u * 64 + lane;
      const u32x2 p = NT ? __builtin_nontemporal_load(aos + k) : aos[k];
      oo[u] = p.x & 0xffffu;
      rr[u] = p.x >> 16;
      vv[u] = __uint_as_float(p.y);
    }
    float xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = x[base + oo[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) atomicAdd(&acc[rr[u]], (Acc)(vv[u] * xv[u]));
  }
  __syncthreads();
  double *out = part + (int64_t)h * m + r0;
  for (int i = threadIdx.x; i < nr; i += NTH) out[i] = (double)acc[i];
}

template <int H>
__global__ __launch_bounds__(256) void csort_finish(int64_t m, const double *__restrict__ part,
                                                    float *__restrict__ y) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= m) return;
  double s = part[r];
#pragma unroll
  for (int h = 1; h < H; ++h) s += part[(int64_t)h * m + r];
  y[r] = (float)s;
}

// ------------------------------------------------------------------ host

struct Csr {
  int64_t m = 0;
  std::vector<int64_t> rp;
  std::vector<int32_t> ci;
  std::vector<float> v;
};

static Csr powerlaw(int64_t m, uint64_t seed) {
  std::mt19937_64 g(seed);
  std::exponential_distribution<double> ex(1.0);
  std::uniform_int_distribution<int64_t> uc(0, m - 1);
  std::vector<uint64_t> e;
  e.reserve((size_t)(m * 26));
  for (int64_t r = 0; r < m; ++r) {
    const double p = std::exp(ex(g) / 1.5) - 1.0;
    const int64_t d = std::min<int64_t>((int64_t)(4.0 * (p + 1.0)), std::max<int64_t>(m / 10, 1));
    for (int64_t j = 0; j < d; ++j) {
      const uint64_t c = (uint64_t)uc(g);
      e.push_back(((uint64_t)r << 32) | c);
      e.push_back((c << 32) | (uint64_t)r);
    }
    e.push_back(((uint64_t)r << 32) | (uint64_t)r);
  }
  std::sort(e.begin(), e.end());
  e.erase(std::unique(e.begin(), e.end()), e.end());
  Csr A;
  A.m = m;
  A.rp.assign((size_t)m + 1, 0);
  A.ci.resize(e.size());
  A.v.resize(e.size());
  std::uniform_real_distribution<float> uv(-1.f, 1.f);
  for (size_t k = 0; k < e.size(); ++k) {
    A.rp[(e[k] >> 32) + 1]++;
    A.ci[k] = (int32_t)(e[k] & 0xffffffffu);
    A.v[k] = uv(g);
  }
  for (int64_t r = 0; r < m; ++r) A.rp[r + 1] += A.rp[r];
  return A;
}

struct Blocked {
  int G = 0, U = 0;
  std::vector<int64_t> bk;   // entry offsets per block (padded to 64U for the 16-bit form)
  std::vector<int32_t> br;   // row offsets per block
  std::vector<int32_t> col;  // variant A
  std::vector<uint16_t> rowl;
  std::vector<float> val;
  std::vector<int32_t> cbase;  // variant B
  std::vector<uint16_t> coff;
  int max_rows = 0;
  int64_t pad = 0;
};

// nnz-balanced row blocks (split rows excluded), entries sorted by (col, row)
static Blocked block_sort(const Csr &A, int G, int U, bool sort_cols, bool pad16, int H = 1) {
  Blocked B;
  B.G = G;
  B.U = U;
  const int64_t m = A.m;
  std::vector<int64_t> kin((size_t)m + 1, 0);  // in-kernel prefix
  for (int64_t r = 0; r < m; ++r) {
    const int64_t d = A.rp[r + 1] - A.rp[r];
    kin[r + 1] = kin[r] + (d > kLong ? 0 : d);
  }
  const int NB = G / H;  // row blocks; workgroup b = (row block b / H, column part b % H)
  B.br.assign((size_t)NB + 1, 0);
  for (int b = 1; b < NB; ++b) {
    const int64_t t = kin[m] * b / NB;
    B.br[b] = (int32_t)(std::lower_bound(kin.begin(), kin.end(), t) - kin.begin());
    B.br[b] = std::max(B.br[b], B.br[b - 1]);
    B.br[b] = std::min<int32_t>(B.br[b], B.br[b - 1] + 65535);
  }
  B.br[NB] = (int32_t)m;
  if (B.br[NB] - B.br[NB - 1] > 65535) { fprintf(stderr, "block too tall\n"); exit(1); }
  const int64_t ncol = m;  // square
  const int64_t C = 64 * U;
  std::vector<std::vector<uint64_t>> ent((size_t)G);
  std::vector<std::thread> th;
  const int nt = 16;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t]() {
      for (int b = t; b < G; b += nt) {
        auto &E = ent[(size_t)b];
        const int rb = b / H, h = b % H;
        const int64_t c0 = ncol * h / H, c1 = ncol * (h + 1) / H;
        for (int32_t r = B.br[rb]; r < B.br[rb + 1]; ++r) {
          if (A.rp[r + 1] - A.rp[r] > kLong) continue;
          for (int64_t k = A.rp[r]; k < A.rp[r + 1]; ++k)
            if (A.ci[k] >= c0 && A.ci[k] < c1)
              E.push_back(((uint64_t)(uint32_t)A.ci[k] << 32) | ((uint64_t)(r - B.br[rb]) << 16) |
                          0);  // value looked up below via (row, col)
        }
        if (sort_cols) std::sort(E.begin(), E.end());
      }
    });
  for (auto &x : th) x.join();
  // values: find (row, col) in row r of A by binary search
  auto find_val = [&](int32_t r, int32_t c) -> float {
    const int32_t *p = std::lower_bound(A.ci.data() + A.rp[r], A.ci.data() + A.rp[r + 1], c);
    return A.v[(size_t)(p - A.ci.data())];
  };
  B.bk.assign((size_t)G + 1, 0);
  for (int b = 0; b < G; ++b) {
    int64_t n = (int64_t)ent[(size_t)b].size();
    if (pad16) {
      // chunks of C entries whose columns span <= 65535: count padded size
      int64_t cnt = 0, i = 0;
      const auto &E = ent[(size_t)b];
      while (i < n) {
        const uint32_t c0 = (uint32_t)(E[(size_t)i] >> 32);
        int64_t j = i;
        while (j < n && j - i < C && (uint32_t)(E[(size_t)j] >> 32) - c0 <= 65535) ++j;
        cnt += C;
        i = j;
      }
      n = cnt;
    }
    B.bk[b + 1] = B.bk[b] + n;
    B.max_rows = std::max(B.max_rows, B.br[b / H + 1] - B.br[b / H]);
  }
  const int64_t tot = B.bk[G];
  B.rowl.assign((size_t)tot, 0);
  B.val.assign((size_t)tot, 0.f);
  if (pad16) {
    B.coff.assign((size_t)tot, 0);
    B.cbase.assign((size_t)(tot / C) + 1, 0);
  } else {
    B.col.assign((size_t)tot, 0);
  }
  th.clear();
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t]() {
      for (int b = t; b < G; b += nt) {
        const auto &E = ent[(size_t)b];
        const int64_t n = (int64_t)E.size();
        int64_t o = B.bk[b];
        if (!pad16) {
          for (int64_t i = 0; i < n; ++i, ++o) {
            const int32_t c = (int32_t)(E[(size_t)i] >> 32);
            const int32_t rl = (int32_t)((E[(size_t)i] >> 16) & 0xffff);
            B.col[(size_t)o] = c;
            B.rowl[(size_t)o] = (uint16_t)rl;
            B.val[(size_t)o] = find_val(B.br[b / H] + rl, c);
          }
        } else {
          int64_t i = 0;
          while (i < n) {
            const uint32_t c0 = (uint32_t)(E[(size_t)i] >> 32);
            B.cbase[(size_t)(o / C)] = (int32_t)c0;
            int64_t j = i;
            while (j < n && j - i < C && (uint32_t)(E[(size_t)j] >> 32) - c0 <= 65535) {
              const int32_t c = (int32_t)(E[(size_t)j] >> 32);
              const int32_t rl = (int32_t)((E[(size_t)j] >> 16) & 0xffff);
              B.coff[(size_t)(o + j - i)] = (uint16_t)(c - (int32_t)c0);
              B.rowl[(size_t)(o + j - i)] = (uint16_t)rl;
              B.val[(size_t)(o + j - i)] = find_val(B.br[b / H] + rl, c);
              ++j;
            }
            // padding: value 0 into the block's row 0 (adds +0.0f)
            o += C;
            i = j;
          }
        }
      }
    });
  for (auto &x : th) x.join();
  B.pad = pad16 ? tot - kin[m] : 0;
  return B;
}

template <typename T>
static T *up(const std::vector<T> &h) {
  T *d = nullptr;
  CK(hipMalloc(&d, std::max<size_t>(h.size(), 1) * sizeof(T)));
  if (!h.empty()) CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char **argv) {
  const int64_t m = argc > 1 ? atoll(argv[1]) : 2000000;
  const int iters = argc > 2 ? atoi(argv[2]) : 50;
  auto t0 = std::chrono::steady_clock::now();
  Csr A = powerlaw(m, 1234);
  const int64_t nnz = (int64_t)A.ci.size();
  int64_t long_nnz = 0, n_long = 0;
  for (int64_t r = 0; r < m; ++r)
    if (A.rp[r + 1] - A.rp[r] > kLong) { long_nnz += A.rp[r + 1] - A.rp[r]; ++n_long; }
  fprintf(stderr, "gen %.1fs m=%lld nnz=%lld split rows %lld (%lld nnz)\n",
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(),
          (long long)m, (long long)nnz, (long long)n_long, (long long)long_nnz);
  std::vector<float> xh((size_t)m);
  std::mt19937 gx(42);
  std::uniform_real_distribution<float> ux(-1.f, 1.f);
  for (auto &v : xh) v = ux(gx);
  std::vector<double> yref((size_t)m, 0.0), mag((size_t)m, 0.0);
  for (int64_t r = 0; r < m; ++r) {
    if (A.rp[r + 1] - A.rp[r] > kLong) continue;
    for (int64_t k = A.rp[r]; k < A.rp[r + 1]; ++k) {
      yref[r] += (double)A.v[k] * xh[(size_t)A.ci[k]];
      mag[r] += fabs((double)A.v[k] * xh[(size_t)A.ci[k]]);
    }
  }
  float *dx = up(xh);
  float *dy = nullptr;
  CK(hipMalloc(&dy, (size_t)m * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double alg = (double)nnz * 8.0 + (double)(m + 1) * 4.0 + 2.0 * 4.0 * (double)m;

  auto run = [&](const char *name, int G, int U, int nth, bool acc64, bool sort_cols, bool pad16) {
    Blocked B = block_sort(A, G, U, sort_cols, pad16);
    int64_t *dbk = up(B.bk);
    int32_t *dbr = up(B.br);
    uint16_t *drl = up(B.rowl);
    float *dv = up(B.val);
    int32_t *dc = pad16 ? nullptr : up(B.col);
    int32_t *dcb = pad16 ? up(B.cbase) : nullptr;
    uint16_t *dco = pad16 ? up(B.coff) : nullptr;
    const size_t lds = (size_t)B.max_rows * (acc64 ? 8 : 4);
    if (lds > 160 * 1024) {
      printf("{\"name\":\"%s\",\"skip\":\"lds %zu\"}\n", name, lds);
      return;
    }
    auto launch = [&]() {
#define L(ACC, UU, NT)                                                                          \
  if (pad16)                                                                                    \
    hipLaunchKernelGGL((csort16_kernel<ACC, UU, NT>), dim3(G), dim3(NT), lds, 0, dbk, dbr, dcb, \
                       dco, drl, dv, dx, dy);                                                   \
  else                                                                                          \
    hipLaunchKernelGGL((csort_kernel<ACC, UU, NT>), dim3(G), dim3(NT), lds, 0, dbk, dbr, dc,    \
                       drl, dv, dx, dy);
      if (acc64) {
        if (U == 4 && nth == 1024) { L(double, 4, 1024) }
        else if (U == 2 && nth == 1024) { L(double, 2, 1024) }
        else if (U == 8 && nth == 1024) { L(double, 8, 1024) }
        else if (U == 4 && nth == 512) { L(double, 4, 512) }
        else if (U == 4 && nth == 256) { L(double, 4, 256) }
      } else {
        if (U == 4 && nth == 1024) { L(float, 4, 1024) }
        else if (U == 2 && nth == 1024) { L(float, 2, 1024) }
        else if (U == 8 && nth == 1024) { L(float, 8, 1024) }
        else if (U == 4 && nth == 512) { L(float, 4, 512) }
        else if (U == 4 && nth == 256) { L(float, 4, 256) }
      }
#undef L
    };
    CK(hipMemset(dy, 0, (size_t)m * 4));
    for (int i = 0; i < 5; ++i) launch();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    std::vector<float> yh((size_t)m);
    CK(hipMemcpy(yh.data(), dy, (size_t)m * 4, hipMemcpyDeviceToHost));
    double maxrel = 0;
    int64_t bad = 0;
    for (int64_t r = 0; r < m; ++r) {
      if (A.rp[r + 1] - A.rp[r] > kLong) continue;
      const double err = fabs((double)yh[r] - yref[r]);
      const double rel = err / (mag[r] + 1e-30);
      maxrel = std::max(maxrel, rel);
      if (err > 1e-5 * mag[r] + 1e-30) ++bad;
    }
    printf("{\"name\":\"%s\",\"G\":%d,\"U\":%d,\"nth\":%d,\"acc64\":%d,\"sorted\":%d,\"pad16\":%d,"
           "\"max_rows\":%d,\"pad\":%lld,\"us\":%.2f,\"alg_gbps\":%.1f,\"frac\":%.4f,\"maxrel\":%.3e,"
           "\"bad\":%lld}\n",
           name, G, U, nth, acc64 ? 1 : 0, sort_cols ? 1 : 0, pad16 ? 1 : 0, B.max_rows,
           (long long)B.pad, us, alg / us * 1e-3, alg / us * 1e-3 / 8000.0, maxrel, (long long)bad);
    fflush(stdout);
    (void)hipFree(dbk); (void)hipFree(dbr); (void)hipFree(drl); (void)hipFree(dv);
    if (dc) (void)hipFree(dc);
    if (dcb) (void)hipFree(dcb);
    if (dco) (void)hipFree(dco);
  };
  // generic variants (fp64 accumulators, padded chunks)
  auto run2 = [&](const char *name, int G, int U, int nth, int pack, bool nt, int diag) {
    Blocked B = block_sort(A, G, U, true, true);
    const int64_t tot = B.bk[G];
    std::vector<uint32_t> pidx((size_t)tot);
    std::vector<uint64_t> aos((size_t)tot);
    for (int64_t k = 0; k < tot; ++k) {
      pidx[(size_t)k] = ((uint32_t)B.rowl[(size_t)k] << 16) | B.coff[(size_t)k];
      uint32_t vb;
      memcpy(&vb, &B.val[(size_t)k], 4);
      aos[(size_t)k] = ((uint64_t)vb << 32) | pidx[(size_t)k];
    }
    int64_t *dbk = up(B.bk);
    int32_t *dbr = up(B.br);
    int32_t *dcb = up(B.cbase);
    uint16_t *dco = pack == 0 ? up(B.coff) : nullptr;
    uint16_t *drl = pack == 0 ? up(B.rowl) : nullptr;
    uint32_t *dpi = pack == 1 ? up(pidx) : nullptr;
    float *dv = pack != 2 ? up(B.val) : nullptr;
    u32x2 *da = nullptr;
    if (pack == 2) da = reinterpret_cast<u32x2 *>(up(aos));
    const size_t lds = (size_t)B.max_rows * 8;
    bool ok = true;
    auto launch = [&]() {
#define G_(UU, NT_, PK, NTL, DG)                                                               \
  if (U == UU && nth == NT_ && pack == PK && nt == NTL && diag == DG) {                        \
    hipLaunchKernelGGL((csortg_kernel<double, UU, NT_, PK, NTL, DG>), dim3(G), dim3(NT_), lds, \
                       0, dbk, dbr, dcb, dco, drl, dpi, dv, da, dx, dy);                       \
    return;                                                                                    \
  }
      G_(4, 1024, 0, false, 0) G_(4, 1024, 1, false, 0) G_(4, 1024, 2, false, 0)
      G_(4, 1024, 2, true, 0) G_(2, 1024, 2, false, 0) G_(8, 1024, 2, false, 0)
      G_(4, 512, 2, false, 0) G_(4, 1024, 2, false, 1) G_(4, 1024, 2, false, 2)
      G_(8, 512, 2, false, 0) G_(4, 256, 2, false, 0)
#undef G_
      ok = false;
    };
    CK(hipMemset(dy, 0, (size_t)m * 4));
    for (int i = 0; i < 5; ++i) launch();
    if (!ok) { printf("{\"name\":\"%s\",\"skip\":\"no instance\"}\n", name); return; }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    std::vector<float> yh((size_t)m);
    CK(hipMemcpy(yh.data(), dy, (size_t)m * 4, hipMemcpyDeviceToHost));
    double maxrel = 0;
    int64_t bad = 0;
    for (int64_t r = 0; r < m; ++r) {
      if (A.rp[r + 1] - A.rp[r] > kLong) continue;
      const double err = fabs((double)yh[r] - yref[r]);
      maxrel = std::max(maxrel, err / (mag[r] + 1e-30));
      if (err > 1e-5 * mag[r] + 1e-30) ++bad;
    }
    printf("{\"name\":\"%s\",\"G\":%d,\"U\":%d,\"nth\":%d,\"pack\":%d,\"nt\":%d,\"diag\":%d,"
           "\"max_rows\":%d,\"pad\":%lld,\"us\":%.2f,\"alg_gbps\":%.1f,\"frac\":%.4f,\"maxrel\":%.3e,"
           "\"bad\":%lld}\n",
           name, G, U, nth, pack, nt ? 1 : 0, diag, B.max_rows, (long long)B.pad, us,
           alg / us * 1e-3, alg / us * 1e-3 / 8000.0, maxrel, (long long)bad);
    fflush(stdout);
    (void)hipFree(dbk); (void)hipFree(dbr); (void)hipFree(dcb);
    if (dco) (void)hipFree(dco);
    if (drl) (void)hipFree(drl);
    if (dpi) (void)hipFree(dpi);
    if (dv) (void)hipFree(dv);
    if (da) (void)hipFree(da);
  };
  auto run3 = [&](const char *name, int G, int U, bool nt, int H, bool acc32 = false) {
    Blocked B = block_sort(A, G, U, true, true, H);
    const int64_t tot = B.bk[G];
    std::vector<uint64_t> aos((size_t)tot);
    for (int64_t k = 0; k < tot; ++k) {
      uint32_t vb;
      memcpy(&vb, &B.val[(size_t)k], 4);
      aos[(size_t)k] = ((uint64_t)vb << 32) | (((uint32_t)B.rowl[(size_t)k] << 16) | B.coff[(size_t)k]);
    }
    int64_t *dbk = up(B.bk);
    int32_t *dbr = up(B.br);
    int32_t *dcb = up(B.cbase);
    u32x2 *da = reinterpret_cast<u32x2 *>(up(aos));
    double *dpart = nullptr;
    CK(hipMalloc(&dpart, (size_t)H * m * 8));
    const size_t lds = (size_t)B.max_rows * (acc32 ? 4 : 8);
    if (lds > 160 * 1024) { printf("{\"name\":\"%s\",\"skip\":\"lds %zu\"}\n", name, lds); return; }
    bool ok = true;
    auto launch = [&]() {
#define H_(UU, NTL, HH, AC)                                                                   \
  if (U == UU && nt == NTL && H == HH && acc32 == (sizeof(AC) == 4)) {                        \
    hipLaunchKernelGGL((csorth_kernel<UU, 1024, NTL, HH, AC>), dim3(G), dim3(1024), lds, 0,   \
                       dbk, dbr, dcb, da, dx, m, dpart);                                      \
    hipLaunchKernelGGL((csort_finish<HH>), dim3((unsigned)((m + 255) / 256)), dim3(256), 0, 0, \
                       m, dpart, dy);                                                         \
    return;                                                                                   \
  }
      H_(16, true, 2, double) H_(16, true, 2, float) H_(16, true, 4, float) H_(8, true, 4, float)
      H_(16, true, 1, double)
#undef H_
      ok = false;
    };
    CK(hipMemset(dy, 0, (size_t)m * 4));
    for (int i = 0; i < 5; ++i) launch();
    if (!ok) { printf("{\"name\":\"%s\",\"skip\":\"no instance\"}\n", name); return; }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    std::vector<float> yh((size_t)m);
    CK(hipMemcpy(yh.data(), dy, (size_t)m * 4, hipMemcpyDeviceToHost));
    double maxrel = 0;
    int64_t bad = 0;
    for (int64_t r = 0; r < m; ++r) {
      if (A.rp[r + 1] - A.rp[r] > kLong) continue;
      const double err = fabs((double)yh[r] - yref[r]);
      maxrel = std::max(maxrel, err / (mag[r] + 1e-30));
      if (err > 1e-5 * mag[r] + 1e-30) ++bad;
    }
    printf("{\"name\":\"%s\",\"G\":%d,\"U\":%d,\"nt\":%d,\"H\":%d,\"max_rows\":%d,\"pad\":%lld,"
           "\"us\":%.2f,\"alg_gbps\":%.1f,\"frac\":%.4f,\"maxrel\":%.3e,\"bad\":%lld}\n",
           name, G, U, nt ? 1 : 0, H, B.max_rows, (long long)B.pad, us, alg / us * 1e-3,
           alg / us * 1e-3 / 8000.0, maxrel, (long long)bad);
    fflush(stdout);
    (void)hipFree(dbk); (void)hipFree(dbr); (void)hipFree(dcb); (void)hipFree(da);
    (void)hipFree(dpart);
  };
  run3("h2_U16_f64", 256, 16, true, 2);
  run3("h2_U16_f32", 256, 16, true, 2, true);
  run3("h4_U16_f32", 256, 16, true, 4, true);
  run3("h4_U8_f32", 256, 8, true, 4, true);
  run3("h1_U16_f64", 256, 16, true, 1);
  return 0;
}
