// gather_probe.hip -- calibration microbenchmark (not product code): what does
// a 64-lane fp32 gather instruction cost the CU's L1 path (TA/TD/TCP) as a
// function of its address pattern?  The column-sorted C5 kernel
// (csrc/csort.hip) spends its time on gathers; r04 cut its modelled
// (quad, 32-byte sector) pairs by 14 % without any change in time
// (profiles/r04/ab_c5_quad_pack.jsonl), so the charging unit is unknown.
//
// Shape = C5's: 256 workgroups x 1024 threads (one per CU); workgroup b works
// in half b % 2 (4 MiB of fp32) of an 8 MiB x, which its XCD's L2 keeps.
// Every wave issues the same number of gather instructions (8 in flight per
// batch, like csort's U); instruction i of a wave starts at a base that
// advances by the pattern's span, so each instruction touches lines the CU
// has not read yet (L2 hits, "sweep", within 2 MiB), or stays inside a 16 KiB window that
// the L1 keeps ("hot").  Lane l of an instruction reads, relative to base:
//   line2   : l                         64 floats: 8 sectors, 2 lines (coalesced)
//   one     : 0                         1 sector
//   quad1   : 8 * (l / 4) + l % 4       16 sectors, each quad in one sector
//   quad2   : 8 * ((l + 2) / 4) + l % 4 17 sectors, each quad across two
//   sector  : 8 * l                     64 sectors (16 lines), one per lane
//   line    : 32 * l                    64 lines, one per lane
//   c5      : sorted columns at 0.19 entries per column (~340-column span,
//             ~34 sectors, as the csort gathers of C5)
// Reported per mode: ms (min of 10) and ns per gather instruction per CU.
// PMC passes over the same binary (tools/gpu_r04w.sh) give the L1 counters.
//
//   hipcc -O3 --offload-arch=gfx950 gather_probe.hip -o gather_probe
//   ./gather_probe [mode ...]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      return 1;                                                             \
    }                                                                       \
  } while (0)

constexpr int kThreads = 1024, kWaves = 16, kBlocks = 256, kBatch = 8;
constexpr long kHalf = 1L << 20;        // fp32 entries per half (4 MiB)
constexpr int kInstr = 2048;            // gather instructions per wave
constexpr int kHotWindow = 4096;        // floats: 16 KiB

enum { LINE2 = 0, ONE, QUAD1, QUAD2, SECTOR, LINE, C5, C5R, SQR, NMODES };
const char *kNames[NMODES] = {"line2", "one", "quad1", "quad2", "sector", "line", "c5", "c5+rec", "sq+rec"};
// c5+rec : the c5 gather after a per-lane 8-byte record load (csort's entry
//          stream, 64 entries per instruction; records from a separate buffer)
// sq+rec : "sector quads": quad q of an instruction holds the entries of one
//          32-byte sector (1-4, pattern averaging 1.9 as C5's ~1.9 entries
//          per touched sector), the other lanes predicated off; active lanes
//          load their 8-byte record (compact) and gather inside the quad's sector

// offset of lane l (relative to the instruction base) and the span (floats)
// the base advances by per instruction
template <int MODE>
__device__ __forceinline__ int lane_off(int l) {
  if constexpr (MODE == LINE2) return l;
  if constexpr (MODE == ONE) return 0;
  if constexpr (MODE == QUAD1) return 8 * (l >> 2) + (l & 3);
  if constexpr (MODE == QUAD2) return 8 * ((l + 2) >> 2) + (l & 3);
  if constexpr (MODE == SECTOR) return 8 * l;
  if constexpr (MODE == LINE) return 32 * l;
  if constexpr (MODE == SQR) return 16 * (l >> 2) + (l & 3);  // quad q: sector 2q (every other one touched)
  return (l * 16) / 3;  // C5: 64 sorted entries over ~340 columns
}
template <int MODE>
constexpr int span() {
  return MODE == LINE2 ? 64 : MODE == ONE ? 8 : MODE == QUAD1 ? 128 : MODE == QUAD2 ? 136
         : MODE == SECTOR ? 512 : MODE == LINE ? 2048 : MODE == SQR ? 256 : 344;
}

template <int MODE, bool HOT>
__global__ __launch_bounds__(kThreads) void probe(const float *__restrict__ x, float *__restrict__ out,
                                                  long window, long limit,
                                                  const uint2 *__restrict__ rec, long rlimit) {
  const int b = blockIdx.x, wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float *xh = x + (long)(b & 1) * kHalf;
  constexpr long S = span<MODE>();
  const int off = lane_off<MODE>(lane);
  float acc = 0.f;
  // wave w's instruction i: base = ((i * kWaves + w) * S) within the half
  // (the 16 waves sweep the half together, as csort's waves take chunk c + 16)
  for (int i0 = 0; i0 < kInstr; i0 += kBatch) {
    float v[kBatch];
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      const long i = i0 + u;
      long base = ((i * kWaves + wid) * S);
      // (window / limit are power-of-two masks passed as kernel arguments: a
      // compile-time modulus lets the compiler merge repeated loads, a
      // runtime 64-bit modulus costs more VALU than the cheap patterns'
      // gathers themselves)
      base = HOT ? (base & window) : (base & limit);
      if constexpr (MODE == C5R || MODE == SQR) {
        // the record stream: 64 (c5+rec) or the active lanes' (sq+rec) 8-byte
        // records of this instruction, contiguous
        constexpr int kCnt[16] = {2, 1, 3, 2, 1, 2, 4, 1, 2, 2, 1, 3, 1, 2, 2, 2};  // mean 1.94
        const int q = lane >> 2, sub = lane & 3;
        int pre = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) pre += t < q ? kCnt[t] : 0;
        const bool act = MODE == C5R || sub < kCnt[q];
        const long per = MODE == C5R ? 64 : 31;
        const long ridx = (((i * kWaves + wid) * per) & (rlimit)) + (MODE == C5R ? lane : pre + sub);
        uint2 r = act ? rec[ridx] : make_uint2(0, 0);
        const float xv = act ? xh[base + off + (r.x & 1)] : 0.f;
        v[u] = xv * __uint_as_float(r.y | 0x3f800000u);
      } else {
        v[u] = xh[base + off];
      }
    }
#pragma unroll
    for (int u = 0; u < kBatch; ++u) acc += v[u];
  }
  if (acc == 123.456f) out[b * kThreads + threadIdx.x] = acc;  // keep it live
}

static uint2 *g_rec = nullptr;
constexpr long kRec = 1L << 24;  // records (128 MiB): the stream comes from HBM

template <int MODE, bool HOT>
float run(const float *x, float *out, hipStream_t st) {
  hipEvent_t a, z;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&z);
  float best = 1e30f;
  for (int it = 0; it < 12; ++it) {
    (void)hipEventRecord(a, st);
    hipLaunchKernelGGL((probe<MODE, HOT>), dim3(kBlocks), dim3(kThreads), 0, st, x, out,
                       (long)kHotWindow - 1, kHalf / 2 - 1, g_rec, kRec / 2 - 1);
    (void)hipEventRecord(z, st);
    (void)hipEventSynchronize(z);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, z);
    if (it >= 2) best = std::min(best, ms);
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(z);
  return best;
}

template <int MODE>
void report(const float *x, float *out, hipStream_t st) {
  const double per_cu = (double)kWaves * kInstr;  // gather instructions per CU
  for (int hot = 0; hot < 2; ++hot) {
    const float ms = hot ? run<MODE, true>(x, out, st) : run<MODE, false>(x, out, st);
    printf("{\"probe\": \"gather\", \"mode\": \"%s\", \"where\": \"%s\", \"ms\": %.4f, "
           "\"ns_per_instr_per_cu\": %.4f, \"span_floats\": %d}\n",
           kNames[MODE], hot ? "hot" : "sweep", ms, ms * 1e6 / per_cu, span<MODE>());
  }
}

int main(int argc, char **argv) {
  float *x, *out;
  CK(hipMalloc(&x, 2 * kHalf * sizeof(float)));
  CK(hipMalloc(&out, kBlocks * kThreads * sizeof(float)));
  std::vector<float> h(2 * kHalf, 1.0f);
  CK(hipMemcpy(x, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
  CK(hipMalloc(&g_rec, kRec * sizeof(uint2)));
  CK(hipMemset(g_rec, 0, kRec * sizeof(uint2)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  auto want = [&](const char *n) {
    if (argc < 2) return true;
    for (int i = 1; i < argc; ++i)
      if (!strcmp(argv[i], n)) return true;
    return false;
  };
  if (want("line2")) report<LINE2>(x, out, st);
  if (want("one")) report<ONE>(x, out, st);
  if (want("quad1")) report<QUAD1>(x, out, st);
  if (want("quad2")) report<QUAD2>(x, out, st);
  if (want("sector")) report<SECTOR>(x, out, st);
  if (want("line")) report<LINE>(x, out, st);
  if (want("c5")) report<C5>(x, out, st);
  if (want("c5+rec")) report<C5R>(x, out, st);
  if (want("sq+rec")) report<SQR>(x, out, st);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
