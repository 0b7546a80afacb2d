// Internal interfaces shared by the host runtime (hspmv_runtime.h units) and the
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
  // 16-bit column offsets (row kernels): col[k] = cbase[k >> kC16Shift] + col16[k]
  // plus bit 16+p of (col - base) in plane p: bit k&63 of cplanes[p*cplane_words + k/64]
  const uint16_t *col16 = nullptr;
  const int32_t *cbase = nullptr;
  const uint64_t *cplanes = nullptr;
  int32_t n_cplanes = 0, cplane_words = 0;
  // c16_mode 2 (STREAM only): col[k] = cbase[g] + col16[k] with g = the
  // nonzero's 64-row group, when every group's columns span < 65536
  int32_t c16_mode = 1;
  int32_t col_span_bits = 0;  // bits of the widest 256-nonzero block's column span (0 = unknown)
  // planner hints from the host tables: STREAM x windows / block x
  // dictionaries were built for this shard
  bool has_xwin = false, has_xdict = false;
  bool has_xdict_tasks = false;  // x dictionaries built for packed CSR3 tasks
  int32_t n_slabs = 1;        // x slabs: the row kernel's passes (each sees ~nnz / n_slabs)
  int32_t task_waves = 4;     // CSR3 wave tasks per workgroup: 4 (8 with 8-task dictionary
                              // blocks); the SSR plan: ssr_waves() per super-super-row
  bool has_csort = false;     // column-sorted row blocks were built (irregular gathers)
  bool slab_stream = false;   // x-slab passes with CSR-3 tasks: AUTO runs STREAM (slab_kernel_rule)
  int32_t serial_len = 0;     // median length of the rows summed serially (<= kSerialMax), 0 = none
};

// Planner choices of one handle.  The first block mirrors hspmv_options
// (include/hspmv.h; 0 = the library's choice); the second holds A/B-only
// knobs that product builds never change: only a diagnostic build
// (make diag-env: -DHSPMV_ENV_KNOBS) reads them, and the public fields, from
// HSPMV_* environment variables (tuning_from_env, hspmv_options.cpp), so a
// production handle's kernel choice cannot move with the environment.
struct Tuning {
  int csr3_plan = 0;        // 0/1 aligned 64-row tasks, 2 packed super-rows, 3 workgroup per SSR
  int task_nnz = 0;         // wave-task nonzero budget (0: 2048)
  int x_windows = 0;        // -1 off, 0 auto
  int x_dict = 0;           // -1 off, 0 auto, 1 whenever it fits
  int x_dict_cap = 0;       // LDS bytes per dictionary block (0: 20 KiB; <= 64 KiB)
  int x_slabs = 0;          // -1 off, 0 auto, B > 0 forced
  int col16_group = 0;      // -1 off, 0 auto, 1 whenever it fits
  int csort = 0;            // -1 off, 0 auto, 1 whenever it can be built
  int csort_parts = 0;      // 0 auto, 1/2/4
  int csort_u = 0;          // 0 auto, 4/8/16
  int stream_waves = 0;     // 0 auto, 1/2/4
  int deterministic = 0;    // 1: ordered row kernels (omp_spmv's order); 2: reproducible (fixed-point csort allowed)
  int serial_max = 0;       // A/B: the row kernels' serial bound (0: kSerialMax)
  int placement_trials = 0; // 0/1 off, K <= 8 array sets
  int ssr_w = 0;            // SSR plan waves per workgroup (0: ssr_waves(); A/B)
  int ssr_align = -1;       // SSR plan wave cut: 2 row-granular nnz balance (-1: default), 0 super-rows, 1 aligned pieces
  // A/B only (diagnostic builds)
  int contig = 0;           // hipDeviceMallocContiguous allocations
  int xd_waves = 0;         // packed CSR3 tasks per dictionary block (0: 4; 8)
  int xd_blocks_per_cu = 0; // CSR3 dictionary blocks sized for this many per CU (0: 6; -1: no cuts)
  double xslab_bytes = 0;   // x bytes per slab (0: 2 MiB)
  int csort_nt = -1, csort_pf = -1;      // -1: the library's choice
  int csort_blocks_per_cu = 0;           // row blocks per CU and part (0: 1)
  int csort_slot32 = -1;                 // fp32 LDS row slots (fp32 data)
  int csort_wide = -1;                   // 16-byte entry loads (interleaved layout)
  int csort_lds_cap = 0;                 // LDS bytes per workgroup for the row slots (0: all)
  int csort_seg = -1;                    // segmented chunks: 0 never, 2 always (-1: by conflicts)
  int csort_seg_extra = 0;               // serialised same-slot lanes that flag a chunk (0: default)
  int csort_trace = 0;                   // per-workgroup timestamps (hspmv_diag_csort_trace)
  int csort_long = 0;                    // rows above this many nonzeros are sliced (0: kLongRow)
  int csort_balance = 0;                 // -1: equal-width column parts, nnz-balanced rows (r03)
  int csort_fin_rows = 0;                // rows per finishing-pass thread (0: default; 1, 2, 4)
  int csort_dyn = -1;                    // chunks claimed from an LDS queue (-1: the library's choice)
  double csort_sweep_w = 0;              // column-part cost of a column per row block (0: kSweepPerRowBlock)
  double csort_slack = 0;                // widest column part / (n / H) when balancing (0: kPartSlack)
  int csort_part32 = -1;                 // fp32 row partials over fp64 slots (fp32 data; -1: on, 0 off)
  int lds_pad = -1;                      // STREAM padded product buffers (-1: by row length, 0 off, 1 on)
  int pf = -1, y_nt = -1, nt = -1;       // row kernels: prefetch, nt y stores, nt col/val
  int dyn_lds = 0;
};

constexpr int kC16Shift = 8;  // 256 nonzeros per column-base block
constexpr int kXWin = 256;    // largest LDS-staged x window of a row group (entries)

enum Kernel : int { kAuto = 0, kVector = 1, kStream = 2, kCsr3 = 3, kCsort = 4 };

// Rows longer than this many nonzeros ("split rows") are cut into chunks of
// kLongChunk nonzeros, each summed by its own workgroup, and the chunk sums
// are added per row by a second small kernel (deterministic order).
constexpr int32_t kLongRow = 4096;
// Rows of up to this many nonzeros are summed serially (omp_spmv's order) by
// one lane in the row kernels; longer ones cooperatively (fixed DPP trees) --
// unless DevPlan.serial_max raises the bound (deterministic = 3).
constexpr int32_t kSerialMax = 40;
// fp32 data: 56 -- rows of 41-56 nonzeros summed serially ran 15-27 % faster
// than in the cooperative trees (d41 113.7 -> 83.0 us, d48 106.3 -> 90.2 at
// 48, profiles/r06s3/ab_serial48_f32.jsonl; d50 104.7 -> 81.8, d52 100.4 ->
// 80.4, d56 94.8 -> 80.2 at 56, r06s5), every other shape flat; 64 lost on
// d64 (+31 %, r06s2).  fp64 rows of 48 serially met in LDS banks (d48 +41 %,
// r06s2), so fp64 keeps 40.
constexpr int32_t kSerialMaxF32 = 56;
constexpr int32_t kLongChunk = 4096;

// Column-sorted row blocks (csort.hip): workgroup b works on column part
// b % H (a fixed slice of x) and walks chunks [blk_c[b], blk_c[b+1]) of 64*u
// entries in column order; its rows are [blk_r[2b], blk_r[2b+1]) (each part
// has its own row partition) and its long-row slices vslice[blk_v[b] ..
// blk_v[b+1]).  Built by build_csort (hspmv_csort_build.cpp).
constexpr int kCsortThreads = 1024;
constexpr int kCsortMaxLds = 160 * 1024;
// Diagnostic trace of a csort launch (DevCsort.trace, HSPMV_CSORT_TRACE=1):
// per workgroup kCsortTraceSlots u64 = {start, end, XCC_ID | HW_ID << 32,
// after the slot-zeroing barrier, then per wave: its end (after its last
// chunk), then per wave: the chunks it ran} (s_memrealtime, 100 MHz).
constexpr int kCsortTraceSlots = 4 + 2 * (kCsortThreads / 64);
// Fixed-point slots: every product rounds to an integer below 2^kCsortFixBits
// (values scaled to |v'| < 1 per row, x to |x'| < 2^kCsortFixBits), so a slot
// of <= 4096 products stays below 2^62; the pre-pass runs kCsortXexpBlocks
// workgroups at most.
constexpr int kCsortFixBits = 50;
constexpr int kCsortXexpBlocks = 256;
constexpr int64_t kCsortXexpChunk = 8192;  // x entries per pre-pass block and chunk
constexpr int32_t kCsortXexpNonFinite = 0x7fffffff;
struct DevCsort {
  int32_t n_wg = 0, H = 1, u = 16, direct = 0, n_long = 0;
  bool nontemporal = true;
  bool prefetch = false;  // next chunk's entries loaded during this chunk's gathers
  bool slot32 = false;    // fp32 LDS row slots and partials (fp32 data; A/B)
  bool wide = false;      // 16-byte entry loads (host-interleaved layout)
  bool dyn = false;       // waves claim the workgroup's chunks from an LDS queue
  bool part32 = false;    // fp32 row partials over fp64 slots (fp32 data; the default)
  // Reproducible (fixed-point) row sums (hspmv_options.deterministic = 2):
  // the slots are int64 sums of each product rounded to an integer at scale
  // 2^(kCsortFixBits - xexp - rexp[row]); xexp = the max exponent of |x|,
  // found per SpMV by hspmv_csort_xexp into xexp_part[n_xexp] (csort.hip)
  bool fixed = false;
  const int16_t *rexp = nullptr;  // per row: the exponent its values were scaled by (2^rexp)
  const int16_t *sexp = nullptr;  // per long-row slice: its row's rexp
  int32_t *xexp_part = nullptr;   // per pre-pass block: max frexp exponent of |x| (INT32_MAX: non-finite)
  int32_t n_xexp = 0;
  int64_t n_x = 0;                // x entries the pre-pass reads
  int32_t fin_rows = 0;   // rows per finishing-pass thread (0: 4, or the most m allows)
  int64_t m = 0;
  int32_t lds_bytes = 0;
  const int32_t *blk_c = nullptr, *blk_r = nullptr, *blk_v = nullptr, *vslice = nullptr;
  int32_t row_blocks = 0;  // blocks per column part (the parts' own row partitions)
  unsigned long long *trace = nullptr;  // diagnostic builds: per-workgroup {start, end, hw_id} (s_memrealtime)
  const int32_t *cbase = nullptr;
  const void *ent = nullptr;  // fp32: {idx, val} records; fp64: idx
  const void *val = nullptr;  // fp64 values (nullptr for fp32)
  void *part = nullptr, *spart = nullptr;  // partial sums in the slot type
  const uint32_t *long_mask = nullptr;
  const int32_t *long_row = nullptr, *long_cs = nullptr;
};

// Device-side tables the host planner builds once per shard (all optional).
struct DevPlan {
  // CSR-3: wave task t covers rows [task_start[t], task_start[t+1]);
  // either super-rows packed into <= 64-row tasks (default), or
  // waves_per_block tasks per super-super-row, nnz-balanced on super-row
  // boundaries (HSPMV_CSR3_PLAN=ssr).
  const int32_t *task_start = nullptr;
  int32_t n_tasks = 0;
  // 1: a task's 64-row groups end on multiples of 64 (its first group may be
  // shorter) -- the SSR plan's aligned cut (ssr_tasks_aligned); 0: groups of
  // 64 rows from the task's first row
  int32_t task_align = 0;
  // split rows
  int32_t long_t = 0x7fffffff;  // rows with more nonzeros are split rows
  int32_t serial_max = kSerialMax;  // rows up to this length are summed serially (fp32: kSerialMaxF32)
  int32_t n_long = 0, n_chunks = 0;
  bool long_serial = false;  // split rows summed in order by hspmv_long_serial (deterministic = 3)
  // ... on a stream of their own, forked from and joined back into the
  // launch stream, so they run beside the row kernel instead of after it
  hipStream_t long_stream = nullptr;
  hipEvent_t long_fork = nullptr, long_join = nullptr;
  const int32_t *long_row = nullptr;    // n_long row ids (shard-local)
  const int32_t *long_cstart = nullptr; // n_long+1, chunk ranges per split row
  const int32_t *chunk_k = nullptr;     // 2*n_chunks: [k0, k1) per chunk
  void *partials = nullptr;             // n_chunks partial sums (dtype)
  // x windows per row group (STREAM: 64-row groups; CSR3: packed tasks):
  // {lo, w} (int32), w = 0 when the group's columns span more than kXWin
  // entries (then it gathers from global x)
  const void *xwin = nullptr;
  // Block x dictionaries (STREAM with one group per wave: 256-row blocks;
  // CSR3: blocks of four packed tasks): xd_blk[b], xd_blk[b+1] bound block
  // b's {x_start, lds_off} run records in xd_runs (int2), the last a sentinel
  // {0, entries}; col16 then holds each nonzero's position in the staged xs.
  // xd_lds_bytes = the largest block's dictionary (dynamic LDS per block).
  const int32_t *xd_blk = nullptr;
  const void *xd_runs = nullptr;
  int32_t xd_lds_bytes = 0;
  // x slabs (irregular gathers, x larger than an XCD's L2): the columns are
  // cut into n_slabs equal ranges and the row kernel runs
  // once per slab over a slab-major copy of the matrix -- pass b reads rows
  // [slab_rp[b*(m+1) + r], slab_rp[b*(m+1) + r + 1]) of slab_col/slab_val,
  // so its gathers stay inside one L2-sized slice of x.  Split rows have
  // empty slab segments (the split-row kernels sum them from the CSR).
  int32_t n_slabs = 0;
  const int32_t *slab_rp = nullptr;
  const int32_t *slab_col = nullptr;
  const void *slab_val = nullptr;
  DevCsort cs;  // kCsort
};

struct LaunchPlan {
  int kernel = kStream;
  int lanes = 64;          // VECTOR: lanes per row; STREAM/CSR3: 64 rows per wave pass
  int waves_per_block = 4; // CSR3: waves per super-super-row workgroup
  int u = 8;               // STREAM/CSR3: elements per lane per LDS chunk
  bool nontemporal = false;
  bool prefetch = false;   // STREAM/CSR3: next chunk's col/val issued early
  bool y_nt = false;       // STREAM/CSR3: nontemporal y stores
  int32_t dyn_lds = 0;     // extra dynamic LDS per block (occupancy experiments)
  int32_t xcd_chunk = 1;   // blocks per XCD turn (1 = dispatch order; see xcd_chunk_remap)
  int32_t groups = 1;      // STREAM: 64-row groups per wave (next group's rp prefetched)
  int32_t carry = 0;       // STREAM/CSR3: rows start from y (x-slab passes after the first)
  bool lds_pad = false;     // STREAM: bank-padded product buffers (spmv_device.cuh lds_ix)
  int64_t blocks = 0;
};

// Waves of the workgroup-per-super-super-row CSR-3 plan: ~64 rows per wave
// (one lane per row in the ordered sums), from the mean rows per SSR.
inline int ssr_waves(double rows_per_ssr) {
  const double w = rows_per_ssr / 64.0;
  return w >= 6.0 ? 8 : (w >= 3.0 ? 4 : (w >= 1.5 ? 2 : 1));
}

// Chooses kernel / lanes / block shape for a shard (host-side heuristic).
// rows_per_ssr: mean rows per super-super-row (CSR-3 workgroup-per-SSR plan);
// packed_tasks > 0: CSR-3 tasks packed from super-rows (4 per workgroup).
LaunchPlan plan_launch(const DevCSR &A, int dtype, unsigned flags, double rows_per_ssr,
                       int64_t packed_tasks, const Tuning &t);

// STREAM / CSR3 row kernels (stream_f32.hip / stream_f64.hip).
hipError_t launch_rows_f32(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p,
                           const float *x, float *y, hipStream_t st);
hipError_t launch_rows_f64(const DevCSR &A, const DevPlan &dp, const LaunchPlan &p,
                           const double *x, double *y, hipStream_t st);

// Column-sorted row-block kernel + its finishing pass (csort.hip).
hipError_t launch_csort(const DevCsort &c, int dtype, const void *x, void *y, hipStream_t st);

// Enqueues one y = A*x (main kernel + split-row kernels when present).
hipError_t launch_spmv(const DevCSR &A, const DevPlan &dp, int dtype, const LaunchPlan &plan,
                       const void *x, void *y, hipStream_t stream);

}  // namespace hspmv
