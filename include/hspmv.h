/*
 * hspmv.h -- C ABI of the MI355X-native CSR / CSR-3 SpMV library
 * (libhspmv.so, built from heterogeneous-spmv_amd/csrc/).
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * has no library: its "boundary" is three things, each replaced here
 * (SURVEY.md §8b):
 *
 *  1. Kernel ABI  -- cuda_spmv (cuda-spmv-csr/spmv.cu:117-119) and
 *     cuSpMV_3 / cuSpMV_3_vec / cuSpMV_2 (cuda-spmv-csrk/hip/csrk.cuh:25-47),
 *     all taking raw device pointers.  Replaced by hspmv_spmv() on a handle
 *     that owns (or borrows, HSPMV_FLAG_DEVICE_PTRS) the device arrays.
 *  2. Host library -- CSRk_Graph(nRows, nCols, nnz, rVec, cVec, val, ...,
 *     k, supRowSizes) + putInCSRkFormat() / setX() / setY() / getY()
 *     (cuda-spmv-csrk/hip/csrk.cuh:321-353, csrk.cu:92-113, 531-641, 875-900).
 *     Replaced by hspmv_create() (+ hspmv_build_csr3_maps()), hspmv_set_x(),
 *     hspmv_get_y().
 *  3. CLI/stdout contract -- spmv-csr/spmv.c:116-225 and
 *     cuda-spmv-csrk/hip/spmv*.cu; reproduced by the spmv-csr / spmv-csrk
 *     executables built on top of this header.
 *
 * Conventions: every int-returning function returns 0 on success and a
 * negative HSPMV_E* code on failure (the reference ignores every hip* status;
 * SURVEY.md §5).  hspmv_last_error() returns a thread-local message.  No C++
 * exceptions cross this boundary.  Indices are 0-based int32 (readers accept
 * 1-based files and rebase them).  Values are fp32 or fp64 (hspmv_dtype).
 */
#ifndef HSPMV_H
#define HSPMV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history.  0.2: hspmv_options, info.deterministic.  0.3: info.rccl_version
 * / csort chunks, hspmv_xdict_plan_ex, hspmv_rccl_version, hspmv_read_mtx,
 * hspmv_rcm_reorder -- and two changes a 0.2 binary could not see
 * (hspmv_xdict_plan's 3rd argument became kernel flags; hspmv_get_info's
 * layout shrank).  1.0 declares that break: the library is libhspmv.so.1
 * (SONAME), so a binary built against 0.x fails to load instead of
 * misreading arguments; hspmv_get_info fills the whole 1.0 hspmv_info.
 * Within a major, structs only grow at the end (hspmv_options.struct_size,
 * hspmv_get_info_sized) and signatures never change. */
#define HSPMV_VERSION_MAJOR 1
#define HSPMV_VERSION_MINOR 1
/* 1.1: hspmv_options.deterministic = 2 (HSPMV_DETERMINISTIC_REPRODUCIBLE)
 * and 3 (HSPMV_DETERMINISTIC_SERIAL), hspmv_info.csort_fixed_point /
 * serial_order / csort_part_begin; hspmv_get_info frozen at the 1.0 layout
 * (HSPMV_INFO_SIZE_1_0). */

/* ---------------------------------------------------------------- status */
#define HSPMV_OK 0
#define HSPMV_E_INVALID (-1)   /* bad argument / malformed matrix          */
#define HSPMV_E_IO (-2)        /* file cannot be opened / parsed           */
#define HSPMV_E_NOMEM (-3)     /* host or device allocation failed         */
#define HSPMV_E_HIP (-4)       /* HIP runtime error                        */
#define HSPMV_E_RCCL (-5)      /* RCCL error                               */
#define HSPMV_E_NODEV (-6)     /* no / not enough HIP devices              */
#define HSPMV_E_STATE (-7)     /* call order violated (e.g. run before x)  */

/* ---------------------------------------------------------------- types */
typedef enum { HSPMV_F32 = 0, HSPMV_F64 = 1 } hspmv_dtype;

/* A CSR matrix.  Borrowed: hspmv_create copies host arrays (the caller may
 * free them afterwards).  With HSPMV_FLAG_DEVICE_PTRS the handle REFERENCES
 * the caller's device arrays: they must stay allocated and unchanged for the
 * handle's lifetime -- the row kernels read row_ptr / col_idx / val on every
 * SpMV, and the derived tables built at creation (16-bit columns, x
 * dictionaries, x slabs, column-sorted blocks) are snapshots of col_idx and
 * val, so an in-place update would be used partly or not at all.  Re-create
 * the handle after changing the matrix. */
typedef struct {
  int64_t m, n, nnz;
  const int32_t *row_ptr; /* m+1 entries, row_ptr[0] == 0                */
  const int32_t *col_idx; /* nnz entries, 0 <= col < n                   */
  const void *val;        /* nnz entries of dtype                        */
  int32_t dtype;          /* hspmv_dtype                                 */
} hspmv_csr;

/* CSR-3 multilevel maps (A12/A13 in SURVEY.md §8a):
 * super-super-row s covers super-rows outer[s] .. outer[s+1]-1,
 * super-row r covers rows inner[r] .. inner[r+1]-1.
 * Same meaning as mapCoarseToFinerRows[2] / [1] of the reference
 * (csrk.cu:1614, .csr3 writer spmv-auto.cpp:38-62). */
typedef struct {
  int64_t n_ssr, n_sr;
  const int32_t *outer; /* n_ssr+1 */
  const int32_t *inner; /* n_sr+1  */
} hspmv_csr3_maps;

/* Owned buffers returned by the readers / builders; free with the matching
 * hspmv_free_* call. */
typedef struct {
  int64_t m, n, nnz;
  int32_t *row_ptr;
  int32_t *col_idx;
  void *val;
  int32_t dtype;
  int32_t index_base; /* base found in the file (0 or 1); arrays are 0-based */
} hspmv_csr_buf;

typedef struct {
  int64_t n_ssr, n_sr;
  int32_t *outer;
  int32_t *inner;
} hspmv_csr3_buf;

/* Timing of hspmv_run: the reference protocol (5 warm-ups, N timed runs,
 * min/max/avg; spmv-csr/spmv.c:164-185, hip/spmv-auto-mi100.cu:200-240).
 * t_* are device times from HIP events around each SpMV (max over GPUs);
 * wall_* are host steady_clock times around launch + synchronize, which is
 * what the reference measures. */
typedef struct {
  double t_min, t_max, t_avg;
  double wall_min, wall_max, wall_avg;
  double gflops;   /* 2*nnz / t_min * 1e-9                                 */
  double gbps_alg; /* hspmv_alg_bytes() / t_min * 1e-9                     */
  int32_t iters;
  int32_t num_gpus;
} hspmv_timing;

/* What a handle decided (kernel, launch shape, bytes). */
typedef struct {
  int32_t kernel;     /* HSPMV_KERNEL_* actually used                      */
  int32_t lanes;      /* lanes per row (VECTOR) / rows per wave task       */
  int32_t waves_per_block;
  int32_t num_gpus;
  int64_t blocks;     /* grid size of the launch (GPU 0)                   */
  double alg_bytes;   /* algorithmic bytes per SpMV        */
  double flops;       /* 2 * nnz                                           */
  int64_t device_bytes; /* device memory held by the handle (all GPUs)     */
  int32_t chunk_u;    /* STREAM/CSR3 elements per lane per LDS chunk        */
  int32_t n_split_rows; /* rows summed by the split-row kernels (GPU 0)     */
  int32_t xcd_remap;  /* blocks per XCD turn (1 = dispatch order)          */
  int32_t groups_per_wave; /* STREAM: 64-row groups one wave walks        */
  int64_t x_entries;  /* distinct columns referenced = x entries one SpMV
                         must read (summed over GPUs); alg_bytes uses it    */
  double format_bytes; /* bytes the device format actually moves per SpMV
                          (< alg_bytes with 16-bit column offsets)          */
  int32_t col16;      /* 0 = 32-bit columns; 1 + p = 16-bit column offsets
                         plus p high-bit planes (see HSPMV_FLAG_NO_COL16)   */
  int32_t wave_tasks; /* CSR3: wave tasks of the launch (GPU 0); 0 otherwise */
  int32_t x_windows;  /* STREAM/CSR3: 1 = row groups whose columns span
                         <= 256 entries gather from an LDS copy of that x
                         window; 0 = every gather from global x (GPU 0)     */
  int32_t x_dict;     /* 1 = block x dictionaries: each workgroup stages the
                         x runs its rows reference in LDS and the column
                         stream holds 16-bit positions in it (GPU 0)        */
  int64_t x_dict_entries; /* x entries staged per SpMV (all GPUs; 0 = none) */
  int32_t x_slabs;    /* STREAM/CSR3: 0, or the number of column slabs the
                         row kernel runs over, one pass each, so irregular
                         gathers stay in an L2-sized slice of x (GPU 0)     */
  int32_t col16_group; /* 1 = the 16-bit column offsets are relative to one
                          base per 64-row STREAM group or packed CSR3 task
                          (every one spans < 65536 columns); 0 = per
                          256-nonzero blocks or none                        */
  int32_t csort_parts; /* CSORT: column parts H of the row blocks (0 = the
                          handle does not use the column-sorted kernel)     */
  int32_t placement_trials; /* array sets timed at creation (0 = none: see
                               hspmv_options.placement_trials)             */
  int32_t placement_pick;   /* the set kept (0 = the first allocation)      */
  double placement_us[8];   /* each set's mean SpMV time at creation, us    */
  /* since 0.2 */
  int32_t deterministic;    /* 1: y is bit-identical run to run (every kernel
                               but CSORT with fp64 slots, whose LDS row sums
                               add in atomic order: fp32 y may differ in the
                               last bit where an fp64 sum sits at an fp32
                               rounding tie, fp64 y in the last bits of rows
                               it sums; CSORT with fixed-point slots is 1)  */
  int32_t csr3_plan;        /* CSR3 kernel: the HSPMV_CSR3_PLAN_* it runs;
                               0 for the other kernels                      */
  int32_t csort_slot_bytes; /* CSORT: LDS row-slot width (8 = fp64 sums)    */
  int32_t csort_row_blocks; /* CSORT: row blocks per column part (each part
                               has its own nnz-balanced row partition)     */
  /* since 0.3 */
  int32_t rccl_version;     /* ncclGetVersion() of the RCCL this process
                               resolved (librccl.so.1 is one SONAME for the
                               ROCm and the PyTorch copy: the first loaded
                               wins), e.g. 22703 = 2.27.3                   */
  int32_t reserved0;
  int64_t csort_chunks;     /* CSORT: 64*U-entry chunks of the launch       */
  int64_t csort_seg_chunks; /* CSORT: of those, chunks stored slot-sorted
                               (crowded rows summed by a segmented scan)   */
  /* since 1.0 */
  int32_t slab_kernel_rule; /* x-slab handles that have CSR-3 tasks (the
                               AUTO kernel): 1 = CSR3 tasks, since heavy
                               64-row groups (> 2048 nonzeros) hold >= 1/8
                               of the nonzeros; 2 = STREAM groups (balanced
                               groups); 0 = the rule did not apply          */
  int32_t lds_pad;          /* STREAM: 1 = bank-padded LDS product buffers
                               (the typical row of <= 40 nonzeros is a
                               multiple of 16 LDS words long)              */
  double heavy_group_frac;  /* the share of nonzeros in heavy 64-row groups
                               the rule read (0 when it did not apply)     */
  /* since 1.1 (hspmv_get_info_sized only) */
  int32_t csort_fixed_point; /* CSORT: 1 = reproducible fixed-point row sums
                                (hspmv_options.deterministic = 2)           */
  int32_t serial_order;     /* 1: every row is summed in omp_spmv's order
                                (hspmv_options.deterministic = 3): y is bit-
                                identical to spmv-csr/spmv.c:92-114's loop  */
  int64_t csort_part_begin[4]; /* CSORT (GPU 0): first column of column part
                                  h (h < csort_parts; part h ends where h + 1
                                  begins, the last at n); 0 past the parts  */
} hspmv_info;

typedef struct hspmv_handle hspmv_handle;

/* ---------------------------------------------------------------- flags */
#define HSPMV_KERNEL_AUTO 0u   /* the planner's pick by shape: STREAM or
                                  CSR3 tasks (CSR3 over maps when given),
                                  CSORT for irregular gathers; the choice
                                  is in hspmv_info.kernel                 */
#define HSPMV_KERNEL_VECTOR 1u /* L lanes (sub-wave) per row, shuffle sum  */
#define HSPMV_KERNEL_STREAM 2u /* wave per 64-row group, LDS-staged,
                                  ordered per-row sums (bit-exact vs CPU)  */
#define HSPMV_KERNEL_CSR3 3u   /* wave tasks planned from the CSR-3 maps,
                                  4 per workgroup (hspmv_options.csr3_plan:
                                  64-row aligned tasks, super-rows packed
                                  into <= 64-row tasks, or one workgroup
                                  per super-super-row)                     */
#define HSPMV_KERNEL_CSORT 4u  /* column-sorted row blocks: each workgroup
                                  walks its rows' nonzeros in column order,
                                  fp64 LDS row sums (irregular gathers).
                                  NOT bitwise vs omp_spmv and NOT bit-
                                  identical run to run: the sums add in
                                  LDS-atomic order (csort.hip,
                                  hspmv_info.deterministic) -- unless
                                  hspmv_options.deterministic = 2, which
                                  sums in fixed point (reproducible).  AUTO
                                  picks it for HBM-resident matrices whose
                                  gathers are irregular, unless
                                  hspmv_options.deterministic = 1          */
#define HSPMV_KERNEL_MASK 0xFu
/* lanes per row for VECTOR: HSPMV_LANES(L), L in {1,2,4,8,16,32,64}; 0=auto */
#define HSPMV_LANES_SHIFT 4
#define HSPMV_LANES(l) ((unsigned)(l) << HSPMV_LANES_SHIFT)
#define HSPMV_LANES_MASK (0x7Fu << HSPMV_LANES_SHIFT)
#define HSPMV_FLAG_NO_COL16 (1u << 11)    /* keep 32-bit column indices in
                                             the row kernels (see below)   */
#define HSPMV_FLAG_NONTEMPORAL (1u << 12) /* nt loads for val/col streams  */
#define HSPMV_FLAG_DEVICE_PTRS (1u << 13) /* A/maps are device pointers on
                                             the target device (borrowed for
                                             the handle's lifetime, unchanged;
                                             see hspmv_csr)                 */
#define HSPMV_FLAG_NO_XCD_REMAP (1u << 14) /* keep dispatch-order blocks    */
/* Default (neither XCD flag): remap only when the matrix's bytes fit the
 * 256 MiB Infinity Cache (<= 192 MiB), where per-XCD L2 reuse of x pays;
 * HBM-resident matrices stream faster in dispatch order (profiles/r01_sweep*). */
#define HSPMV_FLAG_NO_SPLIT (1u << 15)     /* no split-row kernels: very
                                              long rows stay on one wave   */
/* STREAM/CSR3 elements per lane per LDS chunk: HSPMV_U(u), u in {2,3,4,5,6,8,16};
 * 0 = auto from the mean row length */
#define HSPMV_U_SHIFT 16
#define HSPMV_U(u) ((unsigned)(u) << HSPMV_U_SHIFT)
#define HSPMV_FLAG_PREFETCH (1u << 21) /* STREAM/CSR3: software-pipelined
                                          col/val loads one chunk ahead   */
#define HSPMV_FLAG_XCD_REMAP (1u << 22) /* force the XCD-contiguous block
                                           order whatever the size         */
#define HSPMV_FLAG_COL16 (1u << 23)     /* force 16-bit column offsets
                                           whenever p <= 8 (see below)     */
/* Explicit XCD chunk: HSPMV_XCD_CHUNK(s), s a power of two >= 1: each XCD
 * takes s consecutive blocks in turn (1 = dispatch order).  Overrides the
 * two flags above; 0 = automatic. */
#define HSPMV_XCD_CHUNK_SHIFT 24
#define HSPMV_XCD_CHUNK(s) ((unsigned)(__builtin_ctz((unsigned)(s)) + 1) << HSPMV_XCD_CHUNK_SHIFT)
/* STREAM: 64-row groups per wave, HSPMV_GROUPS(g), g in {1,2,4,8,16}; the
 * next group's row pointers are loaded while this one streams.  0 = auto. */
#define HSPMV_GROUPS_SHIFT 29
#define HSPMV_GROUPS(g) ((unsigned)(__builtin_ctz((unsigned)(g)) + 1) << HSPMV_GROUPS_SHIFT)
/* 16-bit column offsets (default when the matrix allows it): at handle
 * creation the column indices are re-encoded per 256-nonzero block as
 * col = base[k / 256] + off16[k] + (p high bits from p bit-planes), with p
 * the fewest bits that cover every block's column span (p = 0 for spans
 * < 65536, e.g. banded matrices); the STREAM and CSR3 kernels then stream
 * 2 + p/8 instead of 4 index bytes per nonzero.  Used by default when p <= 1
 * and the matrix streams from HBM (> 192 MiB); measured slower otherwise.
 * HSPMV_FLAG_COL16 forces them (any size, p <= 8).   Products and summation order are
 * unchanged, so y is bit-identical.  HSPMV_FLAG_NO_COL16 turns it off;
 * hspmv_info.col16 / format_bytes report what a handle uses. */

/* ---------------------------------------------------------------- options */
/* Explicit planner choices for hspmv_create_ex.  Zero-initialise, set
 * struct_size = sizeof(hspmv_options) (a caller built against an older,
 * shorter struct passes its own size; the fields it lacks read as 0), then
 * set what you need: every 0 means "the library's choice", which is what
 * hspmv_create / _on_device / _sharded use.  These replace the HSPMV_*
 * environment variables of earlier versions: a production handle's kernel
 * and tables depend only on the matrix, the flags and these options (only a
 * diagnostic build, `make diag-env`, reads the environment). */
#define HSPMV_CSR3_PLAN_AUTO 0    /* = ALIGNED                                */
#define HSPMV_CSR3_PLAN_ALIGNED 1 /* 64-row aligned wave tasks, 4 per
                                     workgroup (the maps bound the shards)   */
#define HSPMV_CSR3_PLAN_PACKED 2  /* whole super-rows (inner map) packed into
                                     <= 64-row wave tasks                    */
#define HSPMV_CSR3_PLAN_SSR 3     /* one workgroup per super-super-row (outer
                                     map), its super-rows split over W waves
                                     by nonzeros: the reference's cuSpMV_3
                                     mapping (csrk.cu:245-319)               */
#define HSPMV_CSR3_PLAN_ROW_GROUPS 4 /* hspmv_info only: a CSR matrix (no
                                     maps) run by the CSR3 kernel over 64-row
                                     groups with the heavy ones cut         */
#define HSPMV_DETERMINISTIC_ORDERED 1
#define HSPMV_DETERMINISTIC_REPRODUCIBLE 2
#define HSPMV_DETERMINISTIC_SERIAL 3
typedef struct {
  uint32_t struct_size;   /* sizeof(hspmv_options) of the caller            */
  uint32_t flags;         /* HSPMV_KERNEL_* | HSPMV_FLAG_* (hspmv_create)    */
  const int *devices;     /* row-range shard p on devices[p] (may repeat), as
                             hspmv_create_sharded; NULL: one shard on device */
  int32_t n_devices;
  int32_t device;         /* single-shard handle: the HIP device ...         */
  void *stream;           /* ... and its hipStream_t (NULL: library-owned)  */
  int32_t csr3_plan;      /* HSPMV_CSR3_PLAN_*                              */
  int32_t task_nnz;       /* CSR3 wave-task nonzero budget (0: 2048)        */
  int32_t x_windows;      /* -1: no LDS x windows; 0 auto                   */
  int32_t x_dict;         /* -1 off, 0 auto, 1 whenever it fits the cap     */
  int32_t x_dict_cap;     /* LDS bytes per dictionary block (0: 20 KiB)     */
  int32_t x_slabs;        /* -1 off, 0 auto, B > 0: B column slabs          */
  int32_t col16_group;    /* -1 off, 0 auto, 1 whenever every group fits    */
  int32_t csort;          /* -1 off, 0 auto, 1 whenever it can be built     */
  int32_t csort_parts;    /* column parts of the csort row blocks: 0 auto,
                             1, 2, 4                                        */
  int32_t csort_chunk_u;  /* csort entries per lane per chunk: 0, 4, 8, 16  */
  int32_t stream_waves;   /* STREAM waves per workgroup: 0 auto, 1, 2, 4    */
  int32_t deterministic;  /* HSPMV_DETERMINISTIC_*: 0 the fastest kernel
                             (CSORT's fp64 slot sums add in LDS-atomic
                             order); 1 ORDERED: only the row kernels (bit-
                             identical run to run; rows of <= 40 (fp32: 56) nonzeros
                             added in omp_spmv's order, longer ones in fixed
                             trees); 2 REPRODUCIBLE: bit-identical run to
                             run for a finite x -- CSORT then runs with
                             fixed-point (int64) row sums: each product
                             rounded once to 2^-50 of |its row's largest
                             value| * |x|max (hspmv_info.csort_fixed_point);
                             3 SERIAL: the row kernels add EVERY row left to
                             right from 0, one lane per row, as omp_spmv
                             does (spmv-csr/spmv.c:92-114): y bit-identical
                             to it for every input, at the cost of long rows
                             added one product at a time (rows over 4096
                             nonzeros: one workgroup each, or with
                             HSPMV_FLAG_NO_SPLIT their lane; VECTOR and CSORT
                             refused; a matrix the row kernels cannot
                             address fails with HSPMV_E_INVALID;
                             hspmv_info.serial_order)                      */
  int32_t placement_trials; /* array placements timed at creation (0/1
                               off, K <= 8; see hspmv_create_on_device)    */
} hspmv_options;

/* ---------------------------------------------------------------- handle */
/* hspmv_create_on_device / hspmv_create_sharded with explicit options
 * (opt == NULL: all defaults on device 0). */
int hspmv_create_ex(hspmv_handle **h, const hspmv_csr *A, const hspmv_csr3_maps *maps,
                    const hspmv_options *opt);

/* Upload A (and optional CSR-3 maps) to num_gpus devices (0 = all visible).
 * With num_gpus > 1 the rows are partitioned into nnz-balanced contiguous
 * ranges (on super-super-row boundaries when maps are given), x is
 * broadcast and y gathered with RCCL.  Replaces the CSRk_Graph constructor +
 * the H2D uploads of csrk.cu:580-587 / 847-865 and cuda-spmv-csr/spmv.cu:66-71. */
int hspmv_create(hspmv_handle **h, const hspmv_csr *A,
                 const hspmv_csr3_maps *maps, int num_gpus, unsigned flags);

/* The row-range partition of hspmv_create over an explicit device list:
 * shard p lives on devices[p] (n_shards >= 1; a device may repeat).  Distinct
 * devices exchange x / y through RCCL (ncclCommInitAll over the list, also
 * at n_shards = 1); a list that repeats a device exchanges by device-to-
 * device copies.  hspmv_create(num_gpus > 1) is this with devices 0..P-1. */
int hspmv_create_sharded(hspmv_handle **h, const hspmv_csr *A,
                         const hspmv_csr3_maps *maps, const int *devices,
                         int n_shards, unsigned flags);

/* Single-device handle on `device`, launching on `stream` (a hipStream_t;
 * NULL = the library creates one).  This is the entry a one-process-per-GPU
 * caller (torch.distributed, MPI) uses for its row-range shard.
 * Placement trials: for a handle that owns its arrays (no
 * HSPMV_FLAG_DEVICE_PTRS) and whose STREAM / CSR3 kernel streams from HBM,
 * the row pointers, column stream, values, x and y are copied into up to
 * three further allocations, each copy is timed over a few SpMVs and the
 * fastest placement is kept (the others are freed; y bits do not depend on
 * it).  Opt-in: hspmv_options.placement_trials = K (K <= 8 sets; default
 * off -- measured no gain); hspmv_info reports the times.  With trials
 * on, creation launches the kernel. */
int hspmv_create_on_device(hspmv_handle **h, const hspmv_csr *A,
                           const hspmv_csr3_maps *maps, int device,
                           void *stream, unsigned flags);

/* x (n entries of dtype) from host memory -> every GPU (setX, csrk.cu:92-102,
 * minus the x permutation: matrices are used as given). */
int hspmv_set_x(hspmv_handle *h, const void *x_host);
/* Bind caller-owned device vectors (single-device handles).  x: n entries,
 * y: m entries, on the handle's device.  NULL restores the handle's own. */
int hspmv_bind_x_device(hspmv_handle *h, const void *x_dev);
int hspmv_bind_y_device(hspmv_handle *h, void *y_dev);
/* Device pointers currently used for x / y on GPU `gpu`. */
void *hspmv_x_device(hspmv_handle *h, int gpu);
void *hspmv_y_device(hspmv_handle *h, int gpu);

/* Enqueue ONE y = A*x on the handle's stream(s).  Asynchronous; the hot path. */
int hspmv_spmv(hspmv_handle *h);
int hspmv_synchronize(hspmv_handle *h);

/* Reference timing protocol: warmup SpMVs, then iters timed SpMVs, each
 * bracketed by events + synchronize (hip/spmv-auto-mi100.cu:214-236). */
int hspmv_run(hspmv_handle *h, int warmup, int iters, hspmv_timing *out);

/* y (m entries of dtype) -> host; gathers the shards of a multi-GPU handle
 * (getY, csrk.cu:110-113). */
int hspmv_get_y(hspmv_handle *h, void *y_host);

/* Multi-GPU only: RCCL broadcast of x from GPU 0 and all-gather of y into
 * every GPU's full-length buffer, timed (seconds).  Either pointer may be NULL. */
int hspmv_exchange(hspmv_handle *h, double *bcast_x_s, double *gather_y_s);

/* Fills the 1.0 layout of hspmv_info -- exactly HSPMV_INFO_SIZE_1_0 bytes,
 * in every 1.x library, so a 1.0 binary's stack struct is never overrun
 * when a later minor grows hspmv_info (NULL -> E_INVALID).  Fields added
 * after 1.0 come only from hspmv_get_info_sized. */
#define HSPMV_INFO_SIZE_1_0 248
int hspmv_get_info(hspmv_handle *h, hspmv_info *out);
/* Fills min(out_size, sizeof(hspmv_info)) bytes: pass sizeof(hspmv_info) of
 * the header you were built against. */
int hspmv_get_info_sized(hspmv_handle *h, hspmv_info *out, uint32_t out_size);
void hspmv_destroy(hspmv_handle *h);

/* ---------------------------------------------------------------- formats */
/* Text .csr reader (spmv-csr/spmv.c:11-57 layout; index base auto-detected
 * from row_ptr[0]; values parsed correctly rounded into dtype). */
int hspmv_read_csr(const char *path, int dtype, hspmv_csr_buf *out);
/* Text .csr3 reader (reformat-csr-to-csr3/stats.c:10-79 layout). */
int hspmv_read_csr3(const char *path, int dtype, hspmv_csr_buf *A,
                    hspmv_csr3_buf *maps);
/* Matrix Market coordinate reader (the input of the reference's converter,
 * helpers/converter.m:1-50 with helpers/mmread.m): field real | integer |
 * pattern, symmetry general | symmetric | skew-symmetric (symmetric files
 * expanded as A + A.' - diag(diag(A)), mmread.m:207-209); duplicates summed,
 * exact zeros dropped, columns sorted per row (helpers/sparse2csr.m). */
int hspmv_read_mtx(const char *path, int dtype, hspmv_csr_buf *out);
/* Writers (reference text layouts: helpers/sparse2csr.m:1-7 for .csr,
 * reformat-csr-to-csr3/spmv-auto.cpp:30-65 for .csr3; values "%.6f"). */
int hspmv_write_csr(const char *path, const hspmv_csr *A);
int hspmv_write_csr3(const char *path, const hspmv_csr *A,
                     const hspmv_csr3_maps *maps);
/* Binary cache: raw little-endian arrays. */
int hspmv_save_bin(const char *path, const hspmv_csr *A,
                   const hspmv_csr3_maps *maps);
int hspmv_load_bin(const char *path, hspmv_csr_buf *A, hspmv_csr3_buf *maps);
void hspmv_free_csr(hspmv_csr_buf *A);
void hspmv_free_csr3(hspmv_csr3_buf *maps);

/* ---------------------------------------------------------------- CSR-3 */
/* Build CSR-3 maps in file order with the handCoarsen grouping rule
 * (csrk.cu:1438-1484) and level thresholds supRowSizes[i-1]*NNZ/N
 * (csrk.cu:1089-1091).  ssrs = rows->super-rows size, srs =
 * super-rows->super-super-rows size. */
int hspmv_build_csr3_maps(const hspmv_csr *A, int ssrs, int srs,
                          hspmv_csr3_buf *out);
/* The full band-k build of CSRk_Graph::putInCSRkFormat with k = 3 and HAND
 * coarsening (BAND_k::preprocessingForSpMV, csrk.cu:1035-1262; reorderA
 * :722-870): super-rows by the handCoarsen rule, RCM on the super-row graph,
 * super-super-rows over the RCM order, RCM on that graph, uncoarsening into
 * one symmetric permutation.  Outputs the permuted matrix (columns sorted
 * per row; *A_out allocated, free with hspmv_free_csr), its maps (*maps_out,
 * free with hspmv_free_csr3) and, if perm != NULL, perm[m]: new row i is row
 * perm[i] of A (so y = P^T y_out, x_out[i] = x[perm[i]]).  A must be square.
 * Replaces what reformat-csr-to-csr3 (spmv-auto.cpp:183-195) writes. */
int hspmv_build_csr3_bandk(const hspmv_csr *A, int ssrs, int srs, hspmv_csr_buf *A_out,
                           hspmv_csr3_buf *maps_out, int32_t *perm);
/* CSR-2 (one map level; spmv-csrk <file> <num_runs> <super_row_size>,
 * spmv-csrk/spmv.cpp:97-128 with CSRK_LEVEL 2, cuda-spmv-csrk/cuda/spmv.cu:130):
 * super-rows of super_row_size * NNZ / N nonzeros (handCoarsen rule), each
 * its own super-super-row (outer = identity), so every CSR-3 consumer takes
 * it unchanged.  _maps keeps the file order; _bandk also RCM-orders the
 * super-row graph and permutes A as the k = 2 band-k build does
 * (csrk.cu:1072-1096: one coarsening + RCM), outputs as
 * hspmv_build_csr3_bandk. */
int hspmv_build_csr2_maps(const hspmv_csr *A, int super_row_size, hspmv_csr3_buf *out);
int hspmv_build_csr2_bandk(const hspmv_csr *A, int super_row_size, hspmv_csr_buf *A_out,
                           hspmv_csr3_buf *maps_out, int32_t *perm);
/* Reverse Cuthill-McKee of A's symmetrised pattern: the ordering the
 * reference's converter applies before writing X.mtx.rcm.csr
 * (helpers/converter.m:14-15, Octave symrcm; tie-breaking not pinned).
 * Outputs P A P^T (columns sorted; free with hspmv_free_csr) and, if
 * perm != NULL, perm[m]: new row i is row perm[i] of A.  A must be square. */
int hspmv_rcm_reorder(const hspmv_csr *A, hspmv_csr_buf *A_out, int32_t *perm);
/* Auto parameters.  flavour 0: the .csr3 writer / Volta formula
 * (reformat-csr-to-csr3/spmv-auto.cpp:154-173); 1: the MI100 driver formula
 * (hip/spmv-auto-mi100.cu:130-158); 2: this library's MI355X choice. */
int hspmv_csr3_params(double nnz_per_row, int flavour, int *ssrs, int *srs);

/* ---------------------------------------------------------------- misc */
/* nnz-balanced contiguous row ranges: splits[0]=0 .. splits[parts]=m, with
 * row_ptr[splits[p]] ~ p*nnz/parts.  With maps != NULL splits fall on
 * super-super-row boundaries. */
int hspmv_partition_rows(int64_t m, const int32_t *row_ptr,
                         const hspmv_csr3_maps *maps, int parts,
                         int64_t *splits);
/* Algorithmic bytes of one SpMV:
 * nnz*(sv+4) + (m+1)*4 + n*sv + m*sv (+ (n_ssr+1 + n_sr+1)*4 for CSR-3),
 * where n = the x entries the SpMV reads, i.e. the number of distinct
 * columns (the matrix width when every column holds a nonzero; much less for
 * a row-range shard of a banded matrix -- hspmv_info.x_entries). */
/* Block x dictionaries (host planner; hspmv_create builds the same tables
 * when it uses them, see hspmv_info.x_dict).  The row kernel's workgroups
 * (STREAM: 256 consecutive rows; CSR3 with maps: four consecutive wave
 * tasks) each stage the x entries their rows reference -- runs of
 * consecutive columns, gaps of <= 8 bridged, <= 63 runs -- in LDS, and every
 * nonzero's column becomes a 16-bit position in that copy.  Outputs:
 * blk[n_blocks+1] record ranges; runs[2*n_records] = {x_start, lds_off} per
 * run, then a sentinel {0, entries} per block; pos[nnz] (0 for split rows,
 * > 4096 nonzeros, unless HSPMV_FLAG_NO_SPLIT).  So x[col[k]] ==
 * staged_b[pos[k]] with staged_b[lds_off + i] = x[x_start + i].  Call with
 * NULL buffers for the sizes.  *n_blocks = 0: some block needs more than
 * cap_entries (<= 0: the library's LDS cap for A's dtype), so no dictionary.
 * opt (NULL = defaults) supplies the kernel flags and the CSR-3 plan.
 * Not a reference interface: the test and diagnostic view of the format. */
int hspmv_xdict_plan_ex(const hspmv_csr *A, const hspmv_csr3_maps *maps, const hspmv_options *opt,
                        int64_t cap_entries, int64_t *n_blocks, int64_t *n_records,
                        int32_t *blk, int32_t *runs, uint16_t *pos);
/* Kernel flags instead of options (= hspmv_xdict_plan_ex with an
 * hspmv_options holding only these flags). */
int hspmv_xdict_plan(const hspmv_csr *A, const hspmv_csr3_maps *maps, unsigned flags,
                     int64_t cap_entries, int64_t *n_blocks, int64_t *n_records,
                     int32_t *blk, int32_t *runs, uint16_t *pos);
double hspmv_alg_bytes(int64_t m, int64_t n, int64_t nnz, int dtype,
                       int64_t n_ssr, int64_t n_sr);
int hspmv_device_count(int *count);
/* ncclGetVersion() of the RCCL this process resolved (no device needed). */
int hspmv_rccl_version(int *version);
const char *hspmv_last_error(void);
const char *hspmv_version(void);

#ifdef __cplusplus
}
#endif
#endif /* HSPMV_H */
