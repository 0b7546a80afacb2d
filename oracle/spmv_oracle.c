/*
 * oracle/spmv_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's CSR / CSR-3 SpMV path, used as the
 * parity checker for the HIP path and as the CPU baseline timed by bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product (libhspmv.so, the CLIs) never links it.
 *
 * Parity pin: the fp32 mode is checked BITWISE against the reference's own
 * spmv-csr/spmv.c compiled from /root/reference by oracle/Makefile into
 * oracle/_ref/ (tests/golden/make_golden.py records the outputs as fixtures).
 * The fp64 mode runs the identical loop in double.
 *
 * Every function cites the reference file:line it restates.  Rounding
 * contract: per-row sum starts at 0 and adds val[k]*x[col[k]] left to right,
 * product rounded then sum rounded (no FMA contraction: built with
 * -ffp-contract=off, exactly what gcc emits for the reference on x86-64).
 */
#define _GNU_SOURCE
#include <math.h>
#include <omp.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* Reader: restates my_read_csr (spmv-csr/spmv.c:11-57).               */
/* Header "m n nnz", then m+1 row pointers, nnz column indices, nnz     */
/* values.  Values are parsed twice: strtof (bit-identical to the        */
/* reference's fscanf("%f")) and strtod (fp64 mode).  The index base is  */
/* auto-detected from row_ptr[0] (0-based readers: spmv-csr/spmv.c:36-49;*/
/* 1-based readers subtract 1: spmv-csrk/spmv.cpp:60,67).               */
/* ------------------------------------------------------------------ */
static char *orc_slurp(const char *path, size_t *len) {
  FILE *fp = fopen(path, "rb");
  if (!fp) return NULL;
  fseek(fp, 0, SEEK_END);
  long sz = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  char *buf = (char *)malloc((size_t)sz + 1);
  if (!buf) { fclose(fp); return NULL; }
  size_t got = fread(buf, 1, (size_t)sz, fp);
  fclose(fp);
  buf[got] = 0;
  *len = got;
  return buf;
}

/* Returns 0 on success.  Arrays are malloc'd; free with orc_free. */
int orc_read_csr(const char *path, int64_t *m, int64_t *n, int64_t *nnz,
                 int32_t **row_ptr, int32_t **col_idx, float **val32,
                 double **val64, int *base_out) {
  size_t len = 0;
  char *buf = orc_slurp(path, &len);
  if (!buf) return -1;
  char *p = buf, *e;
  long long hm = strtoll(p, &e, 10); if (e == p) { free(buf); return -2; } p = e;
  long long hn = strtoll(p, &e, 10); if (e == p) { free(buf); return -2; } p = e;
  long long hz = strtoll(p, &e, 10); if (e == p) { free(buf); return -2; } p = e;
  if (hm < 0 || hn < 0 || hz < 0) { free(buf); return -2; }
  int32_t *rp = (int32_t *)malloc(sizeof(int32_t) * (size_t)(hm + 1));
  int32_t *ci = (int32_t *)malloc(sizeof(int32_t) * (size_t)(hz ? hz : 1));
  float *v32 = (float *)malloc(sizeof(float) * (size_t)(hz ? hz : 1));
  double *v64 = (double *)malloc(sizeof(double) * (size_t)(hz ? hz : 1));
  for (long long i = 0; i <= hm; ++i) {
    long long t = strtoll(p, &e, 10);
    if (e == p) { free(buf); return -3; }
    p = e; rp[i] = (int32_t)t;
  }
  for (long long i = 0; i < hz; ++i) {
    long long t = strtoll(p, &e, 10);
    if (e == p) { free(buf); return -3; }
    p = e; ci[i] = (int32_t)t;
  }
  for (long long i = 0; i < hz; ++i) {
    char *e32, *e64;
    v32[i] = strtof(p, &e32);
    v64[i] = strtod(p, &e64);
    if (e64 == p) { free(buf); return -3; }
    p = e64;
  }
  free(buf);
  int base = rp[0];
  if (base != 0 && base != 1) return -4;
  if (base == 1) {
    for (long long i = 0; i <= hm; ++i) rp[i] -= 1;
    for (long long i = 0; i < hz; ++i) ci[i] -= 1;
  }
  *m = hm; *n = hn; *nnz = hz;
  *row_ptr = rp; *col_idx = ci;
  if (val32) *val32 = v32; else free(v32);
  if (val64) *val64 = v64; else free(v64);
  if (base_out) *base_out = base;
  return 0;
}

/* Reader for .csr3: restates my_read_csr3 (reformat-csr-to-csr3/stats.c:10-79)
 * and the writer's layout (reformat-csr-to-csr3/spmv-auto.cpp:30-65):
 * "nSSR nSR M N NNZ" / outer[nSSR+1] / inner[nSR+1] / rp[M+1] / col[NNZ] /
 * val[NNZ].  The first two header fields are COUNTS (stats.c:21,41-52). */
int orc_read_csr3(const char *path, int64_t *nssr, int64_t *nsr, int64_t *m,
                  int64_t *n, int64_t *nnz, int32_t **outer, int32_t **inner,
                  int32_t **row_ptr, int32_t **col_idx, float **val32,
                  double **val64) {
  size_t len = 0;
  char *buf = orc_slurp(path, &len);
  if (!buf) return -1;
  char *p = buf, *e;
  long long h[5];
  for (int i = 0; i < 5; ++i) {
    h[i] = strtoll(p, &e, 10);
    if (e == p || h[i] < 0) { free(buf); return -2; }
    p = e;
  }
  int32_t *o = (int32_t *)malloc(sizeof(int32_t) * (size_t)(h[0] + 1));
  int32_t *in = (int32_t *)malloc(sizeof(int32_t) * (size_t)(h[1] + 1));
  int32_t *rp = (int32_t *)malloc(sizeof(int32_t) * (size_t)(h[2] + 1));
  int32_t *ci = (int32_t *)malloc(sizeof(int32_t) * (size_t)(h[4] ? h[4] : 1));
  float *v32 = (float *)malloc(sizeof(float) * (size_t)(h[4] ? h[4] : 1));
  double *v64 = (double *)malloc(sizeof(double) * (size_t)(h[4] ? h[4] : 1));
  int32_t *arrs[3] = {o, in, rp};
  long long cnt[3] = {h[0] + 1, h[1] + 1, h[2] + 1};
  for (int a = 0; a < 3; ++a)
    for (long long i = 0; i < cnt[a]; ++i) {
      long long t = strtoll(p, &e, 10);
      if (e == p) { free(buf); return -3; }
      p = e; arrs[a][i] = (int32_t)t;
    }
  for (long long i = 0; i < h[4]; ++i) {
    long long t = strtoll(p, &e, 10);
    if (e == p) { free(buf); return -3; }
    p = e; ci[i] = (int32_t)t;
  }
  for (long long i = 0; i < h[4]; ++i) {
    char *e32, *e64;
    v32[i] = strtof(p, &e32);
    v64[i] = strtod(p, &e64);
    if (e64 == p) { free(buf); return -3; }
    p = e64;
  }
  free(buf);
  *nssr = h[0]; *nsr = h[1]; *m = h[2]; *n = h[3]; *nnz = h[4];
  *outer = o; *inner = in; *row_ptr = rp; *col_idx = ci;
  if (val32) *val32 = v32; else free(v32);
  if (val64) *val64 = v64; else free(v64);
  return 0;
}

void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------ */
/* Kernels.                                                           */
/* ------------------------------------------------------------------ */

/* test_spmv (spmv-csr/spmv.c:68-90): serial reference yhat. */
void orc_test_spmv_f32(int64_t m, const int32_t *rp, const int32_t *ci,
                       const float *val, const float *x, float *y) {
  for (int64_t row = 0; row < m; ++row) {
    float temp = 0;
    for (int32_t k = rp[row]; k < rp[row + 1]; ++k) temp += val[k] * x[ci[k]];
    y[row] = temp;
  }
}

void orc_test_spmv_f64(int64_t m, const int32_t *rp, const int32_t *ci,
                       const double *val, const double *x, double *y) {
  for (int64_t row = 0; row < m; ++row) {
    double temp = 0;
    for (int32_t k = rp[row]; k < rp[row + 1]; ++k) temp += val[k] * x[ci[k]];
    y[row] = temp;
  }
}

/* omp_spmv (spmv-csr/spmv.c:92-114): the CPU hot path and the baseline.
 * schedule(runtime) so OMP_SCHEDULE picks static/guided as the reference
 * harness does (run_scripts/run_norm.py:66, run_cuda_new.py:79). */
void orc_omp_spmv_f32(int64_t m, const int32_t *rp, const int32_t *ci,
                      const float *val, const float *x, float *y) {
  int64_t row;
#pragma omp parallel for schedule(runtime)
  for (row = 0; row < m; ++row) {
    float temp = 0;
    for (int32_t k = rp[row]; k < rp[row + 1]; ++k) temp += val[k] * x[ci[k]];
    y[row] = temp;
  }
}

void orc_omp_spmv_f64(int64_t m, const int32_t *rp, const int32_t *ci,
                      const double *val, const double *x, double *y) {
  int64_t row;
#pragma omp parallel for schedule(runtime)
  for (row = 0; row < m; ++row) {
    double temp = 0;
    for (int32_t k = rp[row]; k < rp[row + 1]; ++k) temp += val[k] * x[ci[k]];
    y[row] = temp;
  }
}

/* Per-row absolute-magnitude sum  s[r] = sum |val[k] * x[col[k]]|, used by
 * the parity tests for the absolute floor of the fp64 tolerance
 * (|y - y64| <= 1e-6 |y64| + 1e-12 * s). */
void orc_abs_rowsum_f64(int64_t m, const int32_t *rp, const int32_t *ci,
                        const double *val, const double *x, double *s) {
  int64_t row;
#pragma omp parallel for schedule(static)
  for (row = 0; row < m; ++row) {
    double t = 0;
    for (int32_t k = rp[row]; k < rp[row + 1]; ++k) t += fabs(val[k] * x[ci[k]]);
    s[row] = t;
  }
}

/* CSR-3 CPU loop (spmv-csrk/csrk.cpp:247-285; HIP-library host copy
 * cuda-spmv-csrk/hip/csrk.cu:428-459): ssr -> sr -> row, same per-row order
 * as omp_spmv, so it must equal A1 on the .csr3's embedded CSR. */
void orc_csr3_spmv_f64(int64_t nssr, const int32_t *outer, const int32_t *inner,
                       const int32_t *rp, const int32_t *ci, const double *val,
                       const double *x, double *y) {
  int64_t s;
#pragma omp parallel for schedule(runtime)
  for (s = 0; s < nssr; ++s) {
    for (int32_t sr = outer[s]; sr < outer[s + 1]; ++sr) {
      for (int32_t row = inner[sr]; row < inner[sr + 1]; ++row) {
        double temp = 0;
        for (int32_t k = rp[row]; k < rp[row + 1]; ++k) temp += val[k] * x[ci[k]];
        y[row] = temp;
      }
    }
  }
}

void orc_csr3_spmv_f32(int64_t nssr, const int32_t *outer, const int32_t *inner,
                       const int32_t *rp, const int32_t *ci, const float *val,
                       const float *x, float *y) {
  int64_t s;
#pragma omp parallel for schedule(runtime)
  for (s = 0; s < nssr; ++s) {
    for (int32_t sr = outer[s]; sr < outer[s + 1]; ++sr) {
      for (int32_t row = inner[sr]; row < inner[sr + 1]; ++row) {
        float temp = 0;
        for (int32_t k = rp[row]; k < rp[row + 1]; ++k) temp += val[k] * x[ci[k]];
        y[row] = temp;
      }
    }
  }
}

/* ------------------------------------------------------------------ */
/* CSR-3 map construction in file order (no RCM): restates the grouping  */
/* rule of BAND_k::handCoarsen (cuda-spmv-csrk/hip/csrk.cu:1438-1484) and */
/* the level thresholds of preprocessingForSpMV (csrk.cu:1089-1091):      */
/*   threshold_i = supRowSizes[i-1] * NNZ_{i-1} / N_{i-1}  (int math)     */
/* a group keeps absorbing consecutive vertices while its nnz count is   */
/* below the threshold.  The level-1 coarse graph (for NNZ_1, N_1) is the */
/* symmetrised super-row adjacency with duplicate edges merged            */
/* (csrk.cu:1487-1610).                                                   */
/* ------------------------------------------------------------------ */
/* Deliberate deviation: the reference closes the last group only when it
 * holds nonzeros (`if (temp_nnz_count > 0)`, csrk.cu:1466-1467,1481-1484), so a
 * trailing group made of empty rows is dropped and those rows are never
 * mapped (their y is never written).  Here the open group is closed whenever
 * it holds rows; on every matrix without that corner the maps are identical. */
static int64_t orc_group(int64_t N, const int64_t *deg, int64_t thr,
                         int32_t *starts /* may be NULL (count only) */) {
  int64_t ng = 0, acc = 0, last = 0;
  if (starts) starts[0] = 0;
  for (int64_t i = 0; i < N; ++i) {
    if (acc < thr) {
      acc += deg[i];
    } else {
      ng++;
      acc = deg[i];
      last = i;
      if (starts) starts[ng] = (int32_t)i;
    }
  }
  if (N > last) {
    ng++;
    if (starts) starts[ng] = (int32_t)N;
  }
  return ng;
}

static int cmp_i32(const void *a, const void *b) {
  int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  return (x > y) - (x < y);
}

/* Builds outer/inner maps.  Returns 0 and sets *nssr, *nsr; the maps are
 * malloc'd.  ssrs = supRowSizes[0] (rows->super-rows), srs = supRowSizes[1]
 * (super-rows->super-super-rows), matching the CLI naming trap noted in
 * SURVEY.md Appendix A item 11. */
int orc_build_csr3_maps(int64_t m, const int32_t *rp, const int32_t *ci,
                        int64_t ssrs, int64_t srs, int64_t *nssr, int64_t *nsr,
                        int32_t **outer_out, int32_t **inner_out) {
  int64_t nnz = rp[m];
  int64_t *deg = (int64_t *)malloc(sizeof(int64_t) * (size_t)(m ? m : 1));
  for (int64_t i = 0; i < m; ++i) deg[i] = rp[i + 1] - rp[i];
  int64_t thr1 = (int64_t)(int)(ssrs * nnz / (m ? m : 1));
  int64_t n1 = orc_group(m, deg, thr1, NULL);
  int32_t *inner = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n1 + 1));
  orc_group(m, deg, thr1, inner);
  if (n1 == 0) inner[0] = 0;
  /* coarse graph: super-row of every row, then symmetrised edge list */
  int32_t *sup = (int32_t *)malloc(sizeof(int32_t) * (size_t)(m ? m : 1));
  for (int64_t s = 0; s < n1; ++s)
    for (int32_t r = inner[s]; r < inner[s + 1]; ++r) sup[r] = (int32_t)s;
  int64_t *cnt = (int64_t *)calloc((size_t)(n1 + 1), sizeof(int64_t));
  for (int64_t s = 0; s < n1; ++s)
    for (int32_t r = inner[s]; r < inner[s + 1]; ++r)
      for (int32_t k = rp[r]; k < rp[r + 1]; ++k) {
        if (ci[k] >= inner[s] && ci[k] < m) {
          int32_t t = sup[ci[k]];
          cnt[s]++;
          if (t != s) cnt[t]++;
        }
      }
  int64_t *off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n1 + 1));
  off[0] = 0;
  for (int64_t s = 0; s < n1; ++s) off[s + 1] = off[s] + cnt[s];
  int32_t *adj = (int32_t *)malloc(sizeof(int32_t) * (size_t)(off[n1] ? off[n1] : 1));
  int64_t *pos = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n1 + 1));
  for (int64_t s = 0; s <= n1; ++s) pos[s] = off[s];
  for (int64_t s = 0; s < n1; ++s)
    for (int32_t r = inner[s]; r < inner[s + 1]; ++r)
      for (int32_t k = rp[r]; k < rp[r + 1]; ++k) {
        if (ci[k] >= inner[s] && ci[k] < m) {
          int32_t t = sup[ci[k]];
          adj[pos[s]++] = t;
          if (t != s) adj[pos[t]++] = (int32_t)s;
        }
      }
  int64_t *deg1 = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n1 ? n1 : 1));
  int64_t nnz1 = 0;
  for (int64_t s = 0; s < n1; ++s) {
    int64_t c = off[s + 1] - off[s];
    qsort(adj + off[s], (size_t)c, sizeof(int32_t), cmp_i32);
    int64_t d = 0;
    for (int64_t j = 0; j < c; ++j)
      if (j == 0 || adj[off[s] + j] != adj[off[s] + j - 1]) d++;
    deg1[s] = d;
    nnz1 += d;
  }
  int64_t thr2 = (int64_t)(int)(srs * nnz1 / (n1 ? n1 : 1));
  int64_t n2 = orc_group(n1, deg1, thr2, NULL);
  int32_t *outer = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n2 + 1));
  orc_group(n1, deg1, thr2, outer);
  if (n2 == 0) outer[0] = 0;
  free(deg); free(sup); free(cnt); free(off); free(adj); free(pos); free(deg1);
  *nssr = n2; *nsr = n1; *outer_out = outer; *inner_out = inner;
  return 0;
}

/* ------------------------------------------------------------------ */
/* CPU baseline timing: restates the timed loop of spmv-csr/spmv.c:164-185 */
/* (5 warm-ups, N timed runs with omp_get_wtime, min/max/avg).  Doubles   */
/* internally (the reference's float accumulators are Appendix A item 8). */
/* ------------------------------------------------------------------ */
int orc_time_omp_spmv_f64(int64_t m, const int32_t *rp, const int32_t *ci,
                          const double *val, const double *x, double *y,
                          int warmup, int runs, double *tmin, double *tmax,
                          double *tavg) {
  for (int i = 0; i < warmup; ++i) orc_omp_spmv_f64(m, rp, ci, val, x, y);
  double mn = 9999.0, mx = 0.0, sum = 0.0;
  for (int i = 0; i < runs; ++i) {
    double tic = omp_get_wtime();
    orc_omp_spmv_f64(m, rp, ci, val, x, y);
    double toc = omp_get_wtime() - tic;
    sum += toc;
    if (toc < mn) mn = toc;
    if (toc > mx) mx = toc;
  }
  *tmin = mn; *tmax = mx; *tavg = runs ? sum / runs : 0.0;
  return 0;
}

int orc_time_omp_spmv_f32(int64_t m, const int32_t *rp, const int32_t *ci,
                          const float *val, const float *x, float *y,
                          int warmup, int runs, double *tmin, double *tmax,
                          double *tavg) {
  for (int i = 0; i < warmup; ++i) orc_omp_spmv_f32(m, rp, ci, val, x, y);
  double mn = 9999.0, mx = 0.0, sum = 0.0;
  for (int i = 0; i < runs; ++i) {
    double tic = omp_get_wtime();
    orc_omp_spmv_f32(m, rp, ci, val, x, y);
    double toc = omp_get_wtime() - tic;
    sum += toc;
    if (toc < mn) mn = toc;
    if (toc > mx) mx = toc;
  }
  *tmin = mn; *tmax = mx; *tavg = runs ? sum / runs : 0.0;
  return 0;
}

/* The same protocol keeping every run's time (seconds) in samples[runs],
 * so the caller can report the median beside TimeMin/TimeAvg. */
int orc_time_omp_spmv_samples_f64(int64_t m, const int32_t *rp, const int32_t *ci,
                                  const double *val, const double *x, double *y,
                                  int warmup, int runs, double *samples) {
  for (int i = 0; i < warmup; ++i) orc_omp_spmv_f64(m, rp, ci, val, x, y);
  for (int i = 0; i < runs; ++i) {
    double tic = omp_get_wtime();
    orc_omp_spmv_f64(m, rp, ci, val, x, y);
    samples[i] = omp_get_wtime() - tic;
  }
  return 0;
}

int orc_time_omp_spmv_samples_f32(int64_t m, const int32_t *rp, const int32_t *ci,
                                  const float *val, const float *x, float *y,
                                  int warmup, int runs, double *samples) {
  for (int i = 0; i < warmup; ++i) orc_omp_spmv_f32(m, rp, ci, val, x, y);
  for (int i = 0; i < runs; ++i) {
    double tic = omp_get_wtime();
    orc_omp_spmv_f32(m, rp, ci, val, x, y);
    samples[i] = omp_get_wtime() - tic;
  }
  return 0;
}

/* Thread placement for the CPU baseline (what OMP_PLACES + OMP_PROC_BIND=
 * spread do, run_scripts/run_cuda_new.py:75-79; set here because libgomp
 * reads those variables only once, at load, and binding the main thread at
 * load shrinks the affinity mask bench.py reads).  Team thread t is bound to
 * place t % n_places, place p being the CPUs cpus[off[p] .. off[p+1]).
 * Returns the number of threads bound. */
int orc_bind_threads(int nthreads, int n_places, const int *off, const int *cpus) {
  int ok = 0;
  if (nthreads < 1 || n_places < 1) return 0;
  omp_set_num_threads(nthreads);
#pragma omp parallel reduction(+ : ok)
  {
    const int p = omp_get_thread_num() % n_places;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int i = off[p]; i < off[p + 1]; ++i) CPU_SET(cpus[i], &set);
    ok += sched_setaffinity(0, sizeof(set), &set) == 0;
  }
  return ok;
}

/* First-touch copies of a CSR into caller-allocated, untouched buffers, in
 * the static row partition omp_spmv's schedule(runtime) = static uses, so
 * each thread's rows sit on its own NUMA node (spmv-csr/spmv.c reads the
 * file on one thread; on a two-socket host that puts the whole matrix on
 * one node and the timing on where the scheduler happened to run). */
void orc_localize_csr(int64_t m, const int32_t *rp, const int32_t *ci, const void *val,
                      int val_bytes, int32_t *rp2, int32_t *ci2, void *val2) {
  int64_t row;
#pragma omp parallel for schedule(static)
  for (row = 0; row < m; ++row) {
    const int32_t k0 = rp[row], k1 = rp[row + 1];
    rp2[row] = k0;
    memcpy(ci2 + k0, ci + k0, sizeof(int32_t) * (size_t)(k1 - k0));
    memcpy((char *)val2 + (size_t)val_bytes * (size_t)k0, (const char *)val + (size_t)val_bytes * (size_t)k0,
           (size_t)val_bytes * (size_t)(k1 - k0));
  }
  rp2[m] = rp[m];
}

int orc_max_threads(void) { return omp_get_max_threads(); }

/* schedule(runtime) control without relying on OMP_SCHEDULE being read before
 * libgomp initialised (the harness sets it per run: run_scripts/run_norm.py:66).
 * kind: 1 static, 2 dynamic, 3 guided (omp_sched_t). */
void orc_set_schedule(int kind, int chunk) { omp_set_schedule((omp_sched_t)kind, chunk); }
void orc_set_threads(int n) { if (n > 0) omp_set_num_threads(n); }
