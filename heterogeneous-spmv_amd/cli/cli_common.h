// cli_common.h -- shared driver code of the spmv-csr / spmv-csrk executables.
//
// Reproduces the reference benchmark-driver contract:
//   argv:   <matrix file> <num_runs> [...]
//   stdout: "TimeMin: %lg" / "TimeMax: %lg" / "TimeAvg: %lg" (seconds,
//           launch + synchronize wall time, 5 warm-ups first:
//           spmv-csr/spmv.c:164-185, hip/spmv-auto-mi100.cu:200-240) and
//           "Number Wrong: %d" (|y - yhat| > 0.01 against a serial CPU SpMV,
//           cuda-spmv-csr/spmv.cu:270-284), parsed by run_scripts/run_norm.py:94-107.
// plus extra lines: KernelMin/KernelAvg (HIP-event device time), GFLOPs and
// GBps (2 nnz and algorithmic bytes / TimeMin, the wall time printed above),
// KernelGFLOPs/KernelGBps (the same / KernelMin), NumGPUs, Kernel, and
// "Check: PASS|FAIL maxrel=..." (1e-6 relative fp64 tolerance with an
// absolute floor).
//
// Options (after the positional arguments):
//   --gpus N            row-range partition over N GPUs (RCCL x-bcast / y-gather)
//   --dtype f32|f64     value type (default f64; f32 = the reference's type)
//   --x ones|rand:SEED  input vector (default ones, as the reference)
//   --kernel auto|stream|vector[:L]|csr3|csort
//   --nt                non-temporal loads of the matrix streams
//   --plan aligned|packed|ssr   CSR-3 wave-task plan (hspmv_options.csr3_plan;
//                       ssr = one workgroup per super-super-row, the
//                       reference's cuSpMV_3 mapping)
//   --deterministic     only the ordered row kernels (omp_spmv's order; y
//                       bit-identical run to run)
//   --reproducible      y bit-identical run to run, the column-sorted kernel
//                       allowed with fixed-point row sums
//   --serial            every row summed in omp_spmv's order, one lane per
//                       row: y bit-identical to the serial check (reported
//                       as "Bitwise:")
//   --dump-y PATH       write y as raw binary (dtype) for external checks
//   --no-check          skip the serial CPU check
#pragma once
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "hspmv.h"

namespace cli {

struct Options {
  int gpus = 1;
  int dtype = HSPMV_F64;
  bool x_rand = false;
  unsigned long long seed = 42;
  unsigned kernel = HSPMV_KERNEL_AUTO;
  unsigned lanes = 0;
  bool nt = false;
  int plan = HSPMV_CSR3_PLAN_AUTO;
  int deterministic = 0;  // hspmv_options.deterministic
  bool check = true;
  std::string dump_y;
  std::string params = "mi355x";
  bool bandk = true;  // spmv-csrk on a .csr: band-k reorder (the reference's CSRk_Graph)
};

inline bool ends_with(const std::string &s, const char *suf) {
  const size_t n = strlen(suf);
  return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

// Parses "--opt value" style options from argv[first..].  Returns false on error.
inline bool parse_options(int argc, char **argv, int first, Options &o) {
  for (int i = first; i < argc; ++i) {
    std::string a = argv[i];
    auto need = [&](const char *name) -> const char * {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", name);
        return nullptr;
      }
      return argv[++i];
    };
    if (a == "--gpus") {
      const char *v = need("--gpus"); if (!v) return false;
      o.gpus = atoi(v);
    } else if (a == "--dtype") {
      const char *v = need("--dtype"); if (!v) return false;
      if (!strcmp(v, "f32")) o.dtype = HSPMV_F32;
      else if (!strcmp(v, "f64")) o.dtype = HSPMV_F64;
      else { fprintf(stderr, "bad --dtype %s\n", v); return false; }
    } else if (a == "--x") {
      const char *v = need("--x"); if (!v) return false;
      if (!strcmp(v, "ones")) o.x_rand = false;
      else if (!strncmp(v, "rand:", 5)) { o.x_rand = true; o.seed = strtoull(v + 5, nullptr, 10); }
      else { fprintf(stderr, "bad --x %s\n", v); return false; }
    } else if (a == "--kernel") {
      const char *v = need("--kernel"); if (!v) return false;
      if (!strcmp(v, "auto")) o.kernel = HSPMV_KERNEL_AUTO;
      else if (!strcmp(v, "stream")) o.kernel = HSPMV_KERNEL_STREAM;
      else if (!strcmp(v, "csr3")) o.kernel = HSPMV_KERNEL_CSR3;
      else if (!strcmp(v, "csort")) o.kernel = HSPMV_KERNEL_CSORT;
      else if (!strncmp(v, "vector", 6)) {
        o.kernel = HSPMV_KERNEL_VECTOR;
        if (v[6] == ':') o.lanes = (unsigned)atoi(v + 7);
      } else { fprintf(stderr, "bad --kernel %s\n", v); return false; }
    } else if (a == "--nt") {
      o.nt = true;
    } else if (a == "--plan") {
      const char *v = need("--plan"); if (!v) return false;
      if (!strcmp(v, "aligned")) o.plan = HSPMV_CSR3_PLAN_ALIGNED;
      else if (!strcmp(v, "packed")) o.plan = HSPMV_CSR3_PLAN_PACKED;
      else if (!strcmp(v, "ssr")) o.plan = HSPMV_CSR3_PLAN_SSR;
      else { fprintf(stderr, "bad --plan %s\n", v); return false; }
    } else if (a == "--deterministic") {
      o.deterministic = HSPMV_DETERMINISTIC_ORDERED;
    } else if (a == "--reproducible") {
      o.deterministic = HSPMV_DETERMINISTIC_REPRODUCIBLE;
    } else if (a == "--serial") {
      o.deterministic = HSPMV_DETERMINISTIC_SERIAL;
    } else if (a == "--no-check") {
      o.check = false;
    } else if (a == "--dump-y") {
      const char *v = need("--dump-y"); if (!v) return false;
      o.dump_y = v;
    } else if (a == "--file-order") {
      o.bandk = false;
    } else if (a == "--params") {
      const char *v = need("--params"); if (!v) return false;
      o.params = v;
    } else {
      fprintf(stderr, "unknown option %s\n", a.c_str());
      return false;
    }
  }
  return true;
}

inline unsigned flags_of(const Options &o) {
  unsigned f = o.kernel;
  if (o.kernel == HSPMV_KERNEL_VECTOR && o.lanes) f |= HSPMV_LANES(o.lanes);
  if (o.nt) f |= HSPMV_FLAG_NONTEMPORAL;
  return f;
}

// splitmix64 -> U(-1, 1); same generator as hspmv.gen.rand_x in Python.
inline void fill_x(const Options &o, int64_t n, std::vector<double> &x64) {
  x64.assign((size_t)n, 1.0);
  if (!o.x_rand) return;
  unsigned long long s = o.seed;
  for (int64_t i = 0; i < n; ++i) {
    unsigned long long z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    x64[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

// Serial CPU check (test_spmv, spmv-csr/spmv.c:68-90) + reference count
// (|diff| > 0.01) + relative-tolerance verdict.
struct CheckResult {
  int wrong = 0;
  int64_t bit_diff = 0;  // rows whose y is not bit-identical to the serial sum
  double maxrel = 0.0;
  bool pass = true;
};

template <typename T>
CheckResult check_y(const hspmv_csr_buf &A, const T *val, const T *x, const T *y) {
  CheckResult r;
  for (int64_t row = 0; row < A.m; ++row) {
    T temp = 0;
    double mag = 0.0;
    for (int32_t k = A.row_ptr[row]; k < A.row_ptr[row + 1]; ++k) {
      temp += val[k] * x[A.col_idx[k]];
      mag += fabs((double)val[k] * (double)x[A.col_idx[k]]);
    }
    if (memcmp(&y[row], &temp, sizeof(T)) != 0) r.bit_diff++;
    const double d = (double)y[row] - (double)temp;
    if (d > .01 || d < -.01) r.wrong++;
    const double tol_rel = sizeof(T) == 8 ? 1e-6 : 1e-4;
    const double floor = (sizeof(T) == 8 ? 1e-12 : 1e-6) * mag;
    const double err = fabs(d);
    if (err > tol_rel * fabs((double)temp) + floor) r.pass = false;
    const double rel = err / (fabs((double)temp) + floor + 1e-300);
    if (rel > r.maxrel && err > 0) r.maxrel = rel;
  }
  return r;
}

inline int die(const char *what) {
  fprintf(stderr, "%s: %s\n", what, hspmv_last_error());
  return 1;
}

// Runs the timed protocol on an already-read matrix and prints the report.
// perm (optional, m entries): A is the band-k permutation of the file's
// matrix, row i = file row perm[i]; x is generated in file order and
// permuted, and a dumped y is put back in file order.
inline int run_and_report(const hspmv_csr_buf &A, const hspmv_csr3_buf *maps, int num_runs,
                          const Options &o, const int32_t *perm = nullptr) {
  hspmv_csr view = {A.m, A.n, A.nnz, A.row_ptr, A.col_idx, A.val, A.dtype};
  hspmv_csr3_maps mv = {0, 0, nullptr, nullptr};
  if (maps && maps->n_ssr > 0) mv = {maps->n_ssr, maps->n_sr, maps->outer, maps->inner};
  hspmv_handle *h = nullptr;
  int ndev = 0;
  if (hspmv_device_count(&ndev) != HSPMV_OK) return die("hspmv_device_count");
  const int gpus = o.gpus > 0 ? o.gpus : ndev;
  std::vector<int> devs((size_t)(gpus > 0 ? gpus : 1));
  for (size_t p = 0; p < devs.size(); ++p) devs[p] = (int)p;
  hspmv_options opt;
  memset(&opt, 0, sizeof(opt));
  opt.struct_size = sizeof(opt);
  opt.flags = flags_of(o);
  opt.devices = gpus > 1 ? devs.data() : nullptr;  // row-range shards over RCCL
  opt.n_devices = gpus > 1 ? gpus : 0;
  opt.csr3_plan = o.plan;
  opt.deterministic = o.deterministic;
  if (hspmv_create_ex(&h, &view, mv.n_ssr > 0 ? &mv : nullptr, &opt) != HSPMV_OK)
    return die("hspmv_create_ex");
  std::vector<double> x64;
  fill_x(o, A.n, x64);
  if (perm) {
    std::vector<double> xf(x64);
    for (int64_t i = 0; i < A.n; ++i) x64[(size_t)i] = xf[(size_t)perm[i]];
  }
  std::vector<float> x32;
  const void *xp = x64.data();
  if (A.dtype == HSPMV_F32) {
    x32.assign(x64.begin(), x64.end());
    xp = x32.data();
  }
  if (hspmv_set_x(h, xp) != HSPMV_OK) return die("hspmv_set_x");
  hspmv_timing t;
  if (hspmv_run(h, 5, num_runs, &t) != HSPMV_OK) return die("hspmv_run");
  hspmv_info info;
  hspmv_get_info_sized(h, &info, sizeof(info));
  printf("TimeMin: %lg\n", t.wall_min);
  printf("TimeMax: %lg\n", t.wall_max);
  printf("TimeAvg: %lg\n", t.wall_avg);
  printf("KernelMin: %lg\n", t.t_min);
  printf("KernelAvg: %lg\n", t.t_avg);
  // GFLOPs / GBps from TimeMin, as a run_scripts consumer computes them
  // (run_norm.py:94-107 records TimeMin); the HIP-event rates beside them
  printf("GFLOPs: %lg\n", t.wall_min > 0 ? 2.0 * (double)A.nnz / t.wall_min * 1e-9 : 0.0);
  printf("GBps: %lg\n", t.wall_min > 0 ? info.alg_bytes / t.wall_min * 1e-9 : 0.0);
  printf("KernelGFLOPs: %lg\n", t.gflops);
  printf("KernelGBps: %lg\n", t.gbps_alg);
  printf("NumGPUs: %d\n", t.num_gpus);
  static const char *kname[] = {"auto", "vector", "stream", "csr3", "csort"};
  static const char *pname[] = {"-", "aligned", "packed", "ssr"};
  printf("Kernel: %s lanes=%d waves_per_block=%d blocks=%lld plan=%s deterministic=%d\n",
         kname[(info.kernel >= 0 && info.kernel <= 4) ? info.kernel : 0], info.lanes,
         info.waves_per_block, (long long)info.blocks,
         pname[(info.csr3_plan >= 0 && info.csr3_plan <= 3) ? info.csr3_plan : 0], info.deterministic);
  const size_t sv = A.dtype == HSPMV_F64 ? 8 : 4;
  std::vector<char> y(sv * (size_t)(A.m ? A.m : 1));
  if (hspmv_get_y(h, y.data()) != HSPMV_OK) return die("hspmv_get_y");
  if (!o.dump_y.empty()) {
    std::vector<char> yf(y.size());
    if (perm)  // back to the file's row order
      for (int64_t i = 0; i < A.m; ++i) memcpy(&yf[sv * (size_t)perm[i]], &y[sv * (size_t)i], sv);
    else
      yf = y;
    FILE *fp = fopen(o.dump_y.c_str(), "wb");
    if (!fp || fwrite(yf.data(), sv, (size_t)A.m, fp) != (size_t)A.m) {
      fprintf(stderr, "cannot write %s\n", o.dump_y.c_str());
      return 1;
    }
    fclose(fp);
  }
  int rc = 0;
  if (o.check) {
    CheckResult r = A.dtype == HSPMV_F64
                        ? check_y<double>(A, (const double *)A.val, x64.data(), (const double *)y.data())
                        : check_y<float>(A, (const float *)A.val, x32.data(), (const float *)y.data());
    printf("Number Wrong: %d \n", r.wrong);
    printf("Check: %s maxrel=%.3e\n", r.pass ? "PASS" : "FAIL", r.maxrel);
    rc = r.pass ? 0 : 2;
    if (o.deterministic == HSPMV_DETERMINISTIC_SERIAL) {  // the serial order's contract
      printf("Bitwise: %lld rows differ\n", (long long)r.bit_diff);
      if (r.bit_diff) rc = 2;
    }
  }
  hspmv_destroy(h);
  return rc;
}

// Reads .csr / .csr3 / .bin by extension (.csr3 and .bin may carry maps).
inline int read_matrix(const std::string &path, int dtype, hspmv_csr_buf &A, hspmv_csr3_buf &maps) {
  memset(&A, 0, sizeof(A));
  memset(&maps, 0, sizeof(maps));
  int rc;
  if (ends_with(path, ".csr3"))
    rc = hspmv_read_csr3(path.c_str(), dtype, &A, &maps);
  else if (ends_with(path, ".bin"))
    rc = hspmv_load_bin(path.c_str(), &A, &maps);
  else
    rc = hspmv_read_csr(path.c_str(), dtype, &A);
  return rc;
}

}  // namespace cli
