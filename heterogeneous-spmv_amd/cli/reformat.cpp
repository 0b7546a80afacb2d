// reformat-auto / reformat -- the reference's offline converters from a .csr
// file to the inputs of its CSR-k drivers, over this library's band-k build
// (host only: no GPU is touched).
//   reformat-auto <in.csr> <out.csr3>
//       auto (ssrs, srs) by the .csr3 writer's formula (hspmv_csr3_params
//       flavour 0: reformat-csr-to-csr3/spmv-auto.cpp:154-173), the k = 3
//       band-k reordering (hspmv_build_csr3_bandk: CSRk_Graph
//       putInCSRkFormat, spmv-auto.cpp:183-192), then the maps and the
//       permuted matrix as .csr3 (spmv-auto.cpp:30-65, hspmv_write_csr3)
//   reformat <in.csr> <out> [ignored]
//       the same reordering written as a plain .csr without maps
//       (reformat-csr-to-csr3/spmv.cpp:30-65, 132-190; convert-all.sh:14
//       passes a third argument the tool never reads)
// Built twice from this file; HSPMV_REFORMAT_PLAIN selects the second form.
// Options after the positional arguments: --ssrs S --srs R override the
// formula; --dtype f32|f64 is the precision the values are parsed in (f32,
// the default, is the reference's float; both write "%.6f").
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>

#include "hspmv.h"

#ifndef HSPMV_REFORMAT_PLAIN
#define HSPMV_REFORMAT_PLAIN 0
#endif

static int die(const char *what) {
  fprintf(stderr, "%s failed: %s\n", what, hspmv_last_error());
  return 1;
}

int main(int argc, char **argv) {
  if (argc < 3) {
    printf("Syntax: %s inputfile outputfile\n", argv[0]);
    return 0;
  }
  int ssrs = 0, srs = 0, dtype = HSPMV_F32;
  for (int i = 3; i < argc; ++i) {
    const std::string a = argv[i];
    if (a[0] != '-') continue;  // the plain form's ignored third argument
    if (i + 1 >= argc) {
      fprintf(stderr, "%s needs a value\n", a.c_str());
      return 1;
    }
    const char *v = argv[++i];
    if (a == "--ssrs") {
      ssrs = atoi(v);
    } else if (a == "--srs") {
      srs = atoi(v);
    } else if (a == "--dtype") {
      if (strcmp(v, "f32") != 0 && strcmp(v, "f64") != 0) {
        fprintf(stderr, "--dtype f32|f64\n");
        return 1;
      }
      dtype = strcmp(v, "f64") == 0 ? HSPMV_F64 : HSPMV_F32;
    } else {
      fprintf(stderr, "unknown option %s\n", a.c_str());
      return 1;
    }
  }
  if ((ssrs > 0) != (srs > 0) || ssrs < 0 || srs < 0) {
    fprintf(stderr, "--ssrs and --srs go together, both >= 1\n");
    return 1;
  }
  hspmv_csr_buf A;
  memset(&A, 0, sizeof(A));
  if (hspmv_read_csr(argv[1], dtype, &A) != HSPMV_OK) return die("read");
  if (A.m != A.n) {
    fprintf(stderr, "%s is %lld x %lld: the band-k reordering needs a square matrix\n", argv[1],
            (long long)A.m, (long long)A.n);
    hspmv_free_csr(&A);
    return 1;
  }
  if (ssrs == 0) {
    const double d = A.m ? (double)A.nnz / (double)A.m : 1.0;
    hspmv_csr3_params(d > 0 ? d : 1.0, 0, &ssrs, &srs);
  }
  // the reference's banner (spmv-auto.cpp:171-180 prints the two sizes
  // back to back; spmv.cpp:171-176 only the first)
  printf("using ssrs %d, srs %d\n", ssrs, srs);
  if (HSPMV_REFORMAT_PLAIN)
    printf("SpMV\nHAND\n3\n%d\n", ssrs);
  else
    printf("SpMV\nHAND\n3\n%d%d\n", ssrs, srs);
  printf("Read in matrix and config file.\n");
  const hspmv_csr view = {A.m, A.n, A.nnz, A.row_ptr, A.col_idx, A.val, A.dtype};
  hspmv_csr_buf P;
  hspmv_csr3_buf maps;
  memset(&P, 0, sizeof(P));
  memset(&maps, 0, sizeof(maps));
  const auto tic = std::chrono::steady_clock::now();
  if (hspmv_build_csr3_bandk(&view, ssrs, srs, &P, &maps, nullptr) != HSPMV_OK) {
    hspmv_free_csr(&A);
    return die("band-k build");
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - tic).count();
  hspmv_free_csr(&A);
  if (!HSPMV_REFORMAT_PLAIN) printf("%s reordered in %g seconds.\n", argv[1], dt);
  printf("In CSR-k format.\n");
  const hspmv_csr pv = {P.m, P.n, P.nnz, P.row_ptr, P.col_idx, P.val, P.dtype};
  const hspmv_csr3_maps mv = {maps.n_ssr, maps.n_sr, maps.outer, maps.inner};
  const int rc = HSPMV_REFORMAT_PLAIN ? hspmv_write_csr(argv[2], &pv) : hspmv_write_csr3(argv[2], &pv, &mv);
  hspmv_free_csr3(&maps);
  hspmv_free_csr(&P);
  return rc == HSPMV_OK ? 0 : die("write");
}
