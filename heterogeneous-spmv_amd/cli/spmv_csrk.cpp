// spmv-csrk -- MI355X CSR-3 SpMV benchmark driver.
// Command lines of the reference's CSR-k drivers:
//   spmv-csrk <file.csr> <num_runs> <super_super_row_size> <super_row_size>
//       manual sizes, as cuda-spmv-csrk/hip/spmv.cu:112-132
//   spmv-csrk <file.csr> <num_runs> <super_row_size>
//       CSR-2 (one map level), as spmv-csrk/spmv.cpp:97-128 (CSRK_LEVEL 2)
//       and cuda-spmv-csrk/cuda/spmv.cu:130
//   spmv-csrk <file.csr> <num_runs>
//       auto sizes, as hip/spmv-auto-mi100.cu:130-166 (--params
//       mi355x|mi100|volta picks the formula; default mi355x)
//   spmv-csrk <file.csr3> <num_runs>
//       maps read from the .csr3 file (reformat-csr-to-csr3 output)
// On a .csr the matrix goes through the reference's band-k build
// (hspmv_build_csr3_bandk: hand-coarsening + RCM per coarse level + symmetric
// permutation, CSRk_Graph::putInCSRkFormat) -- with the permutation applied
// to the matrix AND x, which the reference's GPU driver misses (SURVEY.md
// Appendix A item 3); --file-order keeps the file's row order (maps only).
#include "cli_common.h"

int main(int argc, char **argv) {
  if (argc < 3) {
    printf("Syntax: %s inputfile num_runs [super_super_row_size super_row_size | super_row_size] [options]\n",
           argv[0]);
    return 0;
  }
  int first_opt = 3;
  int ssrs = 0, srs = 0, csr2 = 0;  // csr2: the super_row_size of the 3-argument form
  if (argc >= 5 && argv[3][0] != '-' && argv[4][0] != '-') {
    ssrs = atoi(argv[3]);
    srs = atoi(argv[4]);
    first_opt = 5;
  } else if (argc >= 4 && argv[3][0] != '-') {
    csr2 = atoi(argv[3]);
    first_opt = 4;
    if (csr2 < 1) {
      fprintf(stderr, "super_row_size must be >= 1\n");
      return 1;
    }
  }
  cli::Options o;
  o.kernel = HSPMV_KERNEL_CSR3;
  if (!cli::parse_options(argc, argv, first_opt, o)) return 1;
  const int num_runs = atoi(argv[2]);
  if (num_runs < 1) {
    fprintf(stderr, "num_runs must be >= 1\n");
    return 1;
  }
  hspmv_csr_buf A;
  hspmv_csr3_buf maps;
  std::vector<int32_t> perm;  // band-k: permuted row i = file row perm[i]
  if (cli::read_matrix(argv[1], o.dtype, A, maps) != HSPMV_OK) return cli::die("read");
  if (A.dtype != o.dtype) {
    fprintf(stderr, "matrix file holds dtype %d, requested %d\n", A.dtype, o.dtype);
    return 1;
  }
  if (maps.n_ssr == 0 && csr2 > 0) {
    // the reference's CSR-k driver banner (spmv-csrk/spmv.cpp:131-137)
    printf("SpMV\nHAND\n2\n%d\nRead in matrix and config file.\n", csr2);
    hspmv_csr view = {A.m, A.n, A.nnz, A.row_ptr, A.col_idx, A.val, A.dtype};
    auto tic = std::chrono::steady_clock::now();
    if (o.bandk && A.m == A.n) {
      hspmv_csr_buf P;
      perm.resize((size_t)A.m);
      if (hspmv_build_csr2_bandk(&view, csr2, &P, &maps, perm.data()) != HSPMV_OK)
        return cli::die("band-k build");
      hspmv_free_csr(&A);
      A = P;
    } else if (hspmv_build_csr2_maps(&view, csr2, &maps) != HSPMV_OK) {
      return cli::die("build maps");
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - tic).count();
    printf("%s reordered in %g seconds.\n", argv[1], dt);
  } else if (maps.n_ssr == 0) {
    if (ssrs <= 0 || srs <= 0) {
      const double d = A.m ? (double)A.nnz / (double)A.m : 1.0;
      const int flavour = o.params == "volta" ? 0 : (o.params == "mi100" ? 1 : 2);
      hspmv_csr3_params(d > 0 ? d : 1.0, flavour, &ssrs, &srs);
    }
    printf("using ssrs %d, srs %d\n", ssrs, srs);
    hspmv_csr view = {A.m, A.n, A.nnz, A.row_ptr, A.col_idx, A.val, A.dtype};
    auto tic = std::chrono::steady_clock::now();
    if (o.bandk && A.m == A.n) {
      hspmv_csr_buf P;
      perm.resize((size_t)A.m);
      if (hspmv_build_csr3_bandk(&view, ssrs, srs, &P, &maps, perm.data()) != HSPMV_OK)
        return cli::die("band-k build");
      hspmv_free_csr(&A);
      A = P;
    } else if (hspmv_build_csr3_maps(&view, ssrs, srs, &maps) != HSPMV_OK) {
      return cli::die("build maps");
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - tic).count();
    printf("%s reordered in %g seconds.\n", argv[1], dt);
  }
  printf("In CSR-k format.\n");
  printf("super-super-rows %lld super-rows %lld rows %lld nnz %lld\n", (long long)maps.n_ssr,
         (long long)maps.n_sr, (long long)A.m, (long long)A.nnz);
  const int rc = cli::run_and_report(A, &maps, num_runs, o, perm.empty() ? nullptr : perm.data());
  hspmv_free_csr3(&maps);
  hspmv_free_csr(&A);
  return rc;
}
