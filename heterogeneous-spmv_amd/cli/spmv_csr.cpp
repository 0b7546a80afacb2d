// spmv-csr -- MI355X CSR SpMV benchmark driver.
// Same command line and timing output as the reference's spmv-csr/spmv.exe
// (spmv-csr/spmv.c:116-225) and cuda-spmv-csr/spmv.exe
// (cuda-spmv-csr/spmv.cu:185-305):
//     spmv-csr <file.csr> <num_runs> [options]      (options: cli_common.h)
// The SpMV runs on the GPU through libhspmv (include/hspmv.h).
#include "cli_common.h"

int main(int argc, char **argv) {
  if (argc < 3) {
    printf("%s inputfile.csr num_runs [--gpus N] [--dtype f32|f64] [--x ones|rand:SEED] "
           "[--kernel auto|stream|vector[:L]] [--nt] [--dump-y PATH] [--no-check]\n",
           argv[0]);
    return 0;
  }
  cli::Options o;
  if (!cli::parse_options(argc, argv, 3, o)) return 1;
  const int num_runs = atoi(argv[2]);
  if (num_runs < 1) {
    fprintf(stderr, "num_runs must be >= 1\n");
    return 1;
  }
  printf("Before Read\n");
  hspmv_csr_buf A;
  hspmv_csr3_buf maps;
  if (cli::read_matrix(argv[1], o.dtype, A, maps) != HSPMV_OK) return cli::die("read");
  printf("After Read\n");
  if (A.dtype != o.dtype) {
    fprintf(stderr, "matrix file holds dtype %d, requested %d\n", A.dtype, o.dtype);
    return 1;
  }
  hspmv_free_csr3(&maps);  // spmv-csr runs plain CSR even on a .csr3 input
  printf("m %lld n %lld nnz %lld index_base %d\n", (long long)A.m, (long long)A.n,
         (long long)A.nnz, A.index_base);
  const int rc = cli::run_and_report(A, nullptr, num_runs, o);
  printf("TEAST\n");
  hspmv_free_csr(&A);
  return rc;
}
