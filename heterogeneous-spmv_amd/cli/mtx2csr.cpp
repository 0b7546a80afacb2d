// mtx2csr -- the reference's Octave converter (helpers/converter.m:1-50,
// run by helpers/run_converter.sh) for one Matrix Market file:
//   mtx2csr <in.mtx> <out.csr> [<out.rcm.csr>]
// reads the file as mmread.m does (hspmv_read_mtx), writes it as .csr
// (helpers/sparse2csr.m layout: "m n nnz", then row_ptr, col_ind and "%f"
// values, 0-based), and with a third argument also the reverse
// Cuthill-McKee ordering of it (converter.m:14-15, symrcm; hspmv_rcm_reorder,
// whose tie-breaking is not Octave's).  converter.m walks a directory
// (~/matrices/mm/*.mtx -> norm/X.mtx.csr and rcm/X.mtx.rcm.csr); a shell
// loop over this tool does the same.  An output named *.bin is written as
// the binary cache instead of text (hspmv_save_bin).  Host only.
#include <stdio.h>
#include <string.h>

#include <chrono>

#include "hspmv.h"

// ".bin" outputs get the binary cache (hspmv_save_bin: what spmv-csr /
// spmv-csrk load fastest), anything else the reference's text .csr
static int write_out(const char *path, const hspmv_csr *A) {
  const size_t n = strlen(path);
  if (n >= 4 && strcmp(path + n - 4, ".bin") == 0) return hspmv_save_bin(path, A, nullptr);
  return hspmv_write_csr(path, A);
}

static int die(const char *what) {
  fprintf(stderr, "%s failed: %s\n", what, hspmv_last_error());
  return 1;
}

int main(int argc, char **argv) {
  if (argc < 3) {
    printf("Syntax: %s input.mtx output.csr [output.rcm.csr]\n", argv[0]);
    return 0;
  }
  const char *name = strrchr(argv[1], '/');
  name = name ? name + 1 : argv[1];
  hspmv_csr_buf A;
  memset(&A, 0, sizeof(A));
  printf("Converting matrix %s...", name);
  fflush(stdout);
  if (hspmv_read_mtx(argv[1], HSPMV_F64, &A) != HSPMV_OK) return die("\nread");
  const hspmv_csr view = {A.m, A.n, A.nnz, A.row_ptr, A.col_idx, A.val, A.dtype};
  hspmv_csr_buf R;
  memset(&R, 0, sizeof(R));
  const bool rcm = argc >= 4;
  if (rcm) {
    const auto tic = std::chrono::steady_clock::now();
    if (hspmv_rcm_reorder(&view, &R, nullptr) != HSPMV_OK) {
      hspmv_free_csr(&A);
      return die("\nRCM");
    }
    printf("reordered in %f...", std::chrono::duration<double>(std::chrono::steady_clock::now() - tic).count());
  }
  if (write_out(argv[2], &view) != HSPMV_OK) {
    hspmv_free_csr(&R);
    hspmv_free_csr(&A);
    return die("\nwrite");
  }
  printf("converted original to csr...wrote row_ptr...wrote col_ind...wrote val...");
  int rc = 0;
  if (rcm) {
    const hspmv_csr rv = {R.m, R.n, R.nnz, R.row_ptr, R.col_idx, R.val, R.dtype};
    if (write_out(argv[3], &rv) != HSPMV_OK)
      rc = die("\nwrite");
    else
      printf("converted reordered to csr...wrote row_ptr...wrote col_ind...wrote val...");
  }
  if (rc == 0) printf("done\n");
  hspmv_free_csr(&R);
  hspmv_free_csr(&A);
  return rc;
}
