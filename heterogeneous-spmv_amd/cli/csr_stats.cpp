// csr-stats -- the reference's structural statistics tools over one reader:
//   csr-stats <file.csr | file.csr3>
// prints the keys of spmv-csr/stats.c:57-123 (.csr) and
// reformat-csr-to-csr3/stats.c:85-160 (.csr3, same statistics of the
// embedded CSR): NNZ Avg/Min/Max/Var, Band Avg/Max/Min/Var, Total NNZ, Dim.
// band(row) = last column - first column of the row.  Two reference quirks
// are kept so that the printed numbers agree: the percentages divide by m,
// and "Band Var" is the squared deviation of the LAST row only, / m (the
// loop assigns instead of accumulating, stats.c:112-116).  One is not: an
// empty row's band is 0 here (the reference reads the neighbouring rows'
// columns, or before the array for a leading empty row).  Host only.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "hspmv.h"

int main(int argc, char **argv) {
  if (argc < 2) {
    printf("%s inputfile.csr|inputfile.csr3\n", argv[0]);
    return 0;
  }
  const std::string path = argv[1];
  hspmv_csr_buf A;
  hspmv_csr3_buf maps;
  memset(&A, 0, sizeof(A));
  memset(&maps, 0, sizeof(maps));
  const bool csr3 = path.size() >= 5 && path.compare(path.size() - 5, 5, ".csr3") == 0;
  const int rc = csr3 ? hspmv_read_csr3(argv[1], HSPMV_F64, &A, &maps) : hspmv_read_csr(argv[1], HSPMV_F64, &A);
  if (rc != HSPMV_OK) {
    fprintf(stderr, "read failed: %s\n", hspmv_last_error());
    return 1;
  }
  const int64_t m = A.m, nnz = A.nnz;
  const double md = m > 0 ? (double)m : 1.0;
  const double avg = (double)nnz / md;
  int64_t min_nnz = nnz, max_nnz = 0, min_band = nnz, max_band = 0, sum_band = 0, last_band = 0;
  double var_nnz = 0.0;
  for (int64_t r = 0; r < m; ++r) {
    const int64_t len = A.row_ptr[r + 1] - A.row_ptr[r];
    const int64_t band = len > 0 ? (int64_t)A.col_idx[A.row_ptr[r + 1] - 1] - A.col_idx[A.row_ptr[r]] : 0;
    min_nnz = std::min(min_nnz, len);
    max_nnz = std::max(max_nnz, len);
    min_band = std::min(min_band, band);
    max_band = std::max(max_band, band);
    var_nnz += ((double)len - avg) * ((double)len - avg);
    sum_band += band;
    last_band = band;
  }
  const double avg_band = (double)sum_band / md;
  printf("NNZ Avg: %f \n", avg);
  printf("NNZ Min: %lld  Percent: %f \n", (long long)min_nnz, (double)min_nnz / md);
  printf("NNZ Max: %lld  Percent: %f \n", (long long)max_nnz, (double)max_nnz / md);
  printf("NNZ Var: %f \n", var_nnz / md);
  printf("Band Avg: %f \n", avg_band);
  printf("Band Max: %lld Percent: %f \n", (long long)max_band, (double)max_band / md);
  printf("Band Min: %lld Percent: %f \n", (long long)min_band, (double)min_band / md);
  printf("Band Var: %f \n", m > 0 ? ((double)last_band - avg_band) * ((double)last_band - avg_band) / md : 0.0);
  printf("Total NNZ: %lld\n", (long long)nnz);
  printf("Dim: %lldx%lld\n", (long long)A.m, (long long)A.n);
  if (csr3) printf("Super-super-rows: %lld Super-rows: %lld\n", (long long)maps.n_ssr, (long long)maps.n_sr);
  hspmv_free_csr3(&maps);
  hspmv_free_csr(&A);
  return 0;
}
