// hspmv_options.cpp -- hspmv_options -> the planner's Tuning
// (see hspmv_runtime.h for the split of the host runtime).
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <thread>
#include <vector>

#include "hspmv_runtime.h"

namespace hspmv {

// Planner options -> Tuning.  Fields past the caller's struct_size read as 0.
int tuning_from_options(const hspmv_options *o, Tuning *t) {
  *t = Tuning();
  if (!o) return HSPMV_OK;
  if (o->struct_size < offsetof(hspmv_options, csr3_plan))
    return set_error(HSPMV_E_INVALID, "hspmv_options.struct_size %u too small", o->struct_size);
  hspmv_options v;
  memset(&v, 0, sizeof(v));
  memcpy(&v, o, std::min<size_t>(o->struct_size, sizeof(v)));
  if (v.csr3_plan < 0 || v.csr3_plan > HSPMV_CSR3_PLAN_SSR)
    return set_error(HSPMV_E_INVALID, "csr3_plan %d unknown", v.csr3_plan);
  if ((v.csort_parts && v.csort_parts != 1 && v.csort_parts != 2 && v.csort_parts != 4) ||
      (v.csort_chunk_u && v.csort_chunk_u != 4 && v.csort_chunk_u != 8 && v.csort_chunk_u != 16) ||
      (v.stream_waves && v.stream_waves != 1 && v.stream_waves != 2 && v.stream_waves != 4) ||
      v.task_nnz < 0 || v.x_dict_cap < 0 || v.placement_trials < 0 || v.placement_trials > 8)
    return set_error(HSPMV_E_INVALID, "hspmv_options: value out of range");
  if (v.deterministic < 0 || v.deterministic > HSPMV_DETERMINISTIC_SERIAL)
    return set_error(HSPMV_E_INVALID, "deterministic %d unknown", v.deterministic);
  if ((v.deterministic == HSPMV_DETERMINISTIC_ORDERED || v.deterministic == HSPMV_DETERMINISTIC_SERIAL) &&
      v.csort > 0)
    return set_error(HSPMV_E_INVALID, "the column-sorted kernel (csort = 1) does not sum in omp_spmv's "
                                      "order (deterministic = 2 runs it with reproducible fixed-point sums)");
  t->csr3_plan = v.csr3_plan;
  t->task_nnz = v.task_nnz;
  t->x_windows = v.x_windows < 0 ? -1 : 0;
  t->x_dict = v.x_dict < 0 ? -1 : (v.x_dict > 0 ? 1 : 0);
  t->x_dict_cap = v.x_dict_cap;
  t->x_slabs = v.x_slabs < 0 ? -1 : v.x_slabs;
  t->col16_group = v.col16_group < 0 ? -1 : (v.col16_group > 0 ? 1 : 0);
  t->csort = v.csort < 0 ? -1 : (v.csort > 0 ? 1 : 0);
  t->csort_parts = v.csort_parts;
  t->csort_u = v.csort_chunk_u;
  t->stream_waves = v.stream_waves;
  t->deterministic = v.deterministic;
  t->placement_trials = v.placement_trials;
  return HSPMV_OK;
}

#ifdef HSPMV_ENV_KNOBS
// Diagnostic builds only (make diag-env): HSPMV_* environment variables
// override the options, for the A/B scripts under tools/.
void tuning_from_env(Tuning *t) {
  auto geti = [](const char *k, int *v) {
    if (const char *e = getenv(k)) *v = atoi(e);
  };
  if (const char *e = getenv("HSPMV_CSR3_PLAN"))
    t->csr3_plan = !strcmp(e, "ssr") ? HSPMV_CSR3_PLAN_SSR
                   : !strcmp(e, "packed") ? HSPMV_CSR3_PLAN_PACKED : HSPMV_CSR3_PLAN_ALIGNED;
  if (const char *e = getenv("HSPMV_TASK_FILL"))
    if (atoi(e) == 0) t->csr3_plan = HSPMV_CSR3_PLAN_PACKED;
  geti("HSPMV_TASK_NNZ", &t->task_nnz);
  if (const char *e = getenv("HSPMV_XWIN")) t->x_windows = atoi(e) == 0 ? -1 : 0;
  if (const char *e = getenv("HSPMV_XDICT")) t->x_dict = atoi(e) == 0 ? -1 : 1;
  geti("HSPMV_XDICT_CAP", &t->x_dict_cap);
  if (const char *e = getenv("HSPMV_XSLABS")) t->x_slabs = atoi(e) == 0 ? -1 : atoi(e);
  if (const char *e = getenv("HSPMV_XSLAB_BYTES")) t->xslab_bytes = atof(e);
  if (const char *e = getenv("HSPMV_COL16G")) t->col16_group = atoi(e) == 0 ? -1 : 1;
  if (const char *e = getenv("HSPMV_CSORT")) t->csort = atoi(e) == 0 ? -1 : 1;
  geti("HSPMV_CSORT_H", &t->csort_parts);
  geti("HSPMV_CSORT_U", &t->csort_u);
  geti("HSPMV_CSORT_NT", &t->csort_nt);
  geti("HSPMV_CSORT_PF", &t->csort_pf);
  geti("HSPMV_CSORT_BPC", &t->csort_blocks_per_cu);
  geti("HSPMV_CSORT_SLOT32", &t->csort_slot32);
  geti("HSPMV_CSORT_WIDE", &t->csort_wide);
  geti("HSPMV_CSORT_LDS", &t->csort_lds_cap);
  geti("HSPMV_CSORT_SEG", &t->csort_seg);
  geti("HSPMV_CSORT_SEG_EXTRA", &t->csort_seg_extra);
  geti("HSPMV_CSORT_TRACE", &t->csort_trace);
  geti("HSPMV_CSORT_LONG", &t->csort_long);
  geti("HSPMV_CSORT_BALANCE", &t->csort_balance);
  geti("HSPMV_CSORT_FIN_ROWS", &t->csort_fin_rows);
  geti("HSPMV_CSORT_DYN", &t->csort_dyn);
  if (const char *e = getenv("HSPMV_CSORT_SWEEP")) t->csort_sweep_w = atof(e);
  if (const char *e = getenv("HSPMV_CSORT_SLACK")) t->csort_slack = atof(e);
  geti("HSPMV_CSORT_PART32", &t->csort_part32);
  geti("HSPMV_DETERMINISTIC", &t->deterministic);
  geti("HSPMV_SERIAL_MAX", &t->serial_max);
  geti("HSPMV_LDS_PAD", &t->lds_pad);
  geti("HSPMV_STREAM_W", &t->stream_waves);
  geti("HSPMV_PLACEMENT", &t->placement_trials);
  geti("HSPMV_SSR_ALIGN", &t->ssr_align);
  geti("HSPMV_SSR_W", &t->ssr_w);
  geti("HSPMV_CONTIG", &t->contig);
  geti("HSPMV_XD_WAVES", &t->xd_waves);
  geti("HSPMV_XD_BPC", &t->xd_blocks_per_cu);
  geti("HSPMV_PF", &t->pf);
  geti("HSPMV_YNT", &t->y_nt);
  geti("HSPMV_NT", &t->nt);
  geti("HSPMV_DYNLDS", &t->dyn_lds);
}
#else
void tuning_from_env(Tuning *) {}
#endif

// The kernel rules of hspmv_options.deterministic 1 and 3 (checked at
// creation, whatever set the mode): no CSORT (its sums do not follow
// omp_spmv's order); SERIAL also no VECTOR (shuffle trees).  SERIAL's rows
// over kLongRow nonzeros go to hspmv_long_serial (one workgroup per row,
// still one add at a time in order), or with HSPMV_FLAG_NO_SPLIT stay in the
// row kernels' lanes.
int check_deterministic(unsigned flags, const Tuning &t) {
  const unsigned k = flags & 0xFu;
  if ((t.deterministic == HSPMV_DETERMINISTIC_ORDERED || t.deterministic == HSPMV_DETERMINISTIC_SERIAL) &&
      k == kCsort)
    return set_error(HSPMV_E_INVALID, "the column-sorted kernel (HSPMV_KERNEL_CSORT) does not sum in "
                                      "omp_spmv's order (deterministic = 2 runs it with reproducible "
                                      "fixed-point sums)");
  if (t.deterministic == HSPMV_DETERMINISTIC_SERIAL) {
    if (k == kVector)
      return set_error(HSPMV_E_INVALID, "deterministic = 3 (serial order) runs the row kernels only: "
                                        "HSPMV_KERNEL_VECTOR sums each row in a shuffle tree");
  }
  return HSPMV_OK;
}

Tuning default_tuning() {
  Tuning t;
  tuning_from_env(&t);  // no-op outside diagnostic builds
  return t;
}

}  // namespace hspmv
