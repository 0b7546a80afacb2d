// hspmv_mtx.cpp -- Matrix Market reader: the input side of the reference's
// pipeline, whose Octave helpers turn SuiteSparse .mtx files into the .csr
// files every driver reads (helpers/converter.m:1-50 with helpers/mmread.m
// and helpers/sparse2csr.m).  Octave is not needed here.
//
// Semantics follow mmread.m + Octave's sparse():
//   * "coordinate" files, field real | integer | pattern (pattern -> 1.0),
//     symmetry general | symmetric | skew-symmetric (mmread.m:85-130);
//     array (dense) and complex files are refused;
//   * duplicates are summed and exact zeros dropped (sparse(i, j, v, m, n));
//   * symmetric: A + A.' - diag(diag(A)) (mmread.m:207-209), i.e. every
//     stored off-diagonal entry mirrored; skew-symmetric: A - A.';
//   * rows in order, columns sorted within a row (sparse2csr.m: find(A.')).
// The nonzero count is the CSR's own; converter.m writes mmread's
// `entries`, which for a general file is the line count even when
// duplicates or zeros made the CSR shorter (a header the reference's own
// reader would then misparse).
//
// The entry lines are parsed in parallel (split at line boundaries,
// std::from_chars), then bucketed by row with a counting sort.
#include <errno.h>
#include <locale.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cctype>
#include <charconv>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "hspmv_common.h"

using namespace hspmv;

namespace {

struct Entry {
  int32_t r, c;
  double v;
};

inline bool blank(char ch) { return ch == ' ' || ch == '\t' || ch == '\r'; }

// One entry line [p, e): "i j [v]" (1-based).  Returns false if malformed or
// if an index lies outside 1..rows / 1..cols (checked on the 64-bit values,
// before narrowing to int32: 4294967297 must not wrap to row 0).
bool parse_line(const char *p, const char *e, bool pattern, long long rows, long long cols, Entry *out) {
  long long ij[2];
  for (int t = 0; t < 2; ++t) {
    while (p < e && blank(*p)) ++p;
    auto r = std::from_chars(p, e, ij[t]);
    if (r.ec != std::errc()) return false;
    p = r.ptr;
  }
  if (ij[0] < 1 || ij[0] > rows || ij[1] < 1 || ij[1] > cols) return false;
  double v = 1.0;
  if (!pattern) {
    while (p < e && blank(*p)) ++p;
    auto r = std::from_chars(p, e, v);
    if (r.ec == std::errc::result_out_of_range) {
      // from_chars leaves v unset here; strtod gives what mmread's fscanf
      // gives: +-HUGE_VAL on overflow, a denormal or +-0 on underflow.  The
      // whole token (any length: a 400-digit literal must overflow, not be
      // cut to 127 digits) in the C locale (a comma-decimal LC_NUMERIC must
      // not stop the parse at the '.').
      static const locale_t c_loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
      const std::string tok(p, r.ptr);
      v = strtod_l(tok.c_str(), nullptr, c_loc);
    } else if (r.ec != std::errc()) {
      return false;
    }
  }
  out->r = (int32_t)(ij[0] - 1);
  out->c = (int32_t)(ij[1] - 1);
  out->v = v;
  return true;
}

int threads() {
  const unsigned hc = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(16u, hc ? hc : 4u));
}

}  // namespace

extern "C" int hspmv_read_mtx(const char *path, int dtype, hspmv_csr_buf *out) {
  clear_error();
  if (!path || !out) return set_error(HSPMV_E_INVALID, "NULL argument");
  if (dtype != HSPMV_F32 && dtype != HSPMV_F64) return set_error(HSPMV_E_INVALID, "bad dtype");
  memset(out, 0, sizeof(*out));
  FILE *fp = fopen(path, "rb");
  if (!fp) return set_error(HSPMV_E_IO, "cannot open %s: %s", path, strerror(errno));
  fseek(fp, 0, SEEK_END);
  const long sz = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  std::vector<char> buf((size_t)std::max(sz, 0L) + 1);
  const size_t got = sz > 0 ? fread(buf.data(), 1, (size_t)sz, fp) : 0;
  fclose(fp);
  buf[got] = '\n';
  const char *p = buf.data(), *end = buf.data() + got;
  auto next_line = [&](const char *q) {
    while (q < end && *q != '\n') ++q;
    return q < end ? q + 1 : end;
  };
  // banner: %%MatrixMarket matrix <format> <field> <symmetry>
  const char *le = next_line(p);
  std::string banner(p, le);
  for (auto &ch : banner) ch = (char)tolower((unsigned char)ch);
  char obj[32] = {0}, fmt[32] = {0}, field[32] = {0}, symm[32] = {0};
  if (sscanf(banner.c_str(), "%%%%matrixmarket %31s %31s %31s %31s", obj, fmt, field, symm) != 4 ||
      strcmp(obj, "matrix") != 0)
    return set_error(HSPMV_E_IO, "%s: not a MatrixMarket matrix file", path);
  if (strcmp(fmt, "coordinate") != 0)
    return set_error(HSPMV_E_INVALID, "%s: %s format (only coordinate files are sparse matrices)", path, fmt);
  const bool pattern = strcmp(field, "pattern") == 0;
  if (!pattern && strcmp(field, "real") != 0 && strcmp(field, "integer") != 0 && strcmp(field, "double") != 0)
    return set_error(HSPMV_E_INVALID, "%s: %s field not supported (real, integer, pattern)", path, field);
  const int sym = strcmp(symm, "general") == 0 ? 0 : strcmp(symm, "symmetric") == 0 ? 1
                  : strcmp(symm, "skew-symmetric") == 0 ? -1 : 2;
  if (sym == 2) return set_error(HSPMV_E_INVALID, "%s: %s symmetry not supported", path, symm);
  // comments, then the size line "rows cols entries"
  p = le;
  long long rows = -1, cols = -1, ents = -1;
  while (p < end) {
    le = next_line(p);
    const char *q = p;
    while (q < le && (blank(*q) || *q == '\n')) ++q;
    if (q < le && *q != '%') {
      if (sscanf(q, "%lld %lld %lld", &rows, &cols, &ents) != 3)
        return set_error(HSPMV_E_IO, "%s: malformed size line", path);
      p = le;
      break;
    }
    p = le;
  }
  if (rows < 0 || cols < 0 || ents < 0) return set_error(HSPMV_E_IO, "%s: no size line", path);
  if (rows >= INT32_MAX || cols >= INT32_MAX || ents >= INT32_MAX / 2)
    return set_error(HSPMV_E_INVALID, "%s: too large for int32 indices", path);
  if (sym != 0 && rows != cols) return set_error(HSPMV_E_INVALID, "%s: %s but not square", path, symm);
  // entry lines, parsed in parallel between line boundaries
  const int T = threads();
  std::vector<const char *> cut((size_t)T + 1);
  cut[0] = p;
  cut[(size_t)T] = end;
  for (int t = 1; t < T; ++t) {
    const char *q = p + (size_t)(end - p) * (size_t)t / (size_t)T;
    if (q < cut[(size_t)t - 1]) q = cut[(size_t)t - 1];
    cut[(size_t)t] = q > p ? next_line(q - 1) : p;  // the start of the line holding q
  }
  std::vector<std::vector<Entry>> part((size_t)T);
  std::vector<int> bad((size_t)T, 0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        const char *q = cut[(size_t)t], *e = cut[(size_t)t + 1];
        auto &v = part[(size_t)t];
        v.reserve((size_t)(ents / T + 16));
        while (q < e) {
          const char *l = q;
          while (l < e && *l != '\n') ++l;
          const char *s = q;
          while (s < l && blank(*s)) ++s;
          if (s < l && *s != '%') {
            Entry en;
            if (!parse_line(s, l, pattern, rows, cols, &en)) {
              bad[(size_t)t] = 1;
              return;
            }
            v.push_back(en);
          }
          q = l + 1;
        }
      });
    for (auto &x : th) x.join();
  }
  int64_t seen = 0;
  for (int t = 0; t < T; ++t) {
    if (bad[(size_t)t]) return set_error(HSPMV_E_IO, "%s: malformed or out-of-range entry line", path);
    seen += (int64_t)part[(size_t)t].size();
  }
  if (seen != ents)
    return set_error(HSPMV_E_IO, "%s: %lld entry lines, the size line says %lld", path, (long long)seen, ents);
  // counting sort by row (mirrored entries included), then per-row column
  // sort, duplicate sums and zero removal
  const int64_t m = rows;
  std::vector<int64_t> cnt((size_t)m + 1, 0);
  for (const auto &v : part)
    for (const Entry &en : v) {
      ++cnt[(size_t)en.r + 1];
      if (sym != 0 && en.r != en.c) ++cnt[(size_t)en.c + 1];
    }
  for (int64_t i = 0; i < m; ++i) cnt[(size_t)i + 1] += cnt[(size_t)i];
  if (cnt[(size_t)m] >= INT32_MAX) return set_error(HSPMV_E_INVALID, "%s: too many nonzeros for int32", path);
  std::vector<std::pair<int32_t, double>> rowbuf((size_t)cnt[(size_t)m]);
  {
    std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
    for (const auto &v : part)
      for (const Entry &en : v) {
        // skew-symmetric: a stored diagonal entry cancels in A - A.' (0 is dropped)
        rowbuf[(size_t)fill[(size_t)en.r]++] = {en.c, sym < 0 && en.r == en.c ? 0.0 : en.v};
        if (sym != 0 && en.r != en.c) rowbuf[(size_t)fill[(size_t)en.c]++] = {en.r, sym > 0 ? en.v : -en.v};
      }
  }
  std::vector<std::vector<Entry>>().swap(part);
  std::vector<int32_t> rlen((size_t)m, 0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        for (int64_t r = m * t / T; r < m * (t + 1) / T; ++r) {
          auto b = rowbuf.begin() + cnt[(size_t)r], e = rowbuf.begin() + cnt[(size_t)r + 1];
          std::stable_sort(b, e, [](const auto &x, const auto &y) { return x.first < y.first; });
          auto w = b;
          for (auto it = b; it != e;) {
            auto jt = it;
            double s = 0.0;
            for (; jt != e && jt->first == it->first; ++jt) s += jt->second;
            if (s != 0.0) *w++ = {it->first, s};
            it = jt;
          }
          rlen[(size_t)r] = (int32_t)(w - b);
        }
      });
    for (auto &x : th) x.join();
  }
  int64_t nnz = 0;
  for (int64_t r = 0; r < m; ++r) nnz += rlen[(size_t)r];
  int32_t *rp = (int32_t *)malloc(4 * (size_t)(m + 1));
  int32_t *ci = (int32_t *)malloc(4 * (size_t)(nnz ? nnz : 1));
  void *val = malloc(dtype_size(dtype) * (size_t)(nnz ? nnz : 1));
  if (!rp || !ci || !val) {
    free(rp);
    free(ci);
    free(val);
    return set_error(HSPMV_E_NOMEM, "out of host memory reading %s", path);
  }
  rp[0] = 0;
  for (int64_t r = 0; r < m; ++r) rp[r + 1] = rp[r] + rlen[(size_t)r];
  for (int64_t r = 0; r < m; ++r) {
    const int64_t src = cnt[(size_t)r];
    for (int32_t k = 0; k < rlen[(size_t)r]; ++k) {
      const auto &e = rowbuf[(size_t)(src + k)];
      ci[rp[r] + k] = e.first;
      if (dtype == HSPMV_F64)
        ((double *)val)[rp[r] + k] = e.second;
      else
        ((float *)val)[rp[r] + k] = (float)e.second;
    }
  }
  out->m = m;
  out->n = cols;
  out->nnz = nnz;
  out->row_ptr = rp;
  out->col_idx = ci;
  out->val = val;
  out->dtype = dtype;
  out->index_base = 1;
  return HSPMV_OK;
}
