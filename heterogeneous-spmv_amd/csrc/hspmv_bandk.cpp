// hspmv_bandk.cpp -- the CSR-3 builder with the reference's full band-k
// semantics: hand-coarsening of the row graph into
// super-rows, RCM on every coarse graph, coarsening again into super-super-
// rows, uncoarsening into one symmetric permutation, and the permuted
// matrix with sorted columns.  Restated from BAND_k::preprocessingForSpMV
// (cuda-spmv-csrk/hip/csrk.cu:1035-1262) and the routines it calls, in the
// same order of operations (std::sort with the same comparators on the same
// sequences, so tie-breaking follows the reference's):
//   handCoarsen                         csrk.cu:1438-1629
//   rcm_reordering_g                    csrk.cu:2483-2568
//   findPseudoPeripheralVertex          csrk.cu:2571-2615
//   findRootedLevelStructures           csrk.cu:2620-2669
//   renumberGraphUsingReorderedVertices csrk.cu:3206-3309
//   uncoarsenTheGraph                   csrk.cu:1343-1419
//   reorderA                            csrk.cu:722-870
// Deviation kept from hspmv_build_csr3_maps: the last group is closed when it
// holds rows (not only nonzeros), so a trailing run of empty rows is mapped.
#include <string.h>

#include <algorithm>
#include <cstdlib>
#include <numeric>
#include <thread>
#include <vector>

#include "hspmv_common.h"

using namespace hspmv;

namespace {

// An undirected (symmetrised) graph with edge multiplicities, as the
// reference's smallGraphs[level] (r_vec, c_vec, degree).
struct Graph {
  int64_t n = 0;
  std::vector<int64_t> r;    // n + 1
  std::vector<int32_t> c;    // adjacency (sorted ascending per vertex)
  std::vector<int32_t> deg;  // multiplicity of each adjacency entry
};

// handCoarsen (csrk.cu:1438-1629): groups consecutive vertices while the
// running row length is below `thr`; builds the coarse graph from every
// edge i -> c with c >= start of i's group (both directions when the groups
// differ), then sorts and de-duplicates each adjacency list, the duplicate
// count becoming the edge's multiplicity.
void hand_coarsen(const Graph &g, int64_t thr, std::vector<int32_t> *starts, Graph *cg) {
  const int64_t N = g.n;
  starts->assign(1, 0);
  int64_t acc = 0, last = 0, ng = 0;
  std::vector<int32_t> sup((size_t)N);
  for (int64_t i = 0; i < N; ++i) {
    const int64_t len = g.r[i + 1] - g.r[i];
    if (acc < thr) {
      acc += len;
    } else {
      ++ng;
      acc = len;
      last = i;
      starts->push_back((int32_t)i);
    }
    sup[(size_t)i] = (int32_t)ng;
  }
  if (N > last) {
    ++ng;
    starts->push_back((int32_t)N);
  }
  if (N == 0) ng = 0;
  // coarse adjacency with multiplicities (two passes, as csrk.cu:1487-1567)
  std::vector<int64_t> cnt((size_t)ng + 1, 0);
  for (int64_t s = 0; s < ng; ++s)
    for (int32_t i = (*starts)[s]; i < (*starts)[s + 1]; ++i)
      for (int64_t k = g.r[i]; k < g.r[i + 1]; ++k) {
        const int32_t col = g.c[k];
        if (col >= (*starts)[s]) {
          const int32_t t = sup[(size_t)col];
          ++cnt[(size_t)s];
          if (t != s) ++cnt[(size_t)t];
        }
      }
  std::vector<int64_t> cr((size_t)ng + 1, 0);
  for (int64_t s = 0; s < ng; ++s) cr[s + 1] = cr[s] + cnt[s];
  std::vector<int32_t> cc((size_t)cr[ng]);
  std::vector<int64_t> fill(cr.begin(), cr.end() - 1);
  for (int64_t s = 0; s < ng; ++s)
    for (int32_t i = (*starts)[s]; i < (*starts)[s + 1]; ++i)
      for (int64_t k = g.r[i]; k < g.r[i + 1]; ++k) {
        const int32_t col = g.c[k];
        if (col >= (*starts)[s]) {
          const int32_t t = sup[(size_t)col];
          if (t == s) {
            cc[(size_t)fill[s]++] = (int32_t)s;
          } else {
            cc[(size_t)fill[s]++] = t;
            cc[(size_t)fill[t]++] = (int32_t)s;
          }
        }
      }
  cg->n = ng;
  cg->r.assign((size_t)ng + 1, 0);
  cg->c.clear();
  cg->deg.clear();
  for (int64_t s = 0; s < ng; ++s) {
    std::sort(cc.begin() + cr[s], cc.begin() + cr[s + 1]);
    for (int64_t k = cr[s]; k < cr[s + 1]; ++k) {
      if (k > cr[s] && cc[(size_t)k] == cc[(size_t)k - 1]) {
        ++cg->deg.back();
      } else {
        cg->c.push_back(cc[(size_t)k]);
        cg->deg.push_back(1);
      }
    }
    cg->r[s + 1] = (int64_t)cg->c.size();
  }
}

// findRootedLevelStructures (csrk.cu:2620-2669): BFS levels from `root` over
// vertices with mask != 0; leaves the mask as it found it.
void rooted_levels(int32_t root, const Graph &g, std::vector<int32_t> &mask, int &num_lvls,
                   std::vector<int32_t> &lr, std::vector<int32_t> &lc) {
  mask[(size_t)root] = 0;
  num_lvls = 0;
  int64_t level_end = 0, cc_size = 1, level_size = 1;
  lc[0] = root;
  while (level_size > 0) {
    const int64_t level_begin = level_end;
    lr[(size_t)num_lvls] = (int32_t)level_begin;
    level_end = cc_size;
    for (int64_t i = level_begin; i < level_end; ++i) {
      const int32_t v = lc[(size_t)i];
      for (int64_t k = g.r[v]; k < g.r[v + 1]; ++k) {
        const int32_t nb = g.c[(size_t)k];
        if (mask[(size_t)nb] != 0) {
          lc[(size_t)cc_size++] = nb;
          mask[(size_t)nb] = 0;
        }
      }
    }
    level_size = cc_size - level_end;
    ++num_lvls;
  }
  lr[(size_t)num_lvls] = (int32_t)level_end;
  for (int64_t i = 0; i < cc_size; ++i) mask[(size_t)lc[(size_t)i]] = 1;
}

// findPseudoPeripheralVertex (csrk.cu:2571-2615).
void pseudo_peripheral(int32_t &root, const Graph &g, std::vector<int32_t> &mask,
                       std::vector<int32_t> &lr, std::vector<int32_t> &lc) {
  int num_lvls = 0, new_lvls = 0;
  rooted_levels(root, g, mask, num_lvls, lr, lc);
  const int32_t cc_size = lr[(size_t)num_lvls];
  if (num_lvls == 1 || num_lvls == cc_size) return;
  while (true) {
    const int32_t j1 = lr[(size_t)num_lvls - 1];
    int32_t min_deg = cc_size;
    root = lc[(size_t)j1];
    if (cc_size != j1) {
      for (int32_t j = j1; j < cc_size; ++j) {
        const int32_t v = lc[(size_t)j];
        int32_t d = 0;
        for (int64_t k = g.r[v]; k < g.r[v + 1]; ++k)
          if (mask[(size_t)g.c[(size_t)k]] > 0) ++d;
        if (d < min_deg) {
          root = v;
          min_deg = d;
        }
      }
    }
    rooted_levels(root, g, mask, new_lvls, lr, lc);
    if (new_lvls <= num_lvls || num_lvls >= cc_size) return;
    num_lvls = new_lvls;
  }
}

// rcm_reordering_g (csrk.cu:2483-2568) called per connected component, as
// preprocessingForSpMV does (csrk.cu:1112-1127): BFS from a pseudo-peripheral
// vertex, children in decreasing edge multiplicity (std::sort, the
// reference's comparator), a vertex placed when dequeued; each component's
// order reversed.  new_to_old / old_to_new: the permutation.
void rcm(const Graph &g, std::vector<int32_t> &new_to_old, std::vector<int32_t> &old_to_new) {
  const int64_t n = g.n;
  new_to_old.assign((size_t)n, 0);
  old_to_new.assign((size_t)n, 0);
  std::vector<int32_t> mask((size_t)n, 1), lr((size_t)n + 1), lc((size_t)n + 1);
  std::vector<int32_t> queue((size_t)std::max<int64_t>(g.r[n], n) + 1);
  struct RevDeg {
    int32_t deg, id;
  };
  std::vector<RevDeg> kids;
  int64_t cc_size = 0;
  for (int64_t i_mask = 0; i_mask < n; ++i_mask) {
    if (cc_size >= n) break;
    if (mask[(size_t)i_mask] == 0) continue;
    int32_t root = (int32_t)i_mask;
    pseudo_peripheral(root, g, mask, lr, lc);
    size_t qh = 0, qt = 0;
    queue[qt++] = root;
    int64_t visited = 0, pos = cc_size;
    while (qh < qt) {
      const int32_t p = queue[qh++];
      if (mask[(size_t)p] != 1) continue;
      mask[(size_t)p] = 0;
      new_to_old[(size_t)pos++] = p;
      ++visited;
      kids.clear();
      for (int64_t k = g.r[p]; k < g.r[p + 1]; ++k) {
        const int32_t a = g.c[(size_t)k];
        if (mask[(size_t)a] == 1) kids.push_back({g.deg[(size_t)k], a});
      }
      std::sort(kids.begin(), kids.end(),
                [](const RevDeg &l, const RevDeg &r) { return l.deg > r.deg; });
      for (const RevDeg &kd : kids) {
        if (qt == queue.size()) queue.resize(queue.size() * 2);
        queue[qt++] = kd.id;
      }
    }
    // reverse this component's segment
    const int64_t mid = visited / 2;
    int64_t last = pos - 1;
    for (int64_t i = 0; i < mid; ++i) {
      std::swap(new_to_old[(size_t)last], new_to_old[(size_t)(cc_size + i)]);
      old_to_new[(size_t)new_to_old[(size_t)last]] = (int32_t)last;
      old_to_new[(size_t)new_to_old[(size_t)(cc_size + i)]] = (int32_t)(cc_size + i);
      --last;
    }
    if (visited % 2 == 1)
      old_to_new[(size_t)new_to_old[(size_t)(cc_size + mid)]] = (int32_t)(cc_size + mid);
    cc_size += visited;
  }
}

// renumberGraphUsingReorderedVertices (csrk.cu:3206-3309): vertex i of the
// new graph is old vertex new_to_old[i]; adjacency mapped and re-sorted.
void renumber(Graph &g, const std::vector<int32_t> &new_to_old,
              const std::vector<int32_t> &old_to_new) {
  Graph h;
  h.n = g.n;
  h.r.assign((size_t)g.n + 1, 0);
  h.c.resize(g.c.size());
  h.deg.resize(g.deg.size());
  for (int64_t i = 0; i < g.n; ++i) {
    const int32_t o = new_to_old[(size_t)i];
    h.r[i + 1] = h.r[i] + (g.r[o + 1] - g.r[o]);
  }
  std::vector<std::pair<int32_t, int32_t>> row;
  for (int64_t i = 0; i < g.n; ++i) {
    const int32_t o = new_to_old[(size_t)i];
    row.clear();
    for (int64_t k = g.r[o]; k < g.r[o + 1]; ++k)
      row.push_back({old_to_new[(size_t)g.c[(size_t)k]], g.deg[(size_t)k]});
    std::sort(row.begin(), row.end(),
              [](const std::pair<int32_t, int32_t> &a, const std::pair<int32_t, int32_t> &b) {
                return a.first < b.first;
              });
    for (size_t t = 0; t < row.size(); ++t) {
      h.c[(size_t)h.r[i] + t] = row[t].first;
      h.deg[(size_t)h.r[i] + t] = row[t].second;
    }
  }
  g = std::move(h);
}

// uncoarsenTheGraph (csrk.cu:1343-1419): the coarse level's group ranges
// rewritten in the coarse permutation's order, and the finer level's
// permutation composed with the resulting order of its vertices.
void uncoarsen(std::vector<int32_t> &map, const std::vector<int32_t> &perm_coarse,
               std::vector<int32_t> &perm_finer) {
  const size_t ns = perm_coarse.size();
  const std::vector<int32_t> old_map = map;
  map[0] = 0;
  for (size_t i = 0; i < ns; ++i) {
    const int32_t o = perm_coarse[i];
    map[i + 1] = map[i] + (old_map[(size_t)o + 1] - old_map[(size_t)o]);
  }
  std::vector<int32_t> np(perm_finer.size());
  for (size_t i = 0; i < ns; ++i) {
    const int32_t o = perm_coarse[i];
    int32_t at = map[i];
    for (int32_t j = old_map[(size_t)o]; j < old_map[(size_t)o + 1]; ++j) np[(size_t)at++] = j;
  }
  const std::vector<int32_t> old_perm = perm_finer;
  for (size_t i = 0; i < perm_finer.size(); ++i) perm_finer[i] = old_perm[(size_t)np[i]];
}

// body(r0, r1) over [0, n) split into contiguous ranges, one thread each.
template <typename F>
void par_ranges(int64_t n, F body) {
  const unsigned hc = std::thread::hardware_concurrency();
  const int64_t T = std::max<int64_t>(1, std::min<int64_t>({16, hc ? (int64_t)hc : 4, n / 65536 + 1}));
  std::vector<std::thread> th;
  for (int64_t t = 1; t < T; ++t) th.emplace_back([&, t]() { body(n * t / T, n * (t + 1) / T); });
  body(0, n / T);
  for (auto &x : th) x.join();
}

// reorderA (csrk.cu:722-870): new row i = row perm0[i] of A, columns
// renumbered by the inverse permutation and sorted per row, values moved.
int permute_symmetric(const hspmv_csr *A, const std::vector<int32_t> &perm0, hspmv_csr_buf *A_out) {
  const int64_t m = A->m, nnz = A->nnz;
  std::vector<int32_t> fwd((size_t)m);
  for (int64_t i = 0; i < m; ++i) fwd[(size_t)perm0[(size_t)i]] = (int32_t)i;
  const size_t sv = dtype_size(A->dtype);
  A_out->m = m;
  A_out->n = m;
  A_out->nnz = nnz;
  A_out->dtype = A->dtype;
  A_out->row_ptr = (int32_t *)malloc(4 * (size_t)(m + 1));
  A_out->col_idx = (int32_t *)malloc(4 * (size_t)(nnz ? nnz : 1));
  A_out->val = malloc(sv * (size_t)(nnz ? nnz : 1));
  if (!A_out->row_ptr || !A_out->col_idx || !A_out->val) {
    hspmv_free_csr(A_out);
    return set_error(HSPMV_E_NOMEM, "out of host memory");
  }
  A_out->row_ptr[0] = 0;
  for (int64_t i = 0; i < m; ++i) {
    const int32_t o = perm0[(size_t)i];
    A_out->row_ptr[i + 1] = A_out->row_ptr[i] + (A->row_ptr[o + 1] - A->row_ptr[o]);
  }
  // rows are independent: row ranges in parallel (the .csr3 builds of the
  // 50-200 M-nonzero configurations spend most of their time here)
  par_ranges(m, [&](int64_t r0, int64_t r1) {
    std::vector<std::pair<int32_t, int32_t>> row;
    for (int64_t i = r0; i < r1; ++i) {
      const int32_t o = perm0[(size_t)i];
      row.clear();
      for (int32_t k = A->row_ptr[o]; k < A->row_ptr[o + 1]; ++k) row.push_back({fwd[(size_t)A->col_idx[k]], k});
      std::sort(row.begin(), row.end());
      int32_t at = A_out->row_ptr[i];
      for (const auto &e : row) {
        A_out->col_idx[at] = e.first;
        memcpy((char *)A_out->val + sv * (size_t)at, (const char *)A->val + sv * (size_t)e.second, sv);
        ++at;
      }
    }
  });
  return HSPMV_OK;
}

// levels = 3: CSR-3 (sizes s1 then s2, two coarsenings); levels = 2: CSR-2
// (one coarsening with s1; the maps get an identity outer level, one
// super-row per super-super-row).  BAND_k::preprocessingForSpMV's loop runs
// "for (i = 1; i < k; i++)" (csrk.cu:1072-1096): CSR-2 coarsens and RCMs
// once (spmv-csrk/spmv.cpp:28 CSRK_LEVEL 2, cuda/spmv.cu:130).
int bandk_build(const hspmv_csr *A, int levels, int ssrs, int srs, hspmv_csr_buf *A_out,
                hspmv_csr3_buf *maps_out, int32_t *perm_out) {
  clear_error();
  if (!A_out || !maps_out) return set_error(HSPMV_E_INVALID, "NULL output");
  memset(A_out, 0, sizeof(*A_out));
  memset(maps_out, 0, sizeof(*maps_out));
  int rc = validate_host_csr(A, true);
  if (rc) return rc;
  if (A->m != A->n) return set_error(HSPMV_E_INVALID, "band-k needs a square matrix (m = %lld, n = %lld)",
                                     (long long)A->m, (long long)A->n);
  if (ssrs < 1 || srs < 1) return set_error(HSPMV_E_INVALID, "ssrs/srs must be >= 1");
  const int64_t m = A->m, nnz = A->nnz;
  try {
    Graph g0;
    g0.n = m;
    g0.r.assign(A->row_ptr, A->row_ptr + m + 1);
    g0.c.assign(A->col_idx, A->col_idx + nnz);
    // level 1: super-rows over the matrix in its given order
    const int64_t thr1 = (int64_t)(int)((int64_t)ssrs * nnz / (m ? m : 1));
    std::vector<int32_t> map1, map2;
    Graph g1, g2;
    hand_coarsen(g0, thr1, &map1, &g1);
    std::vector<int32_t> perm1, inv1, perm2, inv2;
    rcm(g1, perm1, inv1);
    renumber(g1, perm1, inv1);
    if (levels == 3) {
      // level 2: super-super-rows over the RCM-ordered super-rows
      const int64_t nnz1 = (int64_t)g1.c.size();
      const int64_t thr2 = (int64_t)(int)((int64_t)srs * nnz1 / (g1.n ? g1.n : 1));
      hand_coarsen(g1, thr2, &map2, &g2);
      rcm(g2, perm2, inv2);
    } else {  // CSR-2: every super-row is its own super-super-row
      g2.n = g1.n;
      map2.resize((size_t)g1.n + 1);
      std::iota(map2.begin(), map2.end(), 0);
    }
    // uncoarsen: level 2 onto level 1, then level 1 onto the rows
    std::vector<int32_t> perm0((size_t)m);
    std::iota(perm0.begin(), perm0.end(), 0);
    if (levels == 3 && g2.n > 0) uncoarsen(map2, perm2, perm1);
    if (g1.n > 0) uncoarsen(map1, perm1, perm0);
    // reorderA: symmetric permutation, columns sorted per row
    rc = permute_symmetric(A, perm0, A_out);
    if (rc) return rc;
    maps_out->n_ssr = g2.n;
    maps_out->n_sr = g1.n;
    maps_out->outer = (int32_t *)malloc(4 * (size_t)(g2.n + 1));
    maps_out->inner = (int32_t *)malloc(4 * (size_t)(g1.n + 1));
    if (!maps_out->outer || !maps_out->inner) {
      hspmv_free_csr(A_out);
      hspmv_free_csr3(maps_out);
      return set_error(HSPMV_E_NOMEM, "out of host memory");
    }
    memcpy(maps_out->outer, map2.data(), 4 * (size_t)(g2.n + 1));
    memcpy(maps_out->inner, map1.data(), 4 * (size_t)(g1.n + 1));
    if (perm_out) memcpy(perm_out, perm0.data(), 4 * (size_t)m);
  } catch (const std::bad_alloc &) {
    hspmv_free_csr(A_out);
    hspmv_free_csr3(maps_out);
    return set_error(HSPMV_E_NOMEM, "out of host memory");
  }
  return HSPMV_OK;
}

}  // namespace

extern "C" int hspmv_build_csr3_bandk(const hspmv_csr *A, int ssrs, int srs, hspmv_csr_buf *A_out,
                                      hspmv_csr3_buf *maps_out, int32_t *perm_out) {
  return bandk_build(A, 3, ssrs, srs, A_out, maps_out, perm_out);
}

extern "C" int hspmv_build_csr2_bandk(const hspmv_csr *A, int srs, hspmv_csr_buf *A_out,
                                      hspmv_csr3_buf *maps_out, int32_t *perm_out) {
  return bandk_build(A, 2, srs, 1, A_out, maps_out, perm_out);
}

// Reverse Cuthill-McKee of A's symmetrised pattern, the ordering the
// reference's converter applies before writing its .rcm.csr inputs
// (helpers/converter.m:14-15, Octave's symrcm).  Octave's implementation is
// not restated (its tie-breaking is not pinned; Octave is absent here): per
// connected component, BFS from a pseudo-peripheral vertex (the band-k
// build's search, csrk.cu:2571-2669), unvisited neighbours in increasing
// degree (then index), and the whole order reversed.  Outputs P A P^T with
// sorted columns and, if perm != NULL, perm[m] (new row i = row perm[i]).
extern "C" int hspmv_rcm_reorder(const hspmv_csr *A, hspmv_csr_buf *A_out, int32_t *perm_out) {
  clear_error();
  if (!A_out) return set_error(HSPMV_E_INVALID, "NULL output");
  memset(A_out, 0, sizeof(*A_out));
  int rc = validate_host_csr(A, true);
  if (rc) return rc;
  if (A->m != A->n) return set_error(HSPMV_E_INVALID, "RCM needs a square matrix (m = %lld, n = %lld)",
                                     (long long)A->m, (long long)A->n);
  const int64_t m = A->m;
  try {
    // the pattern of A + A^T without the diagonal
    Graph g;
    g.n = m;
    std::vector<int64_t> cnt((size_t)m + 1, 0);
    for (int64_t r = 0; r < m; ++r)
      for (int32_t k = A->row_ptr[r]; k < A->row_ptr[r + 1]; ++k)
        if (A->col_idx[k] != r) {
          ++cnt[(size_t)r + 1];
          ++cnt[(size_t)A->col_idx[k] + 1];
        }
    for (int64_t i = 0; i < m; ++i) cnt[(size_t)i + 1] += cnt[(size_t)i];
    std::vector<int32_t> adj((size_t)cnt[(size_t)m]);
    {
      std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
      for (int64_t r = 0; r < m; ++r)
        for (int32_t k = A->row_ptr[r]; k < A->row_ptr[r + 1]; ++k)
          if (A->col_idx[k] != r) {
            adj[(size_t)fill[(size_t)r]++] = A->col_idx[k];
            adj[(size_t)fill[(size_t)A->col_idx[k]]++] = (int32_t)r;
          }
    }
    // per-vertex sort + de-duplication in parallel, then compaction
    std::vector<int64_t> ulen((size_t)m, 0);
    par_ranges(m, [&](int64_t r0, int64_t r1) {
      for (int64_t r = r0; r < r1; ++r) {
        auto b = adj.begin() + cnt[(size_t)r], e = adj.begin() + cnt[(size_t)r + 1];
        std::sort(b, e);
        ulen[(size_t)r] = std::unique(b, e) - b;
      }
    });
    g.r.assign((size_t)m + 1, 0);
    for (int64_t r = 0; r < m; ++r) g.r[(size_t)r + 1] = g.r[(size_t)r] + ulen[(size_t)r];
    g.c.resize((size_t)g.r[(size_t)m]);
    par_ranges(m, [&](int64_t r0, int64_t r1) {
      for (int64_t r = r0; r < r1; ++r)
        std::copy(adj.begin() + cnt[(size_t)r], adj.begin() + cnt[(size_t)r] + ulen[(size_t)r],
                  g.c.begin() + g.r[(size_t)r]);
    });
    std::vector<int32_t>().swap(adj);
    g.deg.assign(g.c.size(), 1);
    std::vector<int32_t> order;
    order.reserve((size_t)m);
    std::vector<int32_t> mask((size_t)m, 1), lr((size_t)m + 1), lc((size_t)m + 1), kids;
    auto degree = [&](int32_t v) { return g.r[(size_t)v + 1] - g.r[(size_t)v]; };
    for (int64_t s = 0; s < m; ++s) {
      if (mask[(size_t)s] == 0) continue;
      int32_t root = (int32_t)s;
      pseudo_peripheral(root, g, mask, lr, lc);
      size_t head = order.size();
      order.push_back(root);
      mask[(size_t)root] = 0;
      while (head < order.size()) {
        const int32_t v = order[head++];
        kids.clear();
        for (int64_t k = g.r[(size_t)v]; k < g.r[(size_t)v + 1]; ++k) {
          const int32_t a = g.c[(size_t)k];
          if (mask[(size_t)a]) {
            mask[(size_t)a] = 0;
            kids.push_back(a);
          }
        }
        std::sort(kids.begin(), kids.end(), [&](int32_t a, int32_t b) {
          return degree(a) != degree(b) ? degree(a) < degree(b) : a < b;
        });
        order.insert(order.end(), kids.begin(), kids.end());
      }
    }
    std::reverse(order.begin(), order.end());
    rc = permute_symmetric(A, order, A_out);
    if (rc) return rc;
    if (perm_out) memcpy(perm_out, order.data(), 4 * (size_t)m);
  } catch (const std::bad_alloc &) {
    hspmv_free_csr(A_out);
    return set_error(HSPMV_E_NOMEM, "out of host memory");
  }
  return HSPMV_OK;
}
