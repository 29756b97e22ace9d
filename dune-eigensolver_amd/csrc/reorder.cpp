// reorder.cpp -- host reordering utilities for matrices imported from outside the generators
// (Matrix Market files, application assemblies): reverse Cuthill-McKee on the symmetrised
// pattern, and the symmetric permutation B = P A P^T with every row's columns ascending (the ISTL
// order the SELL image keeps).  An RCM ordering turns the scattered gathers of an unstructured
// matrix into a band the L2 / MALL serve; the reference has no counterpart (its matrices come from
// the generators, src/dune-eigensolver.cc:98-156, or from UMFPACK's own ordering,
// umfpacktools.hh:46-199) -- this is the host side of the general CSR/ELL path.
#include <algorithm>
#include <cstdint>
#include <numeric>
#include <thread>
#include <vector>

#include "internal.h"

using namespace eigmi;

namespace {

template <class F>
void parallel_rows(i64 n, F &&f)
{
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < (1 << 16)) nt = 1;
  if (nt == 1) return f(0, n);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back([&, t] { f(n * t / nt, n * (t + 1) / nt); });
  for (auto &t : th) t.join();
}

// Symmetrised adjacency (no self loops, sorted, unique) in CSR form.
void sym_adjacency(i64 n, const int64_t *rowptr, const int32_t *col, std::vector<i64> &xadj, std::vector<int32_t> &adj)
{
  std::vector<i64> cnt(n + 1, 0);
  for (i64 i = 0; i < n; ++i)
    for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
    {
      const i64 j = col[p];
      EIG_CHECK(j >= 0 && j < n, EIG_ERR_SHAPE, "eig_reorder_rcm: column out of range");
      if (j != i)
      {
        ++cnt[i + 1];
        ++cnt[j + 1];
      }
    }
  for (i64 i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
  std::vector<i64> fill(cnt.begin(), cnt.end() - 1);
  std::vector<int32_t> raw(cnt[n]);
  for (i64 i = 0; i < n; ++i)
    for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
    {
      const i64 j = col[p];
      if (j != i)
      {
        raw[fill[i]++] = (int32_t)j;
        raw[fill[j]++] = (int32_t)i;
      }
    }
  xadj.assign(n + 1, 0);
  std::vector<i64> len(n);
  parallel_rows(n, [&](i64 b, i64 e) {
    for (i64 i = b; i < e; ++i)
    {
      int32_t *a = raw.data() + cnt[i], *z = raw.data() + cnt[i + 1];
      std::sort(a, z);
      len[i] = std::unique(a, z) - a;
    }
  });
  for (i64 i = 0; i < n; ++i) xadj[i + 1] = xadj[i] + len[i];
  adj.resize(xadj[n]);
  parallel_rows(n, [&](i64 b, i64 e) {
    for (i64 i = b; i < e; ++i) std::copy(raw.begin() + cnt[i], raw.begin() + cnt[i] + len[i], adj.begin() + xadj[i]);
  });
}

// Reverse Cuthill-McKee; per connected component a BFS from a pseudo-peripheral node (George-Liu:
// restart from a minimum-degree node of the last level while the eccentricity grows), neighbours
// queued by increasing degree (ties: lower index).  perm[k] = old index of new row k.
std::vector<i64> rcm_csr(i64 n, const std::vector<i64> &xadj, const std::vector<int32_t> &adj)
{
  std::vector<i64> perm;
  perm.reserve(n);
  std::vector<char> seen(n, 0);
  std::vector<int32_t> lvl(n, -1);
  auto deg = [&](i64 v) { return xadj[v + 1] - xadj[v]; };
  // level structure from s over the unseen component; returns the BFS order, sets the start of the
  // last level; lvl is reset for the visited nodes afterwards
  auto bfs = [&](i64 s, std::vector<i64> &order, size_t &last) {
    order.clear();
    order.push_back(s);
    lvl[s] = 0;
    for (size_t h = 0; h < order.size(); ++h)
    {
      const i64 u = order[h];
      for (i64 p = xadj[u]; p < xadj[u + 1]; ++p)
      {
        const i64 v = adj[p];
        if (lvl[v] < 0 && !seen[v])
        {
          lvl[v] = lvl[u] + 1;
          order.push_back(v);
        }
      }
    }
    const int maxl = lvl[order.back()];
    last = 0;
    while (lvl[order[last]] != maxl) ++last;
    const int ecc = maxl;
    for (i64 v : order) lvl[v] = -1;
    return ecc;
  };
  std::vector<i64> order, o2, comp, nb;
  for (i64 s0 = 0; s0 < n; ++s0)
  {
    if (seen[s0]) continue;
    i64 s = s0;
    size_t last = 0;
    int ecc = bfs(s, order, last);
    for (int it = 0; it < 8; ++it)
    {
      i64 best = order[last];
      for (size_t h = last; h < order.size(); ++h)
        if (deg(order[h]) < deg(best)) best = order[h];
      size_t l2 = 0;
      const int e2 = bfs(best, o2, l2);
      if (e2 <= ecc) break;
      s = best;
      ecc = e2;
      order.swap(o2);
      last = l2;
    }
    // Cuthill-McKee from s (comp doubles as the BFS queue)
    comp.clear();
    comp.push_back(s);
    seen[s] = 1;
    for (size_t h = 0; h < comp.size(); ++h)
    {
      const i64 u = comp[h];
      nb.clear();
      for (i64 p = xadj[u]; p < xadj[u + 1]; ++p)
        if (!seen[adj[p]])
        {
          seen[adj[p]] = 1;
          nb.push_back(adj[p]);
        }
      std::sort(nb.begin(), nb.end(), [&](i64 a, i64 b) { return deg(a) != deg(b) ? deg(a) < deg(b) : a < b; });
      comp.insert(comp.end(), nb.begin(), nb.end());
    }
    perm.insert(perm.end(), comp.begin(), comp.end());
  }
  std::reverse(perm.begin(), perm.end());
  return perm;
}

}  // namespace

extern "C" int eig_reorder_rcm(int64_t n, const int64_t *rowptr, const int32_t *col, int64_t *perm)
{
  return guard(nullptr, [&] {
    EIG_CHECK(n >= 0 && rowptr && perm && (n == 0 || rowptr[n] == 0 || col), EIG_ERR_ARG,
              "eig_reorder_rcm: null argument");
    EIG_CHECK(n < (int64_t)INT32_MAX, EIG_ERR_SHAPE, "eig_reorder_rcm: too many rows for int32 columns");
    std::vector<i64> xadj;
    std::vector<int32_t> adj;
    sym_adjacency(n, rowptr, col, xadj, adj);
    const std::vector<i64> p = rcm_csr(n, xadj, adj);
    std::copy(p.begin(), p.end(), perm);
  });
}

extern "C" int eig_permute_symmetric(int64_t n, const int64_t *rowptr, const int32_t *col, const double *vals,
                                     const int64_t *perm, int64_t *rowptr_out, int32_t *col_out, double *vals_out)
{
  return guard(nullptr, [&] {
    EIG_CHECK(n >= 0 && rowptr && perm && rowptr_out && (n == 0 || rowptr[n] == 0 || (col && vals && col_out && vals_out)),
              EIG_ERR_ARG, "eig_permute_symmetric: null argument");
    std::vector<i64> inv(n, -1);
    for (i64 k = 0; k < n; ++k)
    {
      EIG_CHECK(perm[k] >= 0 && perm[k] < n && inv[perm[k]] < 0, EIG_ERR_ARG,
                "eig_permute_symmetric: perm is not a permutation");
      inv[perm[k]] = k;
    }
    for (i64 i = 0; i < n; ++i)
      for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
        EIG_CHECK(col[p] >= 0 && col[p] < n, EIG_ERR_SHAPE, "eig_permute_symmetric: column out of range");
    rowptr_out[0] = 0;
    for (i64 k = 0; k < n; ++k) rowptr_out[k + 1] = rowptr_out[k] + (rowptr[perm[k] + 1] - rowptr[perm[k]]);
    parallel_rows(n, [&](i64 b, i64 e) {
      std::vector<std::pair<int32_t, double>> row;
      for (i64 k = b; k < e; ++k)
      {
        const i64 i = perm[k];
        row.clear();
        for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
        {
          row.push_back({(int32_t)inv[col[p]], vals[p]});
        }
        std::stable_sort(row.begin(), row.end(),
                         [](const std::pair<int32_t, double> &a, const std::pair<int32_t, double> &c) {
                           return a.first < c.first;
                         });
        i64 q = rowptr_out[k];
        for (auto &x : row)
        {
          col_out[q] = x.first;
          vals_out[q++] = x.second;
        }
      }
    });
  });
}
