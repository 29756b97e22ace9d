// lu.cpp -- the exported-LU-factor operator of the inverse drivers:
//   * eig_lu_create: upload factors in the form UMFPackFactorizedMatrix exposes
//     (umfpacktools.hh:20-39: L in compressed-row form with the unit diagonal last in each row,
//     U in compressed-column form with the diagonal last in each column, row / column
//     permutations P, Q, row scaling Rs with do_recip) -- a caller that has UMFPACK hands its
//     umfpack_dl_get_numeric arrays over unchanged;
//   * eig_lu_create_bcsr: a host factorisation producing that form (stand-in for
//     umfpack_dl_symbolic / _numeric, umfpacktools.hh:43-199, which SuiteSparse would provide):
//     reverse Cuthill-McKee symmetric ordering, row-sum scaling, envelope (profile) LU without
//     pivoting -- for the matrices the inverse drivers factor (SPD / diagonally dominant /
//     positively shifted operators);
//   * eig_inverse_mv8: Qout = A^-1 Qin on the device (matmul_inverse_tallskinny_blocked,
//     kernels_cpp.hh:660-755), k_trsv.hip.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>
#include <numeric>
#include <vector>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "internal.h"

using namespace eigmi;

namespace {

// device band factorisation admission: coupled 64-row blocks (the block-inverse chain's limit) and
// band + image tiles (2 GiB of 64 x 64 double tiles)
constexpr i64 kBandMaxGD = 8;
constexpr i64 kBandMaxTiles = 65536;

// Reverse Cuthill-McKee on the symmetrised pattern; per connected component a BFS from a
// pseudo-peripheral node, neighbours visited by increasing degree.  perm[k] = old index of new k.
std::vector<i64> rcm(i64 n, const std::vector<std::vector<i64>> &adj)
{
  std::vector<i64> perm;
  perm.reserve(n);
  std::vector<char> seen(n, 0);
  std::vector<i64> deg(n);
  for (i64 i = 0; i < n; ++i) deg[i] = (i64)adj[i].size();
  auto bfs_levels = [&](i64 s, std::vector<i64> &order, i64 &last_level_start) {
    std::vector<i64> lvl(n, -1);
    order.clear();
    order.push_back(s);
    lvl[s] = 0;
    last_level_start = 0;
    for (size_t h = 0; h < order.size(); ++h)
    {
      const i64 u = order[h];
      for (i64 v : adj[u])
        if (lvl[v] < 0 && !seen[v])
        {
          lvl[v] = lvl[u] + 1;
          order.push_back(v);
        }
    }
    const i64 maxl = lvl[order.back()];
    for (size_t h = 0; h < order.size(); ++h)
      if (lvl[order[h]] == maxl)
      {
        last_level_start = (i64)h;
        break;
      }
  };
  std::vector<i64> order;
  for (i64 s0 = 0; s0 < n; ++s0)
  {
    if (seen[s0]) continue;
    // pseudo-peripheral start: repeat BFS from a min-degree node of the last level (George-Liu)
    i64 s = s0, lls = 0;
    bfs_levels(s, order, lls);
    for (int it = 0; it < 4; ++it)
    {
      i64 best = order[lls];
      for (size_t h = lls; h < order.size(); ++h)
        if (deg[order[h]] < deg[best]) best = order[h];
      std::vector<i64> o2;
      i64 l2 = 0;
      bfs_levels(best, o2, l2);
      if (o2.size() > 0 && (size_t)l2 > (size_t)lls && o2.size() == order.size())
      {
        s = best;
        order.swap(o2);
        lls = l2;
      }
      else
        break;
    }
    // Cuthill-McKee from s
    std::vector<i64> comp;
    std::deque<i64> q;
    q.push_back(s);
    seen[s] = 1;
    while (!q.empty())
    {
      const i64 u = q.front();
      q.pop_front();
      comp.push_back(u);
      std::vector<i64> nb;
      for (i64 v : adj[u])
        if (!seen[v])
        {
          seen[v] = 1;
          nb.push_back(v);
        }
      std::sort(nb.begin(), nb.end(), [&](i64 a, i64 b) { return deg[a] != deg[b] ? deg[a] < deg[b] : a < b; });
      for (i64 v : nb) q.push_back(v);
    }
    perm.insert(perm.end(), comp.begin(), comp.end());
  }
  std::reverse(perm.begin(), perm.end());
  return perm;
}

// sum_t a[t] b[t] over a contiguous range with 8 independent partial sums, so the loop runs on
// SIMD accumulators instead of one serial chain (the envelope LU is O(n bw^2) of these dot
// products; its rounding is not part of any parity claim -- solves are checked against the
// exported factors).  AVX2 clone where the host has it.
__attribute__((target_clones("avx2", "default"))) double env_dot(const double *a, const double *b, i64 len)
{
  double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  i64 t = 0;
  for (; t + 8 <= len; t += 8)
    for (int q = 0; q < 8; ++q) s[q] += a[t + q] * b[t + q];
  for (; t < len; ++t) s[0] += a[t] * b[t];
  return ((s[0] + s[4]) + (s[1] + s[5])) + ((s[2] + s[6]) + (s[3] + s[7]));
}

}  // namespace

struct eig_lu_s {
  eig_ctx_t ctx = nullptr;
  i64 n = 0;
  int do_recip = 0;
  // host copy of the factors in the exported (UMFPACK) form
  std::vector<i64> Lp, Lj, Up, Ui, P, Q;
  std::vector<double> Lx, Ux, Rs;
  // device image (k_trsv.hip): L rows without the unit diagonal, ascending columns; U rows
  // (transposed from the columns) without the diagonal, DESCENDING columns; U diagonal
  TrsvImage img;
  // device-factored (band_lu_device): the band of 64 x 64 tiles, the envelope starts f and the block
  // bandwidth; the host copy above is filled from the band on first request (host_ready)
  double *band = nullptr;
  int band_gd = 0;
  std::vector<i64> f;
  bool host_ready = true;
  ~eig_lu_s()
  {
    if (ctx) trsv_free(img);
    if (band) (void)hipFree(band);
  }
};

namespace {

// The factors in the row form the device solves read: L rows without the unit diagonal (ascending
// columns), U rows without the diagonal (descending columns) and the U diagonal.
void factor_rows(const eig_lu_s &lu, std::vector<i64> &lrp, std::vector<i32> &lc, std::vector<double> &lv,
                 std::vector<i64> &urp, std::vector<i32> &uc, std::vector<double> &uv, std::vector<double> &ud)
{
  const i64 n = lu.n;
  // L rows: the reference subtracts entries Lp[i] .. Lp[i+1]-2 in stored order (the last entry is
  // the unit diagonal, kernels_cpp.hh:716-722).  Stored order is kept when ascending; otherwise the
  // row is sorted by column (then equal to the reference to rounding, not bitwise).
  lrp.assign(n + 1, 0);
  urp.assign(n + 1, 0);
  lc.clear();
  lv.clear();
  ud.assign(n, 0.0);
  // L: rows copied as stored when ascending (the usual case), else through a sorted copy
  lc.reserve(lu.Lx.size());
  lv.reserve(lu.Lx.size());
  std::vector<std::pair<i64, double>> e;
  for (i64 i = 0; i < n; ++i)
  {
    const i64 b = lu.Lp[i], t = lu.Lp[i + 1] - 1;  // (the last entry is the unit diagonal)
    bool sorted = true;
    for (i64 k = b; k < t; ++k)
    {
      EIG_CHECK(lu.Lj[k] >= 0 && lu.Lj[k] < i, EIG_ERR_ARG, "L factor: entry not strictly below the diagonal");
      if (k > b && lu.Lj[k] < lu.Lj[k - 1]) sorted = false;
    }
    if (sorted)
      for (i64 k = b; k < t; ++k)
      {
        lc.push_back((i32)lu.Lj[k]);
        lv.push_back(lu.Lx[k]);
      }
    else
    {
      e.clear();
      for (i64 k = b; k < t; ++k) e.push_back({lu.Lj[k], lu.Lx[k]});
      std::stable_sort(e.begin(), e.end(), [](const auto &a, const auto &c) { return a.first < c.first; });
      for (auto &q : e)
      {
        lc.push_back((i32)q.first);
        lv.push_back(q.second);
      }
    }
    lrp[i + 1] = (i64)lc.size();
  }
  // U: column j holds rows Ui[Up[j] .. Up[j+1]-2] above the diagonal Ux[Up[j+1]-1]; the reference's
  // push loop (kernels_cpp.hh:730-745) updates row i with columns j in DECREASING order, which is
  // the order the pull form below uses -- bitwise whatever the order inside a column.  Transposed
  // by a counting sort over the columns in descending order (rows come out descending).
  for (i64 j = 0; j < n; ++j)
  {
    EIG_CHECK(lu.Up[j + 1] > lu.Up[j], EIG_ERR_ARG, "U factor: empty column");
    ud[j] = lu.Ux[lu.Up[j + 1] - 1];
    for (i64 k = lu.Up[j]; k < lu.Up[j + 1] - 1; ++k)
    {
      EIG_CHECK(lu.Ui[k] >= 0 && lu.Ui[k] < j, EIG_ERR_ARG, "U factor: entry not strictly above the diagonal");
      ++urp[lu.Ui[k] + 1];
    }
  }
  for (i64 i = 0; i < n; ++i) urp[i + 1] += urp[i];
  uc.resize((size_t)urp[n]);
  uv.resize((size_t)urp[n]);
  {
    std::vector<i64> next(urp.begin(), urp.end() - 1);
    for (i64 j = n - 1; j >= 0; --j)
      for (i64 k = lu.Up[j]; k < lu.Up[j + 1] - 1; ++k)
      {
        const i64 at = next[lu.Ui[k]]++;
        uc[at] = (i32)j;
        uv[at] = lu.Ux[k];
      }
  }
}

// The exported form from the device band: L rows over the envelope [f_k, k) with the unit diagonal
// last, U columns over [f_k, k) with the pivot last; exact zeros dropped (the host factor's rule).
void ensure_host(eig_lu_s &lu)
{
  if (lu.host_ready) return;
  const i64 n = lu.n, nb = (n + 63) / 64;
  const int gd = lu.band_gd;
  std::vector<double> h((size_t)nb * (2 * gd + 1) * 4096);
  EIG_HIP(hipSetDevice(lu.ctx->device));
  EIG_HIP(hipMemcpyAsync(h.data(), lu.band, h.size() * 8, hipMemcpyDeviceToHost, lu.ctx->stream));
  EIG_HIP(hipStreamSynchronize(lu.ctx->stream));
  auto at = [&](i64 r, i64 c) { return h[((size_t)(r >> 6) * (2 * gd + 1) + ((c >> 6) - (r >> 6)) + gd) * 4096 +
                                         (size_t)(c & 63) * 64 + (r & 63)]; };
  const std::vector<i64> &f = lu.f;
  std::vector<i64> Lp(n + 1, 0), Up(n + 1, 0);
  for (i64 k = 0; k < n; ++k)
  {
    i64 cl = 1, cu = 1;
    for (i64 j = f[k]; j < k; ++j) cl += at(k, j) != 0.0;
    for (i64 i = f[k]; i < k; ++i) cu += at(i, k) != 0.0;
    Lp[k + 1] = Lp[k] + cl;
    Up[k + 1] = Up[k] + cu;
  }
  std::vector<i64> Lj(Lp[n]), Ui(Up[n]);
  std::vector<double> Lx(Lp[n]), Ux(Up[n]);
  for (i64 k = 0; k < n; ++k)
  {
    i64 q = Lp[k];
    for (i64 j = f[k]; j < k; ++j)
      if (at(k, j) != 0.0)
      {
        Lj[q] = j;
        Lx[q++] = at(k, j);
      }
    Lj[q] = k;
    Lx[q] = 1.0;
    q = Up[k];
    for (i64 i = f[k]; i < k; ++i)
      if (at(i, k) != 0.0)
      {
        Ui[q] = i;
        Ux[q++] = at(i, k);
      }
    Ui[q] = k;
    Ux[q] = at(k, k);
  }
  lu.Lp = std::move(Lp);
  lu.Lj = std::move(Lj);
  lu.Lx = std::move(Lx);
  lu.Up = std::move(Up);
  lu.Ui = std::move(Ui);
  lu.Ux = std::move(Ux);
  lu.host_ready = true;
}

void build_device(eig_lu_s &lu)
{
  const i64 n = lu.n;
  std::vector<i64> lrp, urp;
  std::vector<i32> lc, uc;
  std::vector<double> lv, uv, ud;
  factor_rows(lu, lrp, lc, lv, urp, uc, uv, ud);
  std::vector<i64> P(lu.P), Q(lu.Q);
  std::vector<double> scale(n);
  for (i64 k = 0; k < n; ++k)
  {
    EIG_CHECK(P[k] >= 0 && P[k] < n && Q[k] >= 0 && Q[k] < n, EIG_ERR_ARG, "permutation entry out of range");
    scale[k] = lu.do_recip ? lu.Rs[P[k]] : 1.0 / lu.Rs[P[k]];  // kernels_cpp.hh:683-705
  }
  trsv_upload(lu.ctx, n, lrp, lc, lv, urp, uc, uv, ud, P, Q, scale, lu.img);
}

}  // namespace

extern "C" int eig_lu_create(eig_ctx_t ctx, int64_t n, const int64_t *Lp, const int64_t *Lj, const double *Lx,
                             const int64_t *Up, const int64_t *Ui, const double *Ux, const int64_t *P,
                             const int64_t *Q, const double *Rs, int do_recip, eig_lu_t *out)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && out && n > 0 && Lp && Lj && Lx && Up && Ui && Ux && P && Q && Rs, EIG_ERR_ARG,
              "eig_lu_create: null argument");
    EIG_CHECK(n < (int64_t)INT32_MAX, EIG_ERR_SHAPE, "eig_lu_create: n too large for int32 indices");
    EIG_HIP(hipSetDevice(ctx->device));
    auto *lu = new eig_lu_s();
    try
    {
      lu->ctx = ctx;
      lu->n = n;
      lu->do_recip = do_recip ? 1 : 0;
      lu->Lp.assign(Lp, Lp + n + 1);
      lu->Lj.assign(Lj, Lj + Lp[n]);
      lu->Lx.assign(Lx, Lx + Lp[n]);
      lu->Up.assign(Up, Up + n + 1);
      lu->Ui.assign(Ui, Ui + Up[n]);
      lu->Ux.assign(Ux, Ux + Up[n]);
      lu->P.assign(P, P + n);
      lu->Q.assign(Q, Q + n);
      lu->Rs.assign(Rs, Rs + n);
      build_device(*lu);
    }
    catch (...)
    {
      delete lu;
      throw;
    }
    *out = lu;
  });
}

namespace {
// The device band LU factors without pivoting (k_band.hip) where UMFPACK, the reference's factoriser,
// pivots.  Growth through the coupled tiles is not bounded a priori, so after factoring: one solve of
// 8 right-hand sides and the componentwise backward error max |A x - b| / (|A| |x| + |b|) on the host
// (Oettli-Prager); above 1e-9 the factors are rejected (EIG_ERR_BREAKDOWN) instead of returning a
// solve that silently lost its digits.
void check_backward_error(eig_lu_s &lu, const std::vector<std::vector<std::pair<i64, double>>> &rowsA)
{
  const i64 n = lu.n;
  if (n == 0) return;
  hipStream_t s = lu.ctx->stream;
  std::vector<double> b((size_t)n * 8), x((size_t)n * 8);
  u64 h = 0x9e3779b97f4a7c15ull;
  for (auto &v : b)
  {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 29;
    v = (double)(h >> 11) * (2.0 / 9007199254740992.0) - 1.0;
  }
  DevBuf din(b.size() * sizeof(double)), dout(b.size() * sizeof(double));
  EIG_HIP(hipMemcpyAsync(din.d(), b.data(), b.size() * sizeof(double), hipMemcpyHostToDevice, s));
  launch_inverse_mv8(lu.img, 8, din.d(), dout.d(), s);
  EIG_HIP(hipMemcpyAsync(x.data(), dout.d(), x.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  EIG_HIP(hipStreamSynchronize(s));
  EIG_HIP(hipMemcpyAsync(din.d(), b.data(), b.size() * sizeof(double), hipMemcpyHostToDevice, s));  // (restore)
  double worst = 0.0;
  for (i64 i = 0; i < n; ++i)
    for (int j = 0; j < 8; ++j)
    {
      double r = -b[(size_t)i * 8 + j], d = std::fabs(b[(size_t)i * 8 + j]);
      for (auto &e : rowsA[i])
      {
        const double t = e.second * x[(size_t)e.first * 8 + j];
        r += t;
        d += std::fabs(t);
      }
      if (!std::isfinite(r)) worst = HUGE_VAL;
      else if (d > 0.0) worst = std::max(worst, std::fabs(r) / d);
    }
  EIG_HIP(hipStreamSynchronize(s));
  if (!(worst <= 1e-9))
    throw Error(EIG_ERR_BREAKDOWN, "LU without pivoting: backward error " + std::to_string(worst) +
                                       " of a test solve exceeds 1e-9 (the matrix needs pivoting)");
}
}  // namespace

extern "C" int eig_lu_create_bcsr(eig_ctx_t ctx, int64_t nb_rows, int br, const int64_t *rowptr, const int32_t *col,
                                  const double *vals, eig_lu_t *out)
{
  return guard(ctx, [&] {
    EIG_CHECK(out && rowptr && col && vals && nb_rows > 0 && br >= 1 && br <= 4, EIG_ERR_ARG,
              "eig_lu_create_bcsr: bad argument");
    if (ctx) EIG_HIP(hipSetDevice(ctx->device));
    const i64 n = nb_rows * br;
    EIG_CHECK(n < (int64_t)INT32_MAX, EIG_ERR_SHAPE, "eig_lu_create_bcsr: too large");
    // EIGMI_TRACE_SETUP=1: phase times on stderr (as trsv_upload)
    const bool trace = std::getenv("EIGMI_TRACE_SETUP") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto phase = [&](const char *what) {
      if (!trace) return;
      const auto now = std::chrono::steady_clock::now();
      fprintf(stderr, "lu_create  %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - t_last).count());
      t_last = now;
    };
    // scalar entries of the block matrix (zeros skipped, as umfpacktools.hh:66-93 does)
    std::vector<std::vector<std::pair<i64, double>>> rowsA(n);
    for (i64 rb = 0; rb < nb_rows; ++rb)
      for (i64 p = rowptr[rb]; p < rowptr[rb + 1]; ++p)
        for (int a = 0; a < br; ++a)
          for (int b = 0; b < br; ++b)
          {
            const double v = vals[p * br * br + a * br + b];
            if (v != 0.0) rowsA[rb * br + a].push_back({(i64)col[p] * br + b, v});
          }
    std::vector<std::vector<i64>> adj(n);
    for (i64 i = 0; i < n; ++i)
      for (auto &e : rowsA[i])
        if (e.first != i)
        {
          EIG_CHECK(e.first >= 0 && e.first < n, EIG_ERR_SHAPE, "column out of range");
          adj[i].push_back(e.first);
          adj[e.first].push_back(i);
        }
    for (auto &a : adj)
    {
      std::sort(a.begin(), a.end());
      a.erase(std::unique(a.begin(), a.end()), a.end());
    }
    phase("rows+adj");
    std::vector<i64> perm = rcm(n, adj), inv(n);
    phase("rcm");
    for (i64 k = 0; k < n; ++k) inv[perm[k]] = k;
    std::vector<double> Rs(n, 0.0);
    for (i64 i = 0; i < n; ++i)
    {
      for (auto &e : rowsA[i]) Rs[i] += std::fabs(e.second);
      EIG_CHECK(Rs[i] > 0.0, EIG_ERR_BREAKDOWN, "LU: zero row");
    }
    // B = (R^-1 A)[perm, perm] in the envelope: f[k] = first column of new row k (symmetrised)
    std::vector<i64> f(n);
    for (i64 k = 0; k < n; ++k)
    {
      i64 m = k;
      for (i64 v : adj[perm[k]]) m = std::min(m, inv[v]);
      f[k] = m;
    }
    // device factorisation (k_band.hip) when the envelope fits a band of at most kBandMaxGD coupled
    // 64-row blocks: the band LU and the block-inverse image on the GPU, the exported form built
    // from the band only when asked for (eig_lu_info / _export / _set_solver staged or csr)
    {
      i64 gdm = 0;
      for (i64 k = 0; k < n; ++k) gdm = std::max(gdm, k / 64 - f[k] / 64);
      const i64 nb = (n + 63) / 64;
      if (ctx && gdm <= kBandMaxGD && nb * (4 * gdm + 3) <= kBandMaxTiles)
      {
        std::vector<i64> rp(n + 1, 0);
        for (i64 i = 0; i < n; ++i) rp[i + 1] = rp[i] + (i64)rowsA[i].size();
        std::vector<i32> cj(rp[n]), inv32(n);
        std::vector<double> cv(rp[n]);
        for (i64 i = 0; i < n; ++i)
        {
          i64 q = rp[i];
          for (auto &e : rowsA[i])
          {
            cj[q] = (i32)e.first;
            cv[q++] = e.second;
          }
          inv32[i] = (i32)inv[i];
        }
        phase("csr");
        auto *lu = new eig_lu_s();
        try
        {
          lu->ctx = ctx;
          lu->n = n;
          lu->do_recip = 0;
          lu->P = perm;
          lu->Q = perm;
          lu->f = f;
          lu->band_gd = (int)gdm;
          lu->host_ready = false;
          const bool ok = band_lu_device(ctx, n, (int)gdm, rp, cj, cv, inv32, Rs, lu->img, &lu->band);
          phase("band");
          std::vector<double> scale(n);
          for (i64 k = 0; k < n; ++k) scale[k] = 1.0 / Rs[perm[k]];  // kernels_cpp.hh:683-705
          lu->Rs = std::move(Rs);
          if (ok)
            trsv_attach_perm(ctx, n, lu->P, lu->Q, scale, lu->img);
          else
          {
            // a diagonal tile too ill-conditioned for the block-inverse image: the host image path
            // (substitution kernels) on the downloaded factors
            ensure_host(*lu);
            build_device(*lu);
          }
          phase("device");
          check_backward_error(*lu, rowsA);
          phase("check");
        }
        catch (...)
        {
          delete lu;
          throw;
        }
        *out = lu;
        return;
      }
    }
    std::vector<i64> off(n + 1, 0);  // envelope storage: row k of L / column k of U over [f_k, k)
    for (i64 k = 0; k < n; ++k) off[k + 1] = off[k] + (k - f[k]);
    const i64 env = off[n];
    EIG_CHECK(env < (i64)1 << 31, EIG_ERR_SHAPE, "LU: envelope too large for the host factorisation");
    std::vector<double> L(env, 0.0), U(env, 0.0), D(n, 0.0);
    for (i64 k = 0; k < n; ++k)
    {
      const i64 i0 = perm[k];
      for (auto &e : rowsA[i0])
      {
        const i64 j = inv[e.first];
        const double v = e.second / Rs[i0];
        if (j < k) L[off[k] + (j - f[k])] = v;
        else if (j == k) D[k] = v;
        else U[off[j] + (k - f[j])] = v;  // B[k][j], j > k: column j of U, row k
      }
    }
    phase("scatter");
    auto Lat = [&](i64 r, i64 c) -> double & { return L[off[r] + (c - f[r])]; };
    auto Uat = [&](i64 r, i64 c) -> double & { return U[off[c] + (r - f[c])]; };  // r < c
    for (i64 k = 0; k < n; ++k)
    {
      // column k of U, rows f_k .. k-1
      for (i64 i = f[k]; i < k; ++i)
      {
        const i64 t0 = std::max(f[i], f[k]);
        Uat(i, k) -= env_dot(&Lat(i, t0), &Uat(t0, k), i - t0);
      }
      // row k of L, columns f_k .. k-1
      for (i64 j = f[k]; j < k; ++j)
      {
        const i64 t0 = std::max(f[k], f[j]);
        const double s = Lat(k, j) - env_dot(&Lat(k, t0), &Uat(t0, j), j - t0);
        EIG_CHECK(D[j] != 0.0, EIG_ERR_BREAKDOWN, "LU: zero pivot (matrix needs pivoting)");
        Lat(k, j) = s / D[j];
      }
      double s = D[k] - env_dot(&Lat(k, f[k]), &Uat(f[k], k), k - f[k]);
      EIG_CHECK(s != 0.0 && std::isfinite(s), EIG_ERR_BREAKDOWN, "LU: zero pivot (matrix needs pivoting)");
      D[k] = s;
    }
    // exported form: L rows ascending + unit diagonal last; U columns ascending + diagonal last
    phase("factor");
    std::vector<i64> Lp(n + 1, 0), Up(n + 1, 0);
    for (i64 k = 0; k < n; ++k)
    {
      i64 cl = 1, cu = 1;  // + the unit / pivot diagonal
      for (i64 j = f[k]; j < k; ++j) cl += Lat(k, j) != 0.0;
      for (i64 i = f[k]; i < k; ++i) cu += Uat(i, k) != 0.0;
      Lp[k + 1] = Lp[k] + cl;
      Up[k + 1] = Up[k] + cu;
    }
    std::vector<i64> Lj(Lp[n]), Ui(Up[n]);
    std::vector<double> Lx(Lp[n]), Ux(Up[n]);
    for (i64 k = 0; k < n; ++k)
    {
      i64 q = Lp[k];
      for (i64 j = f[k]; j < k; ++j)
        if (Lat(k, j) != 0.0)
        {
          Lj[q] = j;
          Lx[q++] = Lat(k, j);
        }
      Lj[q] = k;
      Lx[q] = 1.0;
      q = Up[k];
      for (i64 i = f[k]; i < k; ++i)
        if (Uat(i, k) != 0.0)
        {
          Ui[q] = i;
          Ux[q++] = Uat(i, k);
        }
      Ui[q] = k;
      Ux[q] = D[k];
    }
    phase("export");
    auto *lu = new eig_lu_s();
    try
    {
      lu->ctx = ctx;
      lu->n = n;
      lu->do_recip = 0;
      lu->Lp = std::move(Lp);
      lu->Lj = std::move(Lj);
      lu->Lx = std::move(Lx);
      lu->Up = std::move(Up);
      lu->Ui = std::move(Ui);
      lu->Ux = std::move(Ux);
      lu->P = perm;
      lu->Q = perm;
      lu->Rs = std::move(Rs);
      if (ctx) build_device(*lu);  // ctx == NULL: host-only factors (export / tests)
      phase("device");
    }
    catch (...)
    {
      delete lu;
      throw;
    }
    *out = lu;
  });
}

extern "C" int eig_lu_info(eig_lu_t lu, int64_t *n, int64_t *lnz, int64_t *unz, int *do_recip)
{
  return guard(lu ? lu->ctx : nullptr, [&] {
    EIG_CHECK(lu, EIG_ERR_ARG, "eig_lu_info: null handle");
    ensure_host(*lu);
    if (n) *n = lu->n;
    if (lnz) *lnz = lu->Lp[lu->n];
    if (unz) *unz = lu->Up[lu->n];
    if (do_recip) *do_recip = lu->do_recip;
  });
}

extern "C" int eig_lu_set_solver(eig_lu_t lu, int kind)
{
  return guard(lu ? lu->ctx : nullptr, [&] {
    EIG_CHECK(lu, EIG_ERR_ARG, "eig_lu_set_solver: null handle");
    EIG_CHECK(kind >= EIG_TRSV_AUTO && kind <= EIG_TRSV_CSR, EIG_ERR_ARG, "eig_lu_set_solver: unknown solver");
    EIG_CHECK(kind != EIG_TRSV_BLOCKINV || !lu->ctx || lu->img.binv, EIG_ERR_ARG,
              "eig_lu_set_solver: these factors have no block-inverse image");
    if ((kind == EIG_TRSV_STAGED || kind == EIG_TRSV_CSR) && lu->ctx && !lu->img.rows)
    {
      // the substitution kernels read the row factors, not uploaded next to a block-inverse image
      EIG_HIP(hipSetDevice(lu->ctx->device));
      ensure_host(*lu);
      std::vector<i64> lrp, urp;
      std::vector<i32> lc, uc;
      std::vector<double> lv, uv, ud;
      factor_rows(*lu, lrp, lc, lv, urp, uc, uv, ud);
      trsv_upload_rows(lu->img, lrp, lc, lv, urp, uc, uv, ud);
    }
    lu->img.solver = kind;
  });
}

extern "C" int eig_lu_solver_info(eig_lu_t lu, int *kind, int *coupled_l, int *coupled_u)
{
  return guard(lu ? lu->ctx : nullptr, [&] {
    EIG_CHECK(lu && lu->ctx, EIG_ERR_ARG, "eig_lu_solver_info: null handle or host-only factors");
    const TrsvImage &im = lu->img;
    const bool csr = im.solver == EIG_TRSV_CSR, staged = im.solver == EIG_TRSV_STAGED;
    if (kind)
      *kind = (im.binv && !csr && !staged) ? EIG_TRSV_BLOCKINV
              : (im.staged && !csr && (im.host || im.staged_built)) ? EIG_TRSV_STAGED
                                                                    : EIG_TRSV_CSR;
    if (coupled_l) *coupled_l = im.gd[0];
    if (coupled_u) *coupled_u = im.gd[1];
  });
}

extern "C" int eig_lu_export(eig_lu_t lu, int64_t *Lp, int64_t *Lj, double *Lx, int64_t *Up, int64_t *Ui, double *Ux,
                             int64_t *P, int64_t *Q, double *Rs)
{
  return guard(lu ? lu->ctx : nullptr, [&] {
    EIG_CHECK(lu && Lp && Lj && Lx && Up && Ui && Ux && P && Q && Rs, EIG_ERR_ARG, "eig_lu_export: null argument");
    ensure_host(*lu);
    std::copy(lu->Lp.begin(), lu->Lp.end(), Lp);
    std::copy(lu->Lj.begin(), lu->Lj.end(), Lj);
    std::copy(lu->Lx.begin(), lu->Lx.end(), Lx);
    std::copy(lu->Up.begin(), lu->Up.end(), Up);
    std::copy(lu->Ui.begin(), lu->Ui.end(), Ui);
    std::copy(lu->Ux.begin(), lu->Ux.end(), Ux);
    std::copy(lu->P.begin(), lu->P.end(), P);
    std::copy(lu->Q.begin(), lu->Q.end(), Q);
    std::copy(lu->Rs.begin(), lu->Rs.end(), Rs);
  });
}

extern "C" int eig_lu_destroy(eig_lu_t lu)
{
  if (!lu) return EIG_OK;
  if (lu->ctx)
  {
    (void)hipSetDevice(lu->ctx->device);
    (void)hipStreamSynchronize(lu->ctx->stream);
  }
  delete lu;
  return EIG_OK;
}

namespace eigmi {
void lu_inverse_device(eig_lu_t lu, i64 m, double *Qin, double *Qout, hipStream_t s)
{
  launch_inverse_mv8(lu->img, m, Qin, Qout, s);
}
i64 lu_size(eig_lu_t lu) { return lu->n; }
}  // namespace eigmi

extern "C" int eig_inverse_mv8(eig_lu_t lu, int64_t m, double *Qin, double *Qout)
{
  return guard(lu ? lu->ctx : nullptr, [&] {
    EIG_CHECK(lu && Qin && Qout, EIG_ERR_ARG, "eig_inverse_mv8: null argument");
    EIG_CHECK(lu->ctx, EIG_ERR_ARG, "eig_inverse_mv8: host-only factors (created without a context)");
    EIG_CHECK(m >= 0 && m % 8 == 0, EIG_ERR_SHAPE, "matmul_inverse_tallskinny_blocked: columns must be a multiple of 8");
    EIG_HIP(hipSetDevice(lu->ctx->device));
    if (m > 0) launch_inverse_mv8(lu->img, m, Qin, Qout, lu->ctx->stream);
  });
}
