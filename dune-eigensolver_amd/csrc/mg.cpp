// mg.cpp -- geometric multigrid inner solve for the spectral transformation of config C5 (the
// smallest end of K x = lambda M x, which GeneralizedInverse returns: eigensolver.hh:204-351; there
// with an UMFPACK LU, which does not exist at 256^3 -- SURVEY 7, hard part 4).
//
// Hierarchy (host setup, once): a box grid nx x ny x nz (lexicographic) is coarsened by keeping the
// fine nodes of odd index in every direction (nc = nf / 2), with trilinear P (k_mg.hip) and the
// Galerkin operator A_c = P^T A P computed on the host from the fine rows (27-point coarse
// stencils; any fine stencil within +-1 node per direction), mirrored so that every coarse matrix
// is bitwise symmetric (it then takes the band / box images of the device upload).  Levels stop at
// <= 64 rows or a direction < 3 nodes; grids whose coarsest level would exceed kMgMaxCoarse rows (flat
// grids: a direction runs out first) are refused.
//
// Solve (device, no reductions): X = S_k B with S_k = sum_{i<k} (I - V A)^i V, i.e. `cycles`
// stationary iterations x += V (b - A x) from x = 0, V one symmetric V-cycle:
//   pre-smooth  x = p(D^-1 A) D^-1 b      (Chebyshev-Jacobi, degree nu, on [lmax / ratio, lmax],
//                                          lmax the Gershgorin bound of D^-1 A; cheb_solve)
//   r = b - A x;  x += P V_c (P^T r);  r = b - A x;  x += p(D^-1 A) D^-1 r   (the same polynomial)
// the coarsest level by a Chebyshev-Jacobi solve on its exact spectrum bounds (host eigenvalues)
// to 1e-15.  With V symmetric, S_k is a fixed symmetric linear operator, so the block Lanczos on
// OP = S_k M (eig_blanczos_create_si_mg) runs on a self-adjoint operator in the M-inner product,
// with no inner product inside the solve (halo-only when distributed -- single rank here).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "internal.h"

using namespace eigmi;

namespace eigmi {
void launch_mg_restrict(const int *fdim, const int *cdim, i64 m, i64 ldf, i64 ldc, const double *Rf, double *Bc,
                        hipStream_t s);
void launch_mg_prolong_add(const int *fdim, const int *cdim, i64 m, i64 ldf, i64 ldc, const double *Xc, double *Xf,
                           hipStream_t s);
void launch_mv8_axpby(i64 n, i64 m, i64 ld, double a, const double *X, double b, double *Y, hipStream_t s);
}  // namespace eigmi

struct MgLevel {
  eig_mat_s *A = nullptr;
  bool own = false;  // coarse levels own their matrix
  int dim[3] = {0, 0, 0};
  i64 n = 0;
  double lmax = 2.0;                          // Gershgorin bound of D^-1 A
  double clo = 0.0, chi = 0.0;                // coarsest: exact spectrum bounds of D^-1 A
  int cdeg = 0;                               // coarsest: Chebyshev degree
  DevBuf *dinv = nullptr, *B = nullptr, *T = nullptr, *C[4] = {nullptr, nullptr, nullptr, nullptr};
};

struct eig_mg_s {
  eig_ctx_t ctx = nullptr;
  std::vector<MgLevel> lev;
  int max_cols = 32, nu = 2;
  double ratio = 10.0;
  ~eig_mg_s()
  {
    for (auto &L : lev)
    {
      for (DevBuf *b : {L.dinv, L.B, L.T, L.C[0], L.C[1], L.C[2], L.C[3]}) delete b;
      if (L.own && L.A) eig_mat_destroy(L.A);
    }
  }
};

namespace {

// largest coarsest level whose D^-1/2 A D^-1/2 spectrum is computed densely on the host
constexpr i64 kMgMaxCoarse = 1024;

// Host CSR of one level (rows ascending columns).
struct HostCsr {
  std::vector<i64> rp;
  std::vector<i32> col;
  std::vector<double> val;
};

double gershgorin(const HostCsr &A, i64 n)
{
  double g = 0.0;
  for (i64 r = 0; r < n; ++r)
  {
    double d = 0.0, s = 0.0;
    for (i64 k = A.rp[r]; k < A.rp[r + 1]; ++k)
    {
      s += std::fabs(A.val[k]);
      if (A.col[k] == r) d = A.val[k];
    }
    EIG_CHECK(d > 0.0, EIG_ERR_BREAKDOWN, "multigrid: a level has a non-positive diagonal entry");
    g = std::max(g, s / d);
  }
  return g;
}

// per-direction coarse neighbours of fine index f: (c0, w) and (c1, w) (c = -1: none)
inline void split1(int f, int nc, int &c0, int &c1, double &w)
{
  if (f & 1)
  {
    c0 = (f - 1) >> 1;
    c1 = -1;
    w = 1.0;
  }
  else
  {
    c0 = (f >> 1) - 1;
    c1 = (f >> 1) < nc ? (f >> 1) : -1;
    w = 0.5;
  }
}

// A_c = P^T A P on the 27-point coarse stencil; rows computed independently (threads over coarse
// rows), every coarse row gathering its fine rows in z, y, x order; then mirrored (entry (J, I), J > I,
// takes the value computed for (I, J)) so the coarse matrix is bitwise symmetric.
void galerkin(const HostCsr &A, const int *fd, const int *cd, HostCsr &Ac)
{
  const i64 nc = (i64)cd[0] * cd[1] * cd[2];
  std::vector<double> slot((size_t)nc * 27, 0.0);
  int nt = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  std::vector<int> bad(nt, 0);
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (i64 I = t; I < nc; I += nt)
      {
        const int X = (int)(I % cd[0]), Y = (int)((I / cd[0]) % cd[1]), Z = (int)(I / ((i64)cd[0] * cd[1]));
        double *acc = &slot[(size_t)I * 27];
        for (int dz = -1; dz <= 1; ++dz)
        {
          const int z = 2 * Z + 1 + dz;
          if (z < 0 || z >= fd[2]) continue;
          for (int dy = -1; dy <= 1; ++dy)
          {
            const int y = 2 * Y + 1 + dy;
            if (y < 0 || y >= fd[1]) continue;
            for (int dx = -1; dx <= 1; ++dx)
            {
              const int x = 2 * X + 1 + dx;
              if (x < 0 || x >= fd[0]) continue;
              const double wi = (dz ? 0.5 : 1.0) * (dy ? 0.5 : 1.0) * (dx ? 0.5 : 1.0);
              const i64 i = ((i64)z * fd[1] + y) * fd[0] + x;
              for (i64 k = A.rp[i]; k < A.rp[i + 1]; ++k)
              {
                const i64 j = A.col[k];
                const int jx = (int)(j % fd[0]), jy = (int)((j / fd[0]) % fd[1]), jz = (int)(j / ((i64)fd[0] * fd[1]));
                int cz[2], cy[2], cx[2];
                double wz, wy, wx;
                split1(jz, cd[2], cz[0], cz[1], wz);
                split1(jy, cd[1], cy[0], cy[1], wy);
                split1(jx, cd[0], cx[0], cx[1], wx);
                const double a = wi * A.val[k] * (wz * wy * wx);
                for (int p = 0; p < 2; ++p)
                {
                  if (cz[p] < 0) continue;
                  for (int q = 0; q < 2; ++q)
                  {
                    if (cy[q] < 0) continue;
                    for (int r = 0; r < 2; ++r)
                    {
                      if (cx[r] < 0) continue;
                      const int oz = cz[p] - Z, oy = cy[q] - Y, ox = cx[r] - X;
                      if (oz < -1 || oz > 1 || oy < -1 || oy > 1 || ox < -1 || ox > 1)
                      {
                        bad[t] = 1;
                        continue;
                      }
                      acc[(oz + 1) * 9 + (oy + 1) * 3 + (ox + 1)] += a;
                    }
                  }
                }
              }
            }
          }
        }
      }
    });
  for (auto &x : th) x.join();
  for (int b : bad)
    EIG_CHECK(!b, EIG_ERR_ARG, "multigrid: the matrix couples nodes more than one grid step apart (not a box stencil "
                               "on the given grid)");
  // mirror the upper entries into the lower ones, then compress (in-bounds neighbours, ascending columns)
  for (i64 I = 0; I < nc; ++I)
  {
    const int X = (int)(I % cd[0]), Y = (int)((I / cd[0]) % cd[1]), Z = (int)(I / ((i64)cd[0] * cd[1]));
    for (int s = 0; s < 13; ++s)  // offsets before the centre: J < I
    {
      const int oz = s / 9 - 1, oy = (s / 3) % 3 - 1, ox = s % 3 - 1;
      const int jx = X + ox, jy = Y + oy, jz = Z + oz;
      if (jx < 0 || jx >= cd[0] || jy < 0 || jy >= cd[1] || jz < 0 || jz >= cd[2]) continue;
      const i64 J = ((i64)jz * cd[1] + jy) * cd[0] + jx;
      slot[(size_t)I * 27 + s] = slot[(size_t)J * 27 + (26 - s)];
    }
  }
  Ac.rp.assign(nc + 1, 0);
  Ac.col.clear();
  Ac.val.clear();
  Ac.col.reserve((size_t)nc * 27);
  Ac.val.reserve((size_t)nc * 27);
  for (i64 I = 0; I < nc; ++I)
  {
    const int X = (int)(I % cd[0]), Y = (int)((I / cd[0]) % cd[1]), Z = (int)(I / ((i64)cd[0] * cd[1]));
    for (int s = 0; s < 27; ++s)
    {
      const int oz = s / 9 - 1, oy = (s / 3) % 3 - 1, ox = s % 3 - 1;
      const int jx = X + ox, jy = Y + oy, jz = Z + oz;
      if (jx < 0 || jx >= cd[0] || jy < 0 || jy >= cd[1] || jz < 0 || jz >= cd[2]) continue;
      Ac.col.push_back((i32)(((i64)jz * cd[1] + jy) * cd[0] + jx));
      Ac.val.push_back(slot[(size_t)I * 27 + s]);
    }
    Ac.rp[I + 1] = (i64)Ac.col.size();
  }
}

// Exact spectrum bounds of D^-1 A (dense symmetric eigenvalues of D^-1/2 A D^-1/2), small n.
void spectrum_bounds(const HostCsr &A, i64 n, double &lo, double &hi)
{
  std::vector<double> d(n), S((size_t)n * n, 0.0), w, Z;
  for (i64 r = 0; r < n; ++r)
    for (i64 k = A.rp[r]; k < A.rp[r + 1]; ++k)
      if (A.col[k] == r) d[r] = A.val[k];
  for (i64 r = 0; r < n; ++r)
    for (i64 k = A.rp[r]; k < A.rp[r + 1]; ++k)
      S[(size_t)r * n + A.col[k]] = A.val[k] / std::sqrt(d[r] * d[A.col[k]]);
  sym_eig((int)n, S, w, Z);
  lo = w.front();
  hi = w.back();
  EIG_CHECK(lo > 0.0, EIG_ERR_BREAKDOWN, "multigrid: the coarsest operator is not positive definite");
}

void alloc_level(MgLevel &L, int m, hipStream_t s)
{
  const size_t bytes = (size_t)std::max<i64>(L.n, 1) * m * sizeof(double);
  L.dinv = new DevBuf((size_t)std::max<i64>(L.n, 1) * sizeof(double));
  L.B = new DevBuf(bytes);
  L.T = new DevBuf(bytes);
  for (auto &c : L.C) c = new DevBuf(bytes);
  (void)s;
}

// V_l b: the V-cycle on level l (all buffers n_l x m, ld = n_l); returns the level buffer (one of
// C[0..3]) that holds the result.  Residuals come from the SpMM's residual epilogue (T = b - A x in
// one pass), the smoothers' zero start is not read (box kernels), and the smoothed iterate stays where
// cheb_solve left it (the post-smoother takes the three other C buffers).
double *vcycle(eig_mg_s &mg, size_t l, i64 m, const double *b)
{
  MgLevel &L = mg.lev[l];
  hipStream_t s = mg.ctx->stream;
  double *C[4] = {L.C[0]->d(), L.C[1]->d(), L.C[2]->d(), L.C[3]->d()};
  if (l + 1 == mg.lev.size())
    return cheb_solve(*L.A, m, L.cdeg, L.clo, L.chi, b, L.dinv->d(), C[0], C[1], C[2], s);
  MgLevel &Cl = mg.lev[l + 1];
  const double lo = L.lmax / mg.ratio, hi = L.lmax;
  double *x = cheb_solve(*L.A, m, mg.nu, lo, hi, b, L.dinv->d(), C[0], C[1], C[2], s);
  double *T = L.T->d();
  launch_resid_mv8(*L.A, m, x, b, T, s);  // T = b - A x
  launch_mg_restrict(L.dim, Cl.dim, m, L.n, Cl.n, T, Cl.B->d(), s);
  const double *xc = vcycle(mg, l + 1, m, Cl.B->d());
  launch_mg_prolong_add(L.dim, Cl.dim, m, L.n, Cl.n, xc, x, s);
  launch_resid_mv8(*L.A, m, x, b, T, s);  // T = b - A x
  // x += post-smoothing correction: a degree-2 smoother on the row-class image adds its x_2 in
  // place (cheb_solve's first step, its gamma and omega_1)
  const double gamma = 2.0 / (lo + hi), mu = (hi - lo) / (hi + lo);
  if (mg.nu == 2 && launch_box_cheb_first_add(*L.A, m, T, 1.0 / (1.0 - 0.5 * mu * mu), gamma, x, s)) return x;
  double *q[3];
  for (int i = 0, j = 0; i < 4; ++i)
    if (C[i] != x) q[j++] = C[i];
  const double *p = cheb_solve(*L.A, m, mg.nu, lo, hi, T, L.dinv->d(), q[0], q[1], q[2], s);
  launch_mv8_axpby(L.n, m, L.n, 1.0, p, 1.0, x, s);
  return x;
}

}  // namespace

namespace eigmi {

// X = S_cycles B (window-layout pointers of the level-0 matrix, m columns), stream-ordered.
void mg_apply(eig_mg_s &mg, i64 m, const double *B, double *X, int cycles)
{
  MgLevel &L = mg.lev[0];
  hipStream_t s = mg.ctx->stream;
  EIG_CHECK(m > 0 && m % 8 == 0 && m <= mg.max_cols && cycles >= 1, EIG_ERR_ARG,
            "multigrid solve: 8 <= m <= max_cols (multiple of 8), cycles >= 1");
  const size_t bytes = (size_t)L.n * m * sizeof(double);
  double *R = L.B->d();
  const double *rhs = B;  // residual of the current iterate (B itself before the first correction)
  for (int it = 0; it < cycles; ++it)
  {
    const double *E = vcycle(mg, 0, m, rhs);
    // r -= A e (in place after the first iteration) and X = E / X += E: one pass on the row-class
    // image (the residual kernel's epilogue also writes X), a copy or axpby and the residual
    // otherwise
    if (it + 1 < cycles && launch_box_resid_acc(*L.A, m, E, rhs, R, X, it == 0, s))
    {
      rhs = R;
      continue;
    }
    if (it == 0)
      EIG_HIP(hipMemcpyAsync(X, E, bytes, hipMemcpyDeviceToDevice, s));
    else
      launch_mv8_axpby(L.n, m, L.n, 1.0, E, 1.0, X, s);
    if (it + 1 < cycles)
    {
      launch_resid_mv8(*L.A, m, E, rhs, R, s);
      rhs = R;
    }
  }
}

}  // namespace eigmi

namespace eigmi {
eig_mat_s *mg_matrix(const eig_mg_s &mg) { return mg.lev.front().A; }
int mg_max_cols(const eig_mg_s &mg) { return mg.max_cols; }
}  // namespace eigmi

extern "C" int eig_mg_create(eig_mat_t A, int nx, int ny, int nz, int max_cols, int smooth_degree, double smooth_ratio,
                             eig_mg_t *out)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && out && nx > 0 && ny > 0 && nz > 0 && max_cols >= 8 && max_cols % 8 == 0 && smooth_degree >= 1 &&
                  smooth_ratio > 1.0,
              EIG_ERR_ARG, "eig_mg_create: bad argument");
    EIG_CHECK(A->br == 1 && A->bc == 1, EIG_ERR_BLOCKSIZE, "eig_mg_create: FieldMatrix<double,1,1> only");
    EIG_CHECK(!A->ctx->distributed() && A->nb_rows == A->nb_cols && A->window == A->nb_rows, EIG_ERR_ARG,
              "eig_mg_create: square single-rank matrix required");
    EIG_CHECK((i64)nx * ny * nz == A->nb_rows, EIG_ERR_SHAPE, "eig_mg_create: nx * ny * nz must equal the rows");
    {
      // the coarsest level is solved through a dense host eigenvalue problem (spectrum_bounds): coarsening
      // halves every direction and stops at a direction below 3 nodes, so a flat grid (e.g. nz = 1, or
      // 256 x 256 x 4) would end far above 64 rows -- refuse it instead of an O(n^3) dense solve
      int d[3] = {nx, ny, nz};
      i64 n = A->nb_rows;
      while (n > 64 && d[0] >= 3 && d[1] >= 3 && d[2] >= 3)
      {
        for (int &x : d) x /= 2;
        n = (i64)d[0] * d[1] * d[2];
      }
      EIG_CHECK(n <= kMgMaxCoarse, EIG_ERR_ARG,
                "eig_mg_create: the grid coarsens only to " + std::to_string(n) + " rows (a direction falls below 3 "
                "nodes first; at most " + std::to_string(kMgMaxCoarse) + " rows are solved densely): semi-"
                "coarsening of flat grids is not implemented");
    }
    eig_ctx_t ctx = A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    auto *mg = new eig_mg_s();
    try
    {
      mg->ctx = ctx;
      mg->max_cols = max_cols;
      mg->nu = smooth_degree;
      mg->ratio = smooth_ratio;
      HostCsr h;
      mat_download_bcsr(*A, h.rp, h.col, h.val);
      MgLevel L0;
      L0.A = A;
      L0.dim[0] = nx, L0.dim[1] = ny, L0.dim[2] = nz;
      L0.n = A->nb_rows;
      mg->lev.push_back(L0);
      for (;;)
      {
        MgLevel &F = mg->lev.back();
        F.lmax = gershgorin(h, F.n);
        alloc_level(F, max_cols, s);
        launch_diag_inv(*F.A, F.dinv->d(), s);
        const bool last = F.n <= 64 || F.dim[0] < 3 || F.dim[1] < 3 || F.dim[2] < 3;
        if (last)
        {
          spectrum_bounds(h, F.n, F.clo, F.chi);
          F.clo *= 0.999;
          F.chi *= 1.001;
          const double kappa = F.chi / F.clo, rho = (std::sqrt(kappa) - 1.0) / (std::sqrt(kappa) + 1.0);
          F.cdeg = rho > 0.0 ? (int)std::ceil(std::log(0.5e-15) / std::log(rho)) : 1;
          F.cdeg = std::min(std::max(F.cdeg, 1), 2000);
          break;
        }
        MgLevel C;
        for (int d = 0; d < 3; ++d) C.dim[d] = F.dim[d] / 2;
        C.n = (i64)C.dim[0] * C.dim[1] * C.dim[2];
        HostCsr hc;
        galerkin(h, F.dim, C.dim, hc);
        eig_mat_t Ac = nullptr;
        const int rc = eig_mat_create_bcsr(ctx, C.n, C.n, 1, 1, hc.rp.data(), hc.col.data(), hc.val.data(), &Ac);
        if (rc != EIG_OK) throw Error(rc, std::string("multigrid: coarse upload: ") + eig_last_error(ctx));
        C.A = Ac;
        C.own = true;
        mg->lev.push_back(C);
        h = std::move(hc);
      }
      EIG_HIP(hipStreamSynchronize(s));
    }
    catch (...)
    {
      delete mg;
      throw;
    }
    *out = mg;
  });
}

extern "C" int eig_mg_info(eig_mg_t mg, int *levels, int64_t *coarse_rows, int *coarse_degree, double *lmax_fine)
{
  return guard(mg ? mg->ctx : nullptr, [&] {
    EIG_CHECK(mg, EIG_ERR_ARG, "eig_mg_info: null handle");
    if (levels) *levels = (int)mg->lev.size();
    if (coarse_rows) *coarse_rows = mg->lev.back().n;
    if (coarse_degree) *coarse_degree = mg->lev.back().cdeg;
    if (lmax_fine) *lmax_fine = mg->lev.front().lmax;
  });
}

extern "C" int eig_mg_solve(eig_mg_t mg, int64_t m, const double *B, double *X, int cycles, double *resid_host)
{
  return guard(mg ? mg->ctx : nullptr, [&] {
    EIG_CHECK(mg && B && X, EIG_ERR_ARG, "eig_mg_solve: null argument");
    EIG_CHECK(X != B, EIG_ERR_ARG, "eig_mg_solve: X must not alias B");
    eig_ctx_t ctx = mg->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    mg_apply(*mg, m, B, X, cycles);
    if (resid_host)
    {
      // max over columns of ||B - A X|| / ||B||
      MgLevel &L = mg->lev[0];
      double *T = L.T->d();
      double *dp = (double *)ctx_buffer(ctx, 9, (size_t)2 * m * sizeof(double));
      launch_resid_mv8(*L.A, m, X, B, T, s);
      launch_dot_diag_mv8(L.n, m, T, T, dp, 0, s, ctx->red);
      launch_dot_diag_mv8(L.n, m, B, B, dp + m, 0, s, ctx->red);
      std::vector<double> h((size_t)2 * m);
      EIG_HIP(hipMemcpyAsync(h.data(), dp, h.size() * sizeof(double), hipMemcpyDeviceToHost, s));
      EIG_HIP(hipStreamSynchronize(s));
      double r = 0.0;
      for (i64 j = 0; j < m; ++j) r = std::max(r, h[j] > 0.0 ? std::sqrt(h[j] / std::max(h[m + j], 1e-300)) : 0.0);
      *resid_host = r;
    }
    EIG_HIP(hipStreamSynchronize(s));
  });
}

extern "C" int eig_mg_destroy(eig_mg_t mg)
{
  if (!mg) return EIG_OK;
  (void)hipSetDevice(mg->ctx->device);
  (void)hipStreamSynchronize(mg->ctx->stream);
  delete mg;
  return EIG_OK;
}
