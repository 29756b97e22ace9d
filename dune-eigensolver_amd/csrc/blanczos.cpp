// blanczos.cpp -- block Lanczos for the symmetric-definite pencil K x = lambda M x (config C5):
// M-inner-product block Lanczos on the operator M^-1 K, with
//   * K V_j on the SELL image (k_sell_mv8),
//   * M^-1 by the Chebyshev-Jacobi semi-iteration fused into the M SpMM (k_sell_mv8<kCheb>) --
//     reduction-free, so a distributed run exchanges halos but never allreduces inside the solve,
//   * full re-orthogonalisation: two classical Gram-Schmidt passes in the M-inner product (the
//     tall-skinny panel V^T (M Z) on MFMA, then Z -= V C),
//   * CholQR2 in the M-inner product for the new block (Gram on MFMA, 32x32 Cholesky on the host).
// The reference reaches the same pencil through GeneralizedInverse (UMFPACK LU + subspace
// iteration, eigensolver.hh:204-351) or ARPACK shift-invert (arpack_geneo_wrapper.hh:581-658);
// both need a sparse factorisation, which does not exist at C5's size (hard part 4).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <random>
#include <vector>

#include "internal.h"

using namespace eigmi;

struct eig_blanczos_s {
  eig_mat_s *K = nullptr, *M = nullptr;
  int b = 32, max_steps = 0, k = 0, degree = 36;
  double lmin = 0.5, lmax = 2.5;
  // spectral transformation (eig_blanczos_create_si): Lanczos on OP = Ks^-1 M, Ks = K - sigma M,
  // the inner solve by `degree` Chebyshev-Jacobi steps on Ks with D^-1 Ks in [lmin, lmax]
  bool si = false;
  eig_mat_s *Ks = nullptr;
  double sigma = 0.0;
  // multigrid inner solve (eig_blanczos_create_si_mg): `cycles` V-cycle iterations instead of the
  // Chebyshev-Jacobi solve
  eig_mg_s *mg = nullptr;
  int cycles = 0;
  long long cholqr_recomputed = 0;  // CholQR2 second passes that recomputed M Z (ill-conditioned blocks)
  i64 ld = 0, own = 0, n = 0;
  DevBuf *V = nullptr;                   // (max_steps + 1) * b columns, window layout
  DevBuf *W = nullptr, *Xa = nullptr, *Xb = nullptr, *Xc = nullptr, *MZ = nullptr;  // b columns each
  DevBuf *dinv = nullptr;                // 1 / diag(M), owned rows
  DevBuf *small = nullptr;               // Gram / coefficient panels
  DevBuf *chol = nullptr;                // CholQR on the device: R, Rtot (b x b each) and a flag
  std::vector<double> A, B;              // host: A_j (b x b), B_{j+1} (b x b, upper) per step
  ~eig_blanczos_s()
  {
    delete V;
    delete W;
    delete Xa;
    delete Xb;
    delete Xc;
    delete MZ;
    delete dinv;
    delete small;
    delete chol;
  }
};

namespace {
// the matrix whose diagonal / Chebyshev solve the operator uses: M (M^-1 K) or Ks (shift-invert)
eig_mat_s &solve_mat(eig_blanczos_s &w) { return w.si ? *w.Ks : *w.M; }
}  // namespace

namespace {

// Exchange the ghost rows of every column block of a window-layout multivector.
void halo_mv(const eig_mat_s &A, double *X, i64 m, hipStream_t s)
{
  if (!A.ctx->distributed()) return;
  for (i64 c = 0; c < m / 8; ++c) halo_exchange(A, X + c * A.window * 8, s, nullptr, 8);
}

// Chebyshev-Jacobi semi-iteration (Golub-Varga three-term form) for M X = Bv, `degree` steps on
// the spectrum bounds [lmin, lmax] of diag(M)^-1 M: x_1 = gamma D^-1 b, then degree - 1 fused
// steps  x_{k+1} = omega_{k+1} (x_k + gamma D^-1 (b - M x_k) - x_{k-1}) + x_{k-1}.  Returns the
// buffer (Xa, Xb or Xc) that holds x_degree.  Error in the D-norm <= 2 rho^degree,
// rho = (sqrt(kappa) - 1) / (sqrt(kappa) + 1), kappa = lmax / lmin.
// Xc (optional third buffer): on the box kernel x_{k+1} goes to a buffer of its own instead of over
// the x_{k-1} it reads (interleaved A/B at 256^3: 4.23 vs 4.28 ms per launch; box-to-box spread of
// the same launch is 4.2-4.8 ms).
}  // namespace

namespace eigmi {
double *cheb_solve(eig_mat_s &M, i64 m, int degree, double lmin, double lmax, const double *Bv, const double *dinv,
                   double *Xa, double *Xb, double *Xc, hipStream_t s)
{
  const i64 n = M.nb_rows, ld = M.window, own = M.own_offset;
  const double gamma = 2.0 / (lmin + lmax), mu = (lmax - lmin) / (lmax + lmin);
  double omega = 1.0 / (1.0 - 0.5 * mu * mu);  // omega_1
  // Row-class image (one rank): x_1 = gamma D^-1 b is never stored -- the first step forms it while
  // b's planes enter the LDS ring (x_2 straight from b), the second forms x_{k-1} = x_1 from the
  // row's b.  Same arithmetic as the k_cheb_init + box-step chain below.
  if (degree >= 2 && Xc && !M.ctx->distributed() && launch_box_cheb_first(M, m, Bv, omega, gamma, Xa, s))
  {
    if (degree == 2) return Xa;
    omega = 1.0 / (1.0 - 0.25 * mu * mu * omega);
    EIG_CHECK(launch_box_cheb_second(M, m, Xa, Bv, omega, gamma, Xc, s), EIG_ERR_ARG,
              "Chebyshev: second row-class step refused");
    double *x2 = Xa;
    Xa = Xc;  // x_3
    Xc = Xb;
    Xb = x2;
    for (int k = 3; k < degree; ++k)
    {
      omega = 1.0 / (1.0 - 0.25 * mu * mu * omega);
      launch_box_cheb(M, m, Xa, Xb, Bv, dinv, omega, gamma, s, Xc);  // Xc = x_{k+1}
      double *t = Xb;
      Xb = Xa;
      Xa = Xc;
      Xc = t;
    }
    return Xa;
  }
  launch_cheb_init(n, ld, own, m, Bv, dinv, gamma, Xa, s);
  if (degree <= 1) return Xa;
  const bool oop = Xc && m % 32 == 0 && box_prepare(M);
  // x_0 = 0: the box kernel (a third output buffer) takes it as "not read"; the in-place kernels
  // read a cleared buffer
  if (!oop) EIG_HIP(hipMemsetAsync(Xb, 0, (size_t)ld * m * sizeof(double), s));
  for (int k = 1; k < degree; ++k)
  {
    if (k > 1) omega = 1.0 / (1.0 - 0.25 * mu * mu * omega);
    halo_mv(M, Xa, m, s);
    if (oop)
    {
      launch_box_cheb(M, m, Xa, k == 1 ? nullptr : Xb, Bv, dinv, omega, gamma, s, Xc);  // Xc = x_{k+1}
      double *t = Xb;
      Xb = Xa;
      Xa = Xc;
      Xc = t;
    }
    else
    {
      launch_cheb_step(M, m, Xa, Xb, Bv, dinv, omega, gamma, s);
      std::swap(Xa, Xb);
    }
  }
  return Xa;
}
}  // namespace eigmi

namespace {
double *dptr(DevBuf *b) { return b->d(); }

// R0 diagonal spread beyond which CholQR2's second pass recomputes M Z instead of reusing (M Z) R0^-1
constexpr double kCholQrReuseCond = 1e4;

// Z (b columns) = Vdst R with Vdst M-orthonormal (CholQR twice); R (b x b upper, row-major) on
// the host.  Vdst may equal Z.  The b x b factorisations run on the device (k_chol_small: the host
// chol_upper / tri_upper_inv arithmetic).  One host round trip in the middle reads R0 back to pick
// the second pass (reuse M Z or recompute it, below), one at the end brings R and the breakdown
// flag back.  The pick is a heuristic: the spread of R0's diagonal is only a lower bound on
// cond(R0), so an ill-conditioned block with an even diagonal can still take the reuse path (its
// second pass then restores M-orthonormality to ~eps cond(Z) instead of ~eps).
void mcholqr2(eig_blanczos_s &w, double *Z, double *Vdst, std::vector<double> &Rtot)
{
  eig_mat_s &M = *w.M;
  eig_ctx_t ctx = M.ctx;
  hipStream_t s = ctx->stream;
  const int b = w.b;
  const i64 n = w.n, ld = w.ld, own = w.own;
  double *Gd = w.small->d();
  double *Sd = Gd + (size_t)b * b;
  double *Rd = w.chol->d(), *Rt = Rd + (size_t)b * b;
  int *flag = reinterpret_cast<int *>(Rt + (size_t)b * b);
  EIG_HIP(hipMemsetAsync(flag, 0, sizeof(int), s));
  halo_mv(M, Z, b, s);
  launch_sell_mv8(M, b, Z, dptr(w.MZ), s);
  launch_panel_gram(ctx, n, ld, b, b, Z + own * 8, dptr(w.MZ) + own * 8, Gd, s);
  allreduce_sum(ctx, Gd, (i64)b * b, s);
  launch_chol_small(b, 0, Gd, Rd, Sd, Rt, flag, s);  // Sd = R0^-1, Rt = R0
  // The second pass may reuse M Z updated by the same factor (row-local: M (Z R0^-1) = (M Z) R0^-1 up
  // to rounding) instead of a second M SpMM -- but that rounding gap is ~eps cond(Z), so for an
  // ill-conditioned block the second pass would no longer restore M-orthonormality to ~eps (CholQR2's
  // guarantee).  R0's diagonal decides (one small read-back): beyond kCholQrReuseCond the second pass
  // recomputes M (Z R0^-1).
  std::vector<double> r0((size_t)b * b);
  EIG_HIP(hipMemcpyAsync(r0.data(), Rd, r0.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  EIG_HIP(hipStreamSynchronize(s));
  double dmax = 0.0, dmin = HUGE_VAL;
  for (int i = 0; i < b; ++i)
  {
    const double d = std::fabs(r0[(size_t)i * b + i]);
    dmax = std::max(dmax, d);
    dmin = std::min(dmin, d);
  }
  const bool reuse = dmin > 0.0 && dmax <= kCholQrReuseCond * dmin;
  w.cholqr_recomputed += !reuse;
  if (reuse && b == 32)
  {
    // Z <- Z R0^-1 and the second pass's Gram (Z R0^-1)^T (M Z R0^-1) in one pass over Z and M Z
    // (k_cholqr_fold): M Z R0^-1 is never stored, Z R0^-1 is not read back
    launch_cholqr_fold(ctx, n, ld, Z + own * 8, dptr(w.MZ) + own * 8, Sd, Gd, s);
  }
  else
  {
    launch_panel_update(n, ld, ld, b, b, Z + own * 8, Sd, 1.0, 0.0, Z + own * 8, s);
    if (reuse)
      launch_panel_update(n, ld, ld, b, b, dptr(w.MZ) + own * 8, Sd, 1.0, 0.0, dptr(w.MZ) + own * 8, s);
    else
    {
      halo_mv(M, Z, b, s);
      launch_sell_mv8(M, b, Z, dptr(w.MZ), s);
    }
    launch_panel_gram(ctx, n, ld, b, b, Z + own * 8, dptr(w.MZ) + own * 8, Gd, s);
  }
  allreduce_sum(ctx, Gd, (i64)b * b, s);
  launch_chol_small(b, 1, Gd, Rd, Sd, Rt, flag, s);  // Sd = R1^-1, Rt <- R1 R0
  launch_panel_update(n, ld, ld, b, b, Z + own * 8, Sd, 1.0, 0.0, Vdst + own * 8, s);
  Rtot.assign((size_t)b * b, 0.0);
  int hflag = 0;
  EIG_HIP(hipMemcpyAsync(Rtot.data(), Rt, Rtot.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  EIG_HIP(hipMemcpyAsync(&hflag, flag, sizeof(int), hipMemcpyDeviceToHost, s));
  EIG_HIP(hipStreamSynchronize(s));
  EIG_CHECK(!hflag, EIG_ERR_BREAKDOWN,
            "block Lanczos: M-Gram of the new block is not positive definite (Krylov space exhausted)");
}

void check_pair(const eig_mat_s *K, const eig_mat_s *M)
{
  EIG_CHECK(K && M && K->ctx == M->ctx, EIG_ERR_ARG, "block Lanczos: K and M must share a context");
  EIG_CHECK(K->br == 1 && K->bc == 1 && M->br == 1 && M->bc == 1, EIG_ERR_BLOCKSIZE,
            "block Lanczos: FieldMatrix<double,1,1> only");
  EIG_CHECK(K->nb_rows == M->nb_rows && K->row_begin == M->row_begin && K->window == M->window &&
                K->own_offset == M->own_offset && K->nb_rows_global == M->nb_rows_global,
            EIG_ERR_SHAPE, "block Lanczos: K and M must have the same rows and column window");
  EIG_CHECK(K->nb_rows_global == K->nb_cols, EIG_ERR_SHAPE, "block Lanczos: square matrices required");
}

}  // namespace

namespace {
void blanczos_create(eig_mat_t K, eig_mat_t M, eig_mat_t Ks, double sigma, int block, int max_steps, int degree,
                     double lmin, double lmax, unsigned seed, eig_blanczos_t *out, eig_mg_t mg = nullptr,
                     int cycles = 0)
{
    EIG_CHECK(out && block >= 8 && block <= 32 && block % 8 == 0 && max_steps >= 1 && degree >= 1 && lmin > 0.0 &&
                  lmax > lmin,
              EIG_ERR_ARG, "eig_blanczos_create: block in {8,16,24,32}, max_steps >= 1, degree >= 1, 0 < lmin < lmax");
    check_pair(K, M);
    if (Ks) check_pair(Ks, M);
    EIG_CHECK((i64)(max_steps + 1) * block <= K->nb_rows_global, EIG_ERR_SHAPE,
              "eig_blanczos_create: (max_steps + 1) * block exceeds the matrix size");
    eig_ctx_t ctx = K->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    auto *w = new eig_blanczos_s();
    try
    {
      w->K = K;
      w->M = M;
      w->si = Ks != nullptr;
      w->Ks = Ks;
      w->sigma = sigma;
      w->mg = mg;
      w->cycles = cycles;
      w->b = block;
      w->max_steps = max_steps;
      w->degree = degree;
      w->lmin = lmin;
      w->lmax = lmax;
      w->ld = K->window;
      w->own = K->own_offset;
      w->n = K->nb_rows;
      const size_t blk = (size_t)w->ld * block * sizeof(double);
      w->V = new DevBuf(blk * (max_steps + 1));
      w->W = new DevBuf(blk);
      w->Xa = new DevBuf(blk);
      w->Xb = new DevBuf(blk);
      w->Xc = new DevBuf(blk);
      w->MZ = new DevBuf(blk);
      w->dinv = new DevBuf((size_t)std::max<i64>(w->n, 1) * sizeof(double));
      w->small = new DevBuf((size_t)(max_steps + 2) * block * block * sizeof(double) * 2);
      w->chol = new DevBuf((size_t)2 * block * block * sizeof(double) + 64);
      EIG_HIP(hipMemsetAsync(w->V->d(), 0, w->V->bytes(), s));
      for (DevBuf *d : {w->W, w->Xa, w->Xb, w->MZ}) EIG_HIP(hipMemsetAsync(d->d(), 0, d->bytes(), s));
      launch_diag_inv(Ks ? *Ks : *M, w->dinv->d(), s);
      // start block: mt19937(seed) + normal(0,1) in MultiVector fill order (block, row, col) over
      // the GLOBAL rows (eigensolver.hh:49-55), this rank keeps its own rows
      {
        const i64 ng = K->nb_rows_global, rb = K->row_begin, n = w->n;
        std::vector<double> h((size_t)w->ld * block, 0.0);
        std::mt19937 urbg{seed};
        std::normal_distribution<double> gen{0.0, 1.0};
        for (int c = 0; c < block / 8; ++c)
          for (i64 i = 0; i < ng; ++i)
            for (int j = 0; j < 8; ++j)
            {
              const double v = gen(urbg);
              if (i >= rb && i < rb + n) h[((size_t)c * w->ld + w->own + (i - rb)) * 8 + j] = v;
            }
        EIG_HIP(hipMemcpyAsync(w->Xa->d(), h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, s));
        EIG_HIP(hipStreamSynchronize(s));
      }
      std::vector<double> R;
      mcholqr2(*w, w->Xa->d(), w->V->d(), R);  // V_0 = M-orthonormal start block
    }
    catch (...)
    {
      delete w;
      throw;
    }
    *out = w;
}
}  // namespace

extern "C" int eig_blanczos_create(eig_mat_t K, eig_mat_t M, int block, int max_steps, int degree, double lmin,
                                   double lmax, unsigned seed, eig_blanczos_t *out)
{
  return guard(K ? K->ctx : nullptr, [&] {
    blanczos_create(K, M, nullptr, 0.0, block, max_steps, degree, lmin, lmax, seed, out);
  });
}

// Spectral transformation (shift-invert, ARPACK mode 3's operator, arpack_geneo_wrapper.hh:581-658):
// Lanczos in the M-inner product on OP = (K - sigma M)^-1 M, whose largest |theta| are the pencil's
// eigenvalues nearest sigma, lambda = sigma + 1 / theta -- the end of the spectrum GeneralizedInverse
// (eigensolver.hh:204-351) returns.  Ks = K - sigma M is given by the caller (Ks = K for sigma = 0);
// its solve is `degree` Chebyshev-Jacobi steps with the spectrum of diag(Ks)^-1 Ks in [lmin, lmax]
// (reduction-free, like the mass solve).
extern "C" int eig_blanczos_create_si(eig_mat_t K, eig_mat_t M, eig_mat_t Ks, double sigma, int block, int max_steps,
                                      int degree, double lmin, double lmax, unsigned seed, eig_blanczos_t *out)
{
  return guard(K ? K->ctx : nullptr, [&] {
    EIG_CHECK(Ks, EIG_ERR_ARG, "eig_blanczos_create_si: Ks = K - sigma M required (K itself for sigma = 0)");
    blanczos_create(K, M, Ks, sigma, block, max_steps, degree, lmin, lmax, seed, out);
  });
}

// The same with the Ks solve by `cycles` multigrid V-cycle iterations (mg.cpp; mg built on Ks).
extern "C" int eig_blanczos_create_si_mg(eig_mat_t K, eig_mat_t M, eig_mat_t Ks, double sigma, eig_mg_t mg, int cycles,
                                         int block, int max_steps, unsigned seed, eig_blanczos_t *out)
{
  return guard(K ? K->ctx : nullptr, [&] {
    EIG_CHECK(Ks && mg && cycles >= 1, EIG_ERR_ARG, "eig_blanczos_create_si_mg: Ks, mg and cycles >= 1 required");
    EIG_CHECK(mg_matrix(*mg) == Ks && block <= mg_max_cols(*mg), EIG_ERR_ARG,
              "eig_blanczos_create_si_mg: mg must be built on Ks with max_cols >= block");
    blanczos_create(K, M, Ks, sigma, block, max_steps, 1, 0.5, 2.5, seed, out, mg, cycles);
  });
}

extern "C" int eig_blanczos_step(eig_blanczos_t w, int steps, eig_blanczos_timing *timing)
{
  return guard(w ? w->K->ctx : nullptr, [&] {
    EIG_CHECK(w && steps >= 0, EIG_ERR_ARG, "eig_blanczos_step: bad argument");
    EIG_CHECK(w->k + steps <= w->max_steps, EIG_ERR_ARG, "eig_blanczos_step: more steps than max_steps");
    eig_ctx_t ctx = w->K->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int b = w->b;
    const i64 n = w->n, ld = w->ld, own = w->own;
    const size_t bs = (size_t)ld * b;  // doubles per basis block
    std::vector<hipEvent_t> ev((size_t)5 * steps);
    for (auto &e : ev) EIG_HIP(hipEventCreate(&e));
    struct EvGuard {
      std::vector<hipEvent_t> &v;
      ~EvGuard()
      {
        for (auto &e : v) (void)hipEventDestroy(e);
      }
    } evg{ev};
    double *Ad = w->small->d();
    double *Cd = Ad + (size_t)b * b;
    for (int i = 0; i < steps; ++i)
    {
      const int j = w->k;
      hipEvent_t *e = &ev[(size_t)5 * i];
      double *Vj = w->V->d() + (size_t)j * bs;
      EIG_HIP(hipEventRecord(e[0], s));
      double *Z;
      if (!w->si)
      {
        // W = K V_j;  Z = M^-1 W;  A_j = V_j^T W is block j of the first CGS pass's V^T W below
        halo_mv(*w->K, Vj, b, s);
        launch_sell_mv8(*w->K, b, Vj, w->W->d(), s);
        EIG_HIP(hipEventRecord(e[1], s));
        Z = cheb_solve(*w->M, b, w->degree, w->lmin, w->lmax, w->W->d(), w->dinv->d(), w->Xa->d(), w->Xb->d(),
                       w->Xc->d(), s);
        EIG_HIP(hipEventRecord(e[2], s));
      }
      else
      {
        // W = M V_j;  Z = Ks^-1 W = OP V_j;  A_j = V_j^T M Z = W^T Z
        halo_mv(*w->M, Vj, b, s);
        launch_sell_mv8(*w->M, b, Vj, w->W->d(), s);
        EIG_HIP(hipEventRecord(e[1], s));
        if (w->mg)
        {
          mg_apply(*w->mg, b, w->W->d(), w->Xa->d(), w->cycles);
          Z = w->Xa->d();
        }
        else
          Z = cheb_solve(*w->Ks, b, w->degree, w->lmin, w->lmax, w->W->d(), w->dinv->d(), w->Xa->d(), w->Xb->d(),
                         w->Xc->d(), s);
        launch_panel_gram(ctx, n, ld, b, b, w->W->d() + own * 8, Z + own * 8, Ad, s);
        allreduce_sum(ctx, Ad, (i64)b * b, s);
        EIG_HIP(hipEventRecord(e[2], s));
      }
      // two CGS passes against V_0..V_j in the M-inner product: C = V^T (M Z), Z -= V C
      const i64 m1 = (i64)(j + 1) * b;
      for (int pass = 0; pass < 2; ++pass)
      {
        // first pass of the M^-1 K operator: M Z = M (M^-1 W) = W to the mass solve's accuracy
        // (2 rho^degree), so W stands in for the M SpMM
        const double *MZ = w->MZ->d();
        if (pass == 0 && !w->si)
          MZ = w->W->d();
        else
        {
          halo_mv(*w->M, Z, b, s);
          launch_sell_mv8(*w->M, b, Z, w->MZ->d(), s);
        }
        launch_panel_gram(ctx, n, ld, m1, b, w->V->d() + own * 8, MZ + own * 8, Cd, s);
        allreduce_sum(ctx, Cd, m1 * b, s);
        if (pass == 0 && !w->si)  // A_j = V_j^T W: rows j b .. (j + 1) b of C
          EIG_HIP(hipMemcpyAsync(Ad, Cd + (size_t)j * b * b, (size_t)b * b * sizeof(double), hipMemcpyDeviceToDevice, s));
        launch_panel_update(n, ld, ld, m1, b, w->V->d() + own * 8, Cd, -1.0, 1.0, Z + own * 8, s);
      }
      EIG_HIP(hipEventRecord(e[3], s));
      std::vector<double> Ah((size_t)b * b);
      EIG_HIP(hipMemcpyAsync(Ah.data(), Ad, Ah.size() * sizeof(double), hipMemcpyDeviceToHost, s));
      std::vector<double> R;
      mcholqr2(*w, Z, w->V->d() + (size_t)(j + 1) * bs, R);  // syncs
      EIG_HIP(hipEventRecord(e[4], s));
      for (int r = 0; r < b; ++r)
        for (int c = r + 1; c < b; ++c)
          Ah[(size_t)r * b + c] = Ah[(size_t)c * b + r] = 0.5 * (Ah[(size_t)r * b + c] + Ah[(size_t)c * b + r]);
      w->A.insert(w->A.end(), Ah.begin(), Ah.end());
      w->B.insert(w->B.end(), R.begin(), R.end());
      w->k = j + 1;
    }
    EIG_HIP(hipStreamSynchronize(s));
    if (timing)
    {
      std::memset(timing, 0, sizeof(*timing));
      for (int i = 0; i < steps; ++i)
      {
        hipEvent_t *e = &ev[(size_t)5 * i];
        float t[4] = {0, 0, 0, 0};
        for (int q = 0; q < 4; ++q) EIG_HIP(hipEventElapsedTime(&t[q], e[q], e[q + 1]));
        timing->kspmm_ms += t[0];
        timing->cheb_ms += t[1];
        timing->orth_ms += t[2];
        timing->norm_ms += t[3];
      }
      if (steps > 0)
      {
        float tt = 0.f;
        EIG_HIP(hipEventElapsedTime(&tt, ev[0], ev[(size_t)5 * (steps - 1) + 4]));
        timing->total_ms = tt;
      }
      timing->steps = steps;
      timing->cheb_launches = (int64_t)steps * std::max(0, w->degree - 1) * sell_mv8_launches(b);
      timing->cholqr_recomputed = w->cholqr_recomputed;
    }
  });
}

namespace {
// The block tridiagonal T (k b x k b, row-major) of the k completed steps.
std::vector<double> assemble_T(const eig_blanczos_s &w)
{
  const int b = w.b, k = w.k, N = k * b;
  std::vector<double> T((size_t)N * N, 0.0);
  for (int j = 0; j < k; ++j)
  {
    for (int r = 0; r < b; ++r)
      for (int c = 0; c < b; ++c) T[(size_t)(j * b + r) * N + j * b + c] = w.A[((size_t)j * b + r) * b + c];
    if (j + 1 < k)  // T_{j+1,j} = B_{j+1}, T_{j,j+1} = B_{j+1}^T
      for (int r = 0; r < b; ++r)
        for (int c = 0; c < b; ++c)
        {
          const double v = w.B[((size_t)j * b + r) * b + c];
          T[(size_t)((j + 1) * b + r) * N + j * b + c] = v;
          T[(size_t)(j * b + c) * N + (j + 1) * b + r] = v;
        }
  }
  return T;
}
}  // namespace

extern "C" int eig_blanczos_tmatrix(eig_blanczos_t w, int *dim, double *T_host)
{
  return guard(w ? w->K->ctx : nullptr, [&] {
    EIG_CHECK(w && dim, EIG_ERR_ARG, "eig_blanczos_tmatrix: bad argument");
    *dim = w->k * w->b;
    if (T_host)
    {
      std::vector<double> T = assemble_T(*w);
      std::memcpy(T_host, T.data(), T.size() * sizeof(double));
    }
  });
}

extern "C" int eig_blanczos_ritz(eig_blanczos_t w, int nev, int which, double *eval_host, double *evec_host,
                                 double *resid_host)
{
  return guard(w ? w->K->ctx : nullptr, [&] {
    EIG_CHECK(w && eval_host && nev > 0, EIG_ERR_ARG, "eig_blanczos_ritz: bad argument");
    EIG_CHECK(which == EIG_WHICH_LA || which == EIG_WHICH_SA, EIG_ERR_ARG, "eig_blanczos_ritz: bad `which`");
    const int b = w->b, N = w->k * b;
    EIG_CHECK(w->k >= 1 && nev <= N, EIG_ERR_ARG, "eig_blanczos_ritz: take steps first (nev <= steps * block)");
    eig_ctx_t ctx = w->K->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    std::vector<double> T = assemble_T(*w), th, S;
    sym_eig(N, T, th, S);
    std::vector<int> pick(nev);
    if (!w->si)
      for (int i = 0; i < nev; ++i) pick[i] = (which == EIG_WHICH_LA) ? N - 1 - i : i;
    else
    {
      // the nev Ritz values of OP of largest |theta| (eigenvalues nearest sigma), ordered by
      // lambda = sigma + 1 / theta: ascending (SA) or descending (LA)
      std::vector<int> ord(N);
      for (int i = 0; i < N; ++i) ord[i] = i;
      std::stable_sort(ord.begin(), ord.end(), [&](int a, int c) { return std::fabs(th[a]) > std::fabs(th[c]); });
      ord.resize(nev);
      for (int i = 0; i < N; ++i) th[i] = th[i] != 0.0 ? w->sigma + 1.0 / th[i] : HUGE_VAL;
      std::stable_sort(ord.begin(), ord.end(), [&](int a, int c) {
        return which == EIG_WHICH_SA ? th[a] < th[c] : th[a] > th[c];
      });
      pick = ord;
    }
    for (int i = 0; i < nev; ++i) eval_host[i] = th[pick[i]];
    if (!evec_host && !resid_host) return;
    const i64 n = w->n, ld = w->ld, own = w->own;
    double *Sd = w->small->d();
    std::vector<double> Sh, rs(nev, 0.0);
    // 32 Ritz vectors at a time: Y = V_{0..k-1} S(:, cols) into Xa; KY into W, MY into MZ
    for (int c0 = 0; c0 < nev; c0 += 32)
    {
      const int nc = std::min(32, nev - c0), m2 = (nc + 7) / 8 * 8;
      Sh.assign((size_t)N * m2, 0.0);
      for (int q = 0; q < N; ++q)
        for (int c = 0; c < nc; ++c) Sh[(size_t)q * m2 + c] = S[(size_t)q * N + pick[c0 + c]];
      DevBuf Sb(Sh.size() * sizeof(double));
      EIG_HIP(hipMemcpyAsync(Sb.d(), Sh.data(), Sh.size() * sizeof(double), hipMemcpyHostToDevice, s));
      double *Y = w->Xa->d();
      EIG_HIP(hipMemsetAsync(Y, 0, (size_t)ld * m2 * sizeof(double), s));
      launch_panel_update(n, ld, ld, N, m2, w->V->d() + own * 8, Sb.d(), 1.0, 0.0, Y + own * 8, s);
      std::vector<double> hy((size_t)ld * m2), hk, hm;
      if (resid_host)
      {
        halo_mv(*w->K, Y, m2, s);
        launch_sell_mv8(*w->K, m2, Y, w->W->d(), s);
        launch_sell_mv8(*w->M, m2, Y, w->MZ->d(), s);
        hk.resize(hy.size());
        hm.resize(hy.size());
        EIG_HIP(hipMemcpyAsync(hk.data(), w->W->d(), hk.size() * sizeof(double), hipMemcpyDeviceToHost, s));
        EIG_HIP(hipMemcpyAsync(hm.data(), w->MZ->d(), hm.size() * sizeof(double), hipMemcpyDeviceToHost, s));
      }
      EIG_HIP(hipMemcpyAsync(hy.data(), Y, hy.size() * sizeof(double), hipMemcpyDeviceToHost, s));
      EIG_HIP(hipStreamSynchronize(s));
      for (int c = 0; c < nc; ++c)
      {
        const int blk = c / 8, jj = c % 8;
        const double theta = th[pick[c0 + c]];
        double r2 = 0.0;
        for (i64 r = 0; r < n; ++r)
        {
          const size_t at = ((size_t)blk * ld + own + r) * 8 + jj;
          if (evec_host) evec_host[(size_t)(c0 + c) * n + r] = hy[at];
          if (resid_host)
          {
            const double d = hk[at] - theta * hm[at];
            r2 += d * d;
          }
        }
        rs[c0 + c] = r2;
      }
    }
    if (resid_host)
    {
      double *rd = Sd;
      EIG_HIP(hipMemcpyAsync(rd, rs.data(), nev * sizeof(double), hipMemcpyHostToDevice, s));
      allreduce_sum(ctx, rd, nev, s);
      EIG_HIP(hipMemcpyAsync(rs.data(), rd, nev * sizeof(double), hipMemcpyDeviceToHost, s));
      EIG_HIP(hipStreamSynchronize(s));
      for (int i = 0; i < nev; ++i) resid_host[i] = std::sqrt(rs[i]);
    }
  });
}

extern "C" int eig_blanczos_destroy(eig_blanczos_t w)
{
  if (!w) return EIG_OK;
  (void)hipSetDevice(w->K->ctx->device);
  (void)hipStreamSynchronize(w->K->ctx->stream);
  delete w;
  return EIG_OK;
}

// M^-1 B by the Chebyshev-Jacobi semi-iteration (the block Lanczos operator's inner solve).
extern "C" int eig_mass_solve_mv8(eig_mat_t M, int64_t m, int degree, double lmin, double lmax, const double *B,
                                  double *X)
{
  return guard(M ? M->ctx : nullptr, [&] {
    EIG_CHECK(M && B && X && m > 0 && m % 8 == 0 && degree >= 1 && lmin > 0.0 && lmax > lmin, EIG_ERR_ARG,
              "eig_mass_solve_mv8: bad argument");
    EIG_CHECK(M->br == 1 && M->bc == 1 && M->nb_rows_global == M->nb_cols, EIG_ERR_BLOCKSIZE,
              "eig_mass_solve_mv8: square FieldMatrix<double,1,1> only");
    EIG_CHECK(X != B, EIG_ERR_ARG, "eig_mass_solve_mv8: X must not alias B (B is read by every step)");
    eig_ctx_t ctx = M->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t bytes = (size_t)M->window * m * sizeof(double);
    DevBuf dinv((size_t)std::max<i64>(M->nb_rows, 1) * sizeof(double)), Xb(bytes), Xc(bytes);
    launch_diag_inv(*M, dinv.d(), s);
    EIG_HIP(hipMemsetAsync(X, 0, bytes, s));
    double *res = cheb_solve(*M, m, degree, lmin, lmax, B, dinv.d(), X, Xb.d(), Xc.d(), s);
    if (res != X) EIG_HIP(hipMemcpyAsync(X, res, bytes, hipMemcpyDeviceToDevice, s));
    EIG_HIP(hipStreamSynchronize(s));
  });
}

extern "C" int eig_panel_update_mv8(eig_ctx_t ctx, int64_t n, int64_t m1, int64_t m2, const double *Q, const double *S,
                                    double alpha, double beta, double *Y)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && Q && S && Y && n >= 0 && m1 >= 0 && m1 % 8 == 0 && m2 % 8 == 0 && m2 >= 8 && m2 <= 32,
              EIG_ERR_ARG, "eig_panel_update_mv8: m1 % 8 == 0, m2 in {8,16,24,32}");
    EIG_HIP(hipSetDevice(ctx->device));
    launch_panel_update(n, n, n, m1, m2, Q, S, alpha, beta, Y, ctx->stream);
  });
}

extern "C" int eig_panel_gram_mv8(eig_ctx_t ctx, int64_t n, int64_t m1, int64_t m2, const double *Q1, const double *Q2,
                                  double *G)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && Q1 && Q2 && G && n >= 0 && m1 > 0 && m2 > 0 && m1 % 8 == 0 && m2 % 8 == 0, EIG_ERR_ARG,
              "eig_panel_gram_mv8: bad argument");
    EIG_HIP(hipSetDevice(ctx->device));
    launch_panel_gram(ctx, n, n, m1, m2, Q1, Q2, G, ctx->stream);
  });
}
