// drivers.cpp -- host drivers over the device kernels:
//   eig_standard_largest  StandardLargest subspace iteration (eigensolver.hh:28-112)
//   eig_lanczos_run       the Lanczos three-term recurrence ARPACK's dsaupd runs around multMv
//                         (arpack_geneo_wrapper.hh:257-279, :621-632) -- the benchmark unit
//   eig_lanczos_solve     Lanczos with full DGKS re-orthogonalisation (ARPACK's conditional second pass) + Ritz extraction
#include <algorithm>
#include <complex>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "internal.h"

using namespace eigmi;

namespace {

bool distributed(const eig_mat_s &A) { return A.ctx->distributed(); }

// Page-locked, device-mapped host doubles and a timing-free event: the drivers' per-iteration
// stopping data.  The reducing kernel's last workgroup stores its sums straight into this memory
// through `dev` (no device-to-host copy launch per iteration); the event recorded after the kernel
// on the stream orders those stores before the host reads them.
struct PinnedDoubles {
  double *p = nullptr, *dev = nullptr;
  explicit PinnedDoubles(size_t n)
  {
    EIG_HIP(hipHostMalloc(reinterpret_cast<void **>(&p), (n ? n : 1) * sizeof(double), hipHostMallocMapped));
    EIG_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&dev), p, 0));
  }
  ~PinnedDoubles()
  {
    if (p) (void)hipHostFree(p);
  }
  PinnedDoubles(const PinnedDoubles &) = delete;
  PinnedDoubles &operator=(const PinnedDoubles &) = delete;
};
struct SyncEvent {
  hipEvent_t e = nullptr;
  SyncEvent() { EIG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming)); }
  ~SyncEvent()
  {
    if (e) (void)hipEventDestroy(e);
  }
  SyncEvent(const SyncEvent &) = delete;
  SyncEvent &operator=(const SyncEvent &) = delete;
};

}  // namespace

// ============================================================================================
// a12: StandardLargest (eigensolver.hh:28-112)
// ============================================================================================
extern "C" int eig_standard_largest(eig_mat_t A, double shift, double tol, int maxiter, int nev, unsigned seed,
                                    double *eval_host, double *evec_host, int *iters, int verbose)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && eval_host && nev > 0, EIG_ERR_ARG, "eig_standard_largest: bad argument");
    EIG_CHECK(A->br == A->bc, EIG_ERR_ARG, "StandardLargest: blocks of input matrix must be square");
    EIG_CHECK(A->br == 1, EIG_ERR_BLOCKSIZE,
              "matmul_sparse_tallskinny_blocked: only implemented for FieldMatrix<..,1,1>");
    EIG_CHECK(!distributed(*A), EIG_ERR_ARG, "eig_standard_largest: single rank only");
    eig_ctx_t ctx = A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const i64 n = A->nb_rows;
    const i64 m = (nev / 8 + std::min(nev % 8, 1)) * 8;  // eigensolver.hh:43
    // Three rotating n x m blocks: iteration k orthonormalises B[k % 3] in place (it holds A Q1 of
    // the previous basis, eigensolver.hh:78-81), multiplies it into B[(k + 1) % 3] (:84) and takes the
    // diagonal dots (:85).  So iteration k + 1 writes only B[(k + 1) % 3] and B[(k + 2) % 3], never
    // iteration k's basis, and is queued BEFORE the host reads iteration k's dots for the stopping
    // test (:87-102): the device never idles on the host's round trip.  If iteration k stops the loop,
    // the extra iteration's results are ignored.  The same kernels on the same inputs as the
    // reference's order (one SpMM per iteration from k = 2 on, see :78 below), so the iterates, the Ritz
    // values and the iteration count are bitwise those of the plain loop
    // (tests/test_gpu_drivers.py::test_standard_largest_reuses_product_bitwise).
    DevBuf B0(n * m * 8), B1(n * m * 8), B2(n * m * 8);
    double *B[3] = {B0.d(), B1.d(), B2.d()};
    PinnedDoubles hd(2 * (size_t)m);
    SyncEvent ev[2];
    {
      std::vector<double> h((size_t)(n * m));
      host_random_normal(n * m, seed, h.data());  // eigensolver.hh:50-55
      EIG_HIP(hipMemcpyAsync(B[0], h.data(), h.size() * 8, hipMemcpyHostToDevice, s));
      EIG_HIP(hipStreamSynchronize(s));
    }
    if (shift != 0.0) launch_shift_diag(*A, shift, s);  // eigensolver.hh:59-66
    orthonormalize_device(ctx, n, m, B[0], EIG_ORTHO_MGS); // eigensolver.hh:69
    // :78 of iteration k recomputes A Q1, which iteration k - 1's :84 product already holds (same
    // matrix, same input, deterministic kernel: bitwise the same block), so
    // only iteration 1 runs it.
    // m = 8 (nev <= 8: configs C1 / C2): the product also sums its window Gram (launch_spmm_dot_gram_mv8),
    // so the next iteration's MGS (:81) starts from it (launch_mgs_lookahead_gram) instead of reading
    // the block once more for its first look-ahead pass.  The same MGS steps on the same block; only
    // the Gram's summation order is the product's (eig_spmm_dot_gram_mv8 / eig_orthonormalize_gram_mv8
    // are the exported pair, tests/test_gpu_drivers.py runs the reference loop with them).
    DevBuf Gb(64 * 8), dscr(8 * 8);
    static const bool no_gram = std::getenv("EIGMI_NO_SPMM_GRAM") != nullptr;  // A/B: the round-5 loop
    const bool gram = m == 8 && mgs_lookahead_default() == 8 && !no_gram;
    if (maxiter > 1)  // :78 (k = 1)
    {
      if (gram)
        spmm_dot_gram_device(*A, B[0], B[1], dscr.d(), Gb.d());
      else
        launch_spmm_mv8(*A, m, B[0], B[1], s);
    }
    auto enqueue = [&](int k) {
      double *Q = B[k % 3], *P = B[(k + 1) % 3], *dp = hd.dev + (k & 1) * m;
      if (gram)
      {
        orthonormalize_device(ctx, n, m, Q, EIG_ORTHO_MGS, Gb.d());  // :81
        spmm_dot_gram_device(*A, Q, P, dp, Gb.d());                  // :84-85, dots to the host, Gram for :81
      }
      else
      {
        orthonormalize_device(ctx, n, m, Q, EIG_ORTHO_MGS);  // :81
        launch_spmm_dot_mv8(*A, m, Q, P, dp, s, ctx->red);   // :84-85, the dots straight to the host
      }
      EIG_HIP(hipEventRecord(ev[k & 1].e, s));
    };
    std::vector<double> s1(m, 0.0), s2(m, 0.0);
    int kk = 1, basis = 0;
    if (maxiter > 1) enqueue(1);
    for (int k = 1; k < maxiter; ++k)
    {
      kk = k;
      if (k + 1 < maxiter) enqueue(k + 1);  // look-ahead: queued before iteration k's stopping test
      EIG_HIP(hipEventSynchronize(ev[k & 1].e));
      for (i64 i = 0; i < m; ++i) s1[i] = hd.p[(k & 1) * m + i] - shift;
      double dist = 0.0;
      for (i64 i = 0; i < m; ++i) dist = std::max(dist, std::fabs(s1[i] - s2[i]));
      if (verbose > 0 && k > 1) fprintf(stdout, "Iter=%d %.17g\n", k, dist);
      std::swap(s1, s2);
      basis = k % 3;  // Q1 after the swap (:96)
      if (k > 1 && dist < tol) break;
    }
    for (int j = 0; j < nev; ++j) eval_host[j] = s2[j];
    if (evec_host)
    {
      // evec[j][i] = Q1(i, j): column j sits at Q1 + (j/8)*8n + i*8 + j%8 (after any look-ahead
      // iteration on the stream, which leaves this block alone)
      std::vector<double> h((size_t)(n * m));
      EIG_HIP(hipMemcpyAsync(h.data(), B[basis], h.size() * 8, hipMemcpyDeviceToHost, s));
      EIG_HIP(hipStreamSynchronize(s));
      for (int j = 0; j < nev; ++j)
        for (i64 i = 0; i < n; ++i) evec_host[(i64)j * n + i] = h[((j / 8) * n + i) * 8 + j % 8];
    }
    EIG_HIP(hipStreamSynchronize(s));  // the look-ahead iteration uses this call's buffers
    mgs_lookahead_check(ctx);          // a timed-out MGS barrier: EIG_ERR_HIP, never NaN with EIG_OK
    if (iters) *iters = kk;
  });
}

// ============================================================================================
// Inverse subspace iteration with exported LU factors
// ============================================================================================
namespace {

// The factors the inverse drivers apply: the caller's, or a host factorisation of `A` (owned).
struct LuRef {
  eig_lu_t lu = nullptr;
  bool owned = false;
  ~LuRef()
  {
    if (owned) eig_lu_destroy(lu);
  }
};

void factor_host(eig_mat_s &A, const std::vector<i64> &rp, const std::vector<i32> &c, const std::vector<double> &v,
                 LuRef &out)
{
  const int rc = eig_lu_create_bcsr(A.ctx, A.nb_rows, A.br, rp.data(), c.data(), v.data(), &out.lu);
  EIG_CHECK(rc == EIG_OK, rc, std::string("LU factorisation: ") + eig_last_error(A.ctx));
  out.owned = true;
}

void copy_evecs(eig_ctx_t ctx, const double *Q, i64 n, int nev, double *evec_host)
{
  if (!evec_host) return;
  const i64 m = (nev + 7) / 8 * 8;
  std::vector<double> h((size_t)(n * m));
  EIG_HIP(hipMemcpyAsync(h.data(), Q, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  EIG_HIP(hipStreamSynchronize(ctx->stream));
  for (int j = 0; j < nev; ++j)
    for (i64 i = 0; i < n; ++i) evec_host[(i64)j * n + i] = h[((j / 8) * n + i) * 8 + j % 8];
}

void random_block(eig_ctx_t ctx, i64 n, i64 m, unsigned seed, double *Q)
{
  std::vector<double> h((size_t)(n * m));
  host_random_normal(n * m, seed, h.data());  // eigensolver.hh:137-142 / :222-227
  EIG_HIP(hipMemcpyAsync(Q, h.data(), h.size() * 8, hipMemcpyHostToDevice, ctx->stream));
  EIG_HIP(hipStreamSynchronize(ctx->stream));
}

void check_inverse_matrix(const eig_mat_s *A, const char *who)
{
  EIG_CHECK(A->br == A->bc, EIG_ERR_ARG, std::string(who) + ": blocks of input matrix must be square");
  EIG_CHECK(A->br == 1, EIG_ERR_BLOCKSIZE, "matmul_sparse_tallskinny_blocked: only implemented for FieldMatrix<..,1,1>");
  EIG_CHECK(!distributed(*A), EIG_ERR_ARG, std::string(who) + ": single rank only");
  EIG_CHECK(A->nb_rows == A->nb_cols, EIG_ERR_SHAPE, std::string(who) + ": square matrix required");
}

}  // namespace

extern "C" int eig_standard_inverse(eig_mat_t A, eig_lu_t lu, double shift, double tol, int maxiter, int nev,
                                    unsigned seed, double *eval_host, double *evec_host, int *iters, int verbose)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && eval_host && nev > 0, EIG_ERR_ARG, "eig_standard_inverse: bad argument");
    check_inverse_matrix(A, "StandardInverse");
    eig_ctx_t ctx = A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const i64 n = A->nb_rows;
    const i64 m = (nev / 8 + std::min(nev % 8, 1)) * 8;  // eigensolver.hh:133
    // basis ping-pong B[0] / B[1] and a product block Z: iteration k solves from B[(k - 1) % 2] into
    // B[k % 2], so the queued iteration k + 1 never touches iteration k's basis (look-ahead over the
    // host's stopping test, as eig_standard_largest)
    DevBuf Q1b(n * m * 8), Q2b(n * m * 8), Zb(n * m * 8);
    double *Bk[2] = {Q1b.d(), Q2b.d()}, *Z = Zb.d();
    PinnedDoubles hd(2 * (size_t)m);
    SyncEvent ev[2];
    random_block(ctx, n, m, seed, Bk[0]);
    if (shift != 0.0) launch_shift_diag(*A, shift, s);  // :145-153 (mutates A)
    LuRef F;                                           // :156 UMFPackFactorizedMatrix<ISTLM> F(A, 1)
    if (lu)
      F.lu = lu;
    else
    {
      std::vector<i64> rp;
      std::vector<i32> c;
      std::vector<double> v;
      EIG_HIP(hipStreamSynchronize(s));
      mat_download_bcsr(*A, rp, c, v);
      factor_host(*A, rp, c, v, F);
    }
    EIG_CHECK(lu_size(F.lu) == n, EIG_ERR_SHAPE,
              "matmul_inverse_tallskinny_blocked: Factorization does not match size of Qout/Qin");
    orthonormalize_device(ctx, n, m, Bk[0], EIG_ORTHO_MGS);  // :159
    auto enqueue = [&](int k) {
      double *Q = Bk[k % 2], *dp = hd.dev + (k & 1) * m;
      // :168 Q2 = A^-1 Q1.  The factor apply may overwrite its input (kernels_cpp.hh:659, and
      // launch_inverse_mv8 does), and with the look-ahead iteration k + 1 runs before the host knows
      // whether iteration k stopped the loop -- so the apply takes a copy of the basis (in Z), and a
      // stop at k still returns basis k intact (round 6: tests/test_inverse.py caught the clobbered
      // eigenvectors of a tolerance-driven stop)
      EIG_HIP(hipMemcpyAsync(Z, Bk[(k + 1) % 2], (size_t)n * m * sizeof(double), hipMemcpyDeviceToDevice, s));
      lu_inverse_device(F.lu, m, Z, Q, s);
      orthonormalize_device(ctx, n, m, Q, EIG_ORTHO_MGS);  // :171
      launch_spmm_dot_mv8(*A, m, Q, Z, dp, s, ctx->red);    // :174-175 (the product only feeds the dots)
      EIG_HIP(hipEventRecord(ev[k & 1].e, s));
    };
    std::vector<double> s1(m, 0.0), s2(m, 0.0);
    int kk = 1, basis = 0;
    if (maxiter > 1) enqueue(1);
    for (int k = 1; k < maxiter; ++k)
    {
      kk = k;
      if (k + 1 < maxiter) enqueue(k + 1);  // look-ahead: queued before iteration k's stopping test
      EIG_HIP(hipEventSynchronize(ev[k & 1].e));
      for (i64 i = 0; i < m; ++i) s1[i] = hd.p[(k & 1) * m + i] - shift;
      double dist = 0.0;
      for (i64 i = 0; i < m; ++i) dist = std::max(dist, std::fabs(s1[i] - s2[i]));
      if (verbose > 0 && k > 1) fprintf(stdout, "iter=%d %.17g\n", k, dist);
      std::swap(s1, s2);
      basis = k % 2;  // Q1 after the swap
      if (k > 1 && dist < tol) break;
    }
    for (int j = 0; j < nev; ++j) eval_host[j] = s2[j];
    copy_evecs(ctx, Bk[basis], n, nev, evec_host);  // (stream order: after any queued iteration)
    EIG_HIP(hipStreamSynchronize(s));
    mgs_lookahead_check(ctx);
    if (iters) *iters = kk;
  });
}

extern "C" int eig_generalized_inverse(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double shift, double reg, double tol,
                                       int maxiter, int nev, unsigned seed, double *eval_host, double *evec_host,
                                       int *iters, int verbose)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && B && eval_host && nev > 0 && A->ctx == B->ctx, EIG_ERR_ARG, "eig_generalized_inverse: bad argument");
    check_inverse_matrix(A, "GeneralizedInverse");
    check_inverse_matrix(B, "GeneralizedInverse");
    EIG_CHECK(A->nb_rows == B->nb_rows, EIG_ERR_SHAPE, "GeneralizedInverse: A and B sizes differ");
    eig_ctx_t ctx = A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const i64 n = A->nb_rows;
    // copy of A, shifted (:208, :240-252): A + shift B (pattern(B) within pattern(A)) + reg I
    std::vector<i64> rp, brp;
    std::vector<i32> c, bc;
    std::vector<double> v, bv;
    EIG_HIP(hipStreamSynchronize(s));
    mat_download_bcsr(*A, rp, c, v);
    mat_download_bcsr(*B, brp, bc, bv);
    for (i64 i = 0; i < n; ++i)
    {
      if (shift != 0.0)
        for (i64 q = brp[i]; q < brp[i + 1]; ++q)
        {
          const i32 *b0 = c.data() + rp[i], *b1 = c.data() + rp[i + 1];
          const i32 *hit = std::lower_bound(b0, b1, bc[q]);
          EIG_CHECK(hit != b1 && *hit == bc[q], EIG_ERR_SHAPE, "GeneralizedInverse: pattern(B) must be contained in pattern(A)");
          v[hit - c.data()] += shift * bv[q];
        }
      if (reg != 0.0)
      {
        const i32 *b0 = c.data() + rp[i], *b1 = c.data() + rp[i + 1];
        const i32 *hit = std::lower_bound(b0, b1, (i32)i);
        EIG_CHECK(hit != b1 && *hit == (i32)i, EIG_ERR_SHAPE, "GeneralizedInverse: A has no diagonal entry");
        v[hit - c.data()] += reg;
      }
    }
    eig_mat_t As = nullptr;
    {
      const int rc = eig_mat_create_bcsr(ctx, n, n, 1, 1, rp.data(), c.data(), v.data(), &As);
      EIG_CHECK(rc == EIG_OK, rc, std::string("shifted copy of A: ") + eig_last_error(ctx));
    }
    struct MatGuard {
      eig_mat_t m;
      ~MatGuard() { eig_mat_destroy(m); }
    } asg{As};
    LuRef F;  // :255
    if (lu)
      F.lu = lu;
    else
      factor_host(*As, rp, c, v, F);
    EIG_CHECK(lu_size(F.lu) == n, EIG_ERR_SHAPE,
              "matmul_inverse_tallskinny_blocked: Factorization does not match size of Qout/Qin");
    const i64 m = (nev / 8 + std::min(nev % 8, 1)) * 8;  // :224
    // basis ping-pong Bk[0] / Bk[1] and a scratch block Z (B Q1, then the As product): iteration i
    // reads Bk[(i - 1) % 2] and leaves its basis in Bk[i % 2], so iteration i + 1 is queued before the
    // host's relative-error test of iteration i without touching that basis (as eig_standard_largest)
    DevBuf Q1b(n * m * 8), Q2b(n * m * 8), Zb(n * m * 8), dpb(2 * m * 8 + 8);
    double *Bk[2] = {Q1b.d(), Q2b.d()}, *Z = Zb.d(), *norm = dpb.d() + 2 * m;
    PinnedDoubles hd(2 * (size_t)m);
    SyncEvent ev[2];
    random_block(ctx, n, m, seed, Bk[0]);
    std::vector<double> ra1(m, 0.0), ra2(m, 0.0);
    b_orthonormalize_device(*B, m, Bk[0], norm);                 // :273
    launch_spmm_dot_mv8(*As, m, Bk[0], Z, dpb.d(), s, ctx->red);  // :274-275
    EIG_HIP(hipMemcpyAsync(hd.p, dpb.d(), m * 8, hipMemcpyDeviceToHost, s));
    EIG_HIP(hipStreamSynchronize(s));
    for (i64 i = 0; i < m; ++i) ra2[i] = hd.p[i] - shift;
    auto enqueue = [&](int i) {
      double *Q = Bk[i % 2], *dp = hd.dev + (i & 1) * m;
      launch_spmm_mv8(*B, m, Bk[(i + 1) % 2], Z, s);        // :302 Q2 = B Q1
      lu_inverse_device(F.lu, m, Z, Q, s);                   // :303 Q1 = A^-1 Q2
      b_orthonormalize_device(*B, m, Q, norm);               // :304
      launch_spmm_dot_mv8(*As, m, Q, Z, dp, s, ctx->red);     // :317 and the dots, straight to the host
      EIG_HIP(hipEventRecord(ev[i & 1].e, s));
    };
    int iter = 0, basis = 0;
    double relerror = 0.0;
    if (maxiter > 0) enqueue(1);
    while (iter < maxiter)
    {
      iter += 1;
      if (iter + 1 <= maxiter) enqueue(iter + 1);  // look-ahead: queued before this iteration's test
      EIG_HIP(hipEventSynchronize(ev[iter & 1].e));
      for (i64 i = 0; i < m; ++i) ra1[i] = hd.p[(iter & 1) * m + i] - shift;
      basis = iter % 2;
      relerror = 0.0;
      for (i64 i = 0; i < m; ++i) relerror = std::max(relerror, std::fabs(ra1[i] - ra2[i]));
      relerror /= *std::max_element(ra1.begin(), ra1.end());
      if (verbose > 2) fprintf(stdout, "iter=%d relerror=%.17g\n", iter, relerror);
      std::swap(ra1, ra2);
      if ((iter > 10) & (relerror < tol)) break;  // :325
    }
    for (int j = 0; j < nev; ++j) eval_host[j] = ra2[j];
    copy_evecs(ctx, Bk[basis], n, nev, evec_host);  // (stream order: after any queued iteration)
    EIG_HIP(hipStreamSynchronize(s));
    if (iters) *iters = iter;
    if (verbose > 0) fprintf(stdout, "GeneralizedInverse: iterations=%d relerror=%.17g\n", iter, relerror);
  });
}

// ============================================================================================
// computeGenSymShiftInvertMinMagnitude (arpack_geneo_wrapper.hh:581-658): thick-restart Lanczos
// in the B-inner product on OP = (A - sigma B)^-1 B, "LM" 
// ============================================================================================
namespace {

// Host copy of A - sigma B on A's pattern (pattern(B) within pattern(A); ashiftb.axpy(-sigma, b_),
// arpack_geneo_wrapper.hh:599-600).
void shifted_copy(eig_mat_s &A, eig_mat_s *B, double sigma, std::vector<i64> &rp, std::vector<i32> &c,
                  std::vector<double> &v)
{
  mat_download_bcsr(A, rp, c, v);
  if (sigma == 0.0) return;
  const i64 n = A.nb_rows;
  if (!B)
  {
    for (i64 i = 0; i < n; ++i)
    {
      const i32 *b0 = c.data() + rp[i], *b1 = c.data() + rp[i + 1];
      const i32 *hit = std::lower_bound(b0, b1, (i32)i);
      EIG_CHECK(hit != b1 && *hit == (i32)i, EIG_ERR_SHAPE, "shift-invert: A has no diagonal entry");
      v[hit - c.data()] -= sigma;
    }
    return;
  }
  std::vector<i64> brp;
  std::vector<i32> bc;
  std::vector<double> bv;
  mat_download_bcsr(*B, brp, bc, bv);
  for (i64 i = 0; i < n; ++i)
    for (i64 q = brp[i]; q < brp[i + 1]; ++q)
    {
      const i32 *b0 = c.data() + rp[i], *b1 = c.data() + rp[i + 1];
      const i32 *hit = std::lower_bound(b0, b1, bc[q]);
      EIG_CHECK(hit != b1 && *hit == bc[q], EIG_ERR_SHAPE, "shift-invert: pattern(B) must be contained in pattern(A)");
      v[hit - c.data()] -= sigma * bv[q];
    }
}

}  // namespace

namespace {

void shift_invert_check(eig_mat_t A, eig_mat_t B)
{
  check_inverse_matrix(A, "computeGenSymShiftInvertMinMagnitude");
  if (B)
  {
    check_inverse_matrix(B, "computeGenSymShiftInvertMinMagnitude");
    EIG_CHECK(B->ctx == A->ctx && B->nb_rows == A->nb_rows, EIG_ERR_SHAPE, "shift-invert: A and B sizes differ");
  }
}

// The factorisation of A - sigma B (arpack_geneo_wrapper.hh:597-601): the caller's, or a host one.
void shift_invert_factor(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double sigma, LuRef &F)
{
  if (lu)
    F.lu = lu;
  else
  {
    std::vector<i64> rp;
    std::vector<i32> c;
    std::vector<double> v;
    EIG_HIP(hipStreamSynchronize(A->ctx->stream));
    shifted_copy(*A, B, sigma, rp, c, v);
    factor_host(*A, rp, c, v, F);
  }
  EIG_CHECK(lu_size(F.lu) == A->nb_rows, EIG_ERR_SHAPE, "shift-invert: factorisation size differs from A");
}

// One computeGenSymShiftInvertMinMagnitude solve (ARSymGenEig 'S' mode, "LM") with the factors F.
void shift_invert_core(eig_mat_t A, eig_mat_t B, const LuRef &F, double sigma, int nev, int ncv, double tol, int maxit,
                       unsigned seed, double *eval_host, double *evec_host, int *restarts)
{
    eig_ctx_t ctx = A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const i64 n = A->nb_rows;
    if (ncv <= 0) ncv = (int)std::min<i64>(n, std::max(2 * nev + 1, 20));  // ARPACK++ ncv = 0 (auto)
    EIG_CHECK(nev < ncv && ncv <= n && ncv <= 500, EIG_ERR_ARG, "shift-invert: need nev < ncv <= min(n, 500)");
    if (tol <= 0.0) tol = 2.220446049250313e-16;  // tol = 0: machine precision (ARPACK)
    if (maxit <= 0) maxit = 100 * nev;            // maxit = 0: 100 nev (ARPACK++)
    const int m = ncv;
    // basis V and BV (= B V; V itself when B is NULL), column-major, m + 1 vectors each
    DevBuf Vb((size_t)(m + 1) * n * 8), BVb(B ? (size_t)(m + 1) * n * 8 : 8), Wb(n * 8), BWb(n * 8), X8b(n * 64),
        Y8b(n * 64), Tb((size_t)2 * (m + 1) * n * 8), cb((size_t)(m + 8) * 8 * 2);
    double *V = Vb.d(), *BV = B ? BVb.d() : Vb.d(), *W = Wb.d(), *BW = BWb.d(), *X8 = X8b.d(), *Y8 = Y8b.d();
    double *cd = cb.d(), *sc = cd + m + 8;
    EIG_HIP(hipMemsetAsync(X8, 0, n * 64, s));
    auto bmul = [&](double *x, double *y) {  // y = B x
      if (B) launch_spmv(*B, x, y, nullptr, 0, B->nslices, s);
      else if (y != x) EIG_HIP(hipMemcpyAsync(y, x, n * 8, hipMemcpyDeviceToDevice, s));
    };
    auto dot = [&](const double *x, const double *y) {
      launch_dot(n, x, y, sc, 0, s, ctx->red);
      double h = 0.0;
      EIG_HIP(hipMemcpyAsync(&h, sc, 8, hipMemcpyDeviceToHost, s));
      EIG_HIP(hipStreamSynchronize(s));
      return h;
    };
    auto op = [&](const double *bx, double *y) {  // y = (A - sigma B)^-1 bx (column 0 of the 8-wide solve)
      EIG_HIP(hipMemcpy2DAsync(X8, 64, bx, 8, 8, n, hipMemcpyDeviceToDevice, s));
      lu_inverse_device(F.lu, 8, X8, Y8, s);
      EIG_HIP(hipMemcpy2DAsync(y, 8, Y8, 64, 8, n, hipMemcpyDeviceToDevice, s));
    };
    // start vector: mt19937(seed) normal numbers put into the range of OP (as ARPACK's dgetv0 does
    // for the generalised modes, so a singular B cannot leave null(B) components in the basis),
    // B-normalised
    {
      std::vector<double> h(n);
      host_random_normal(n, seed, h.data());
      EIG_HIP(hipMemcpyAsync(W, h.data(), n * 8, hipMemcpyHostToDevice, s));
      bmul(W, BW);
      op(BW, V);
      bmul(V, BV);
      const double nb = std::sqrt(dot(V, BV));
      launch_scal(n, 1.0 / nb, V, s);
      if (B) launch_scal(n, 1.0 / nb, BV, s);
    }
    std::vector<double> T((size_t)m * m, 0.0), ctot(m + 1), th, Y;
    // per step j of an extension: the two CGS passes' coefficients (m + 1 each) and (w, B w), kept on
    // the device and read back once per extension -- the steps queue without a host round trip (the
    // host sums and scalars are those the step-by-step loop computed; a breakdown is reported after
    // the extension, with the same error)
    const i64 cstride = 2 * (i64)(m + 1) + 1;
    DevBuf coefb((size_t)m * cstride * 8);
    double *coef = coefb.d();
    std::vector<double> coefh((size_t)m * cstride);
    int k = 0, nrestart = 0;
    double betam = 0.0;
    std::vector<int> want;
    bool done = false;
    while (!done)
    {
      // extend the Lanczos factorisation from k to m vectors
      for (int j = k; j < m; ++j)
      {
        double *bvj = BV + (i64)j * n;
        double *cj = coef + (i64)j * cstride;
        // w = (A - sigma B)^-1 (B v_j): the reverse-communication product of ARSymGenEig 'S' mode
        op(bvj, W);
        for (int pass = 0; pass < 2; ++pass)  // DGKS / CGS2 against v_0 .. v_j in the B-inner product
        {
          launch_gemv_t(n, j + 1, BV, n, W, cj + pass * (m + 1), 0, s, ctx->red);
          launch_gemv_n_sub(n, j + 1, V, n, cj + pass * (m + 1), nullptr, W, s);
        }
        bmul(W, BW);
        launch_dot(n, W, BW, cj + 2 * (m + 1), 0, s, ctx->red);  // beta_j^2
        double *vn = V + (i64)(j + 1) * n, *bvn = BV + (i64)(j + 1) * n;
        EIG_HIP(hipMemcpyAsync(vn, W, n * 8, hipMemcpyDeviceToDevice, s));
        launch_scal_dev(n, cj + 2 * (m + 1), true, vn, s);  // 1 / sqrt(beta_j^2)
        if (B)
        {
          EIG_HIP(hipMemcpyAsync(bvn, BW, n * 8, hipMemcpyDeviceToDevice, s));
          launch_scal_dev(n, cj + 2 * (m + 1), true, bvn, s);
        }
      }
      EIG_HIP(hipMemcpyAsync(coefh.data() + (size_t)k * cstride, coef + (i64)k * cstride,
                             (size_t)(m - k) * cstride * 8, hipMemcpyDeviceToHost, s));
      EIG_HIP(hipStreamSynchronize(s));
      for (int j = k; j < m; ++j)
      {
        const double *ch = coefh.data() + (size_t)j * cstride;
        std::fill(ctot.begin(), ctot.end(), 0.0);
        for (int pass = 0; pass < 2; ++pass)
          for (int i = 0; i <= j; ++i) ctot[i] += ch[pass * (m + 1) + i];
        for (int i = 0; i <= j; ++i) T[(size_t)i * m + j] = T[(size_t)j * m + i] = ctot[i];
        const double beta = std::sqrt(std::max(0.0, ch[2 * (m + 1)]));
        double tn = 0.0;
        for (int i = 0; i <= j; ++i) tn = std::max(tn, std::fabs(ctot[i]));
        EIG_CHECK(beta > 1e-14 * tn, EIG_ERR_BREAKDOWN,
                  "shift-invert Lanczos: invariant subspace reached (choose ncv < n or another seed)");
        if (j + 1 < m) T[(size_t)(j + 1) * m + j] = T[(size_t)j * m + (j + 1)] = beta;
        betam = beta;
      }
      sym_eig(m, T, th, Y);
      // "LM" on OP: the nev Ritz values of largest magnitude (eigenvalues of the pencil nearest sigma)
      std::vector<int> ord(m);
      std::iota(ord.begin(), ord.end(), 0);
      std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return std::fabs(th[a]) > std::fabs(th[b]); });
      want.assign(ord.begin(), ord.begin() + nev);
      bool conv = true;
      for (int i : want)
        if (std::fabs(betam * Y[(size_t)(m - 1) * m + i]) > tol * std::fabs(th[i])) conv = false;
      if (conv || nrestart >= maxit)
      {
        done = true;
        break;
      }
      // thick restart: keep kk Ritz vectors of largest |theta|, then the residual vector
      const int kk = std::min(m - 2, nev + (m - nev) / 2);
      std::vector<double> coef(m);
      double *Tmp = Tb.d();
      for (int q = 0; q < kk; ++q)
      {
        for (int i = 0; i < m; ++i) coef[i] = Y[(size_t)i * m + ord[q]];
        EIG_HIP(hipMemcpyAsync(cd, coef.data(), m * 8, hipMemcpyHostToDevice, s));
        launch_gemv_n_set(n, m, V, n, cd, nullptr, Tmp + (i64)q * n, s);
        if (B) launch_gemv_n_set(n, m, BV, n, cd, nullptr, Tmp + (i64)(kk + q) * n, s);
        EIG_HIP(hipStreamSynchronize(s));
      }
      EIG_HIP(hipMemcpyAsync(V, Tmp, (size_t)kk * n * 8, hipMemcpyDeviceToDevice, s));
      EIG_HIP(hipMemcpyAsync(V + (i64)kk * n, V + (i64)m * n, n * 8, hipMemcpyDeviceToDevice, s));
      if (B)
      {
        EIG_HIP(hipMemcpyAsync(BV, Tmp + (i64)kk * n, (size_t)kk * n * 8, hipMemcpyDeviceToDevice, s));
        EIG_HIP(hipMemcpyAsync(BV + (i64)kk * n, BV + (i64)m * n, n * 8, hipMemcpyDeviceToDevice, s));
      }
      std::fill(T.begin(), T.end(), 0.0);
      for (int q = 0; q < kk; ++q) T[(size_t)q * m + q] = th[ord[q]];
      k = kk;
      ++nrestart;
    }
    // eigenpairs of the pencil: lambda = sigma + 1 / theta, sorted ascending (:636-648)
    std::vector<int> idx(nev);
    std::iota(idx.begin(), idx.end(), 0);
    std::vector<double> lam(nev);
    for (int i = 0; i < nev; ++i) lam[i] = sigma + 1.0 / th[want[i]];
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return lam[a] < lam[b]; });
    for (int i = 0; i < nev; ++i) eval_host[i] = lam[idx[i]];
    if (evec_host)
    {
      // purified Ritz vectors (ARPACK dseupd for the spectral-transformation modes): x = OP(V y) /
      // theta = V y + (beta_m y_m / theta) v_m.  B = I: that linear combination.  Generalised: the
      // operator applied explicitly to B V y = BV y, x = (A - sigma B)^-1 (BV y) / theta, then
      // B-normalised -- with a singular B (the harness's partition-of-unity B) the basis picks up
      // null(B) components through the projections that the B-inner products never see and that
      // grow over thick restarts; OP maps into range(OP), where they cannot live.
      std::vector<double> coef(m + 1);
      for (int q = 0; q < nev; ++q)
      {
        const int col = want[idx[q]];
        for (int i = 0; i < m; ++i) coef[i] = Y[(size_t)i * m + col];
        coef[m] = betam * Y[(size_t)(m - 1) * m + col] / th[col];
        EIG_HIP(hipMemcpyAsync(cd, coef.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
        if (!B)
          launch_gemv_n_set(n, m + 1, V, n, cd, nullptr, W, s);
        else
        {
          launch_gemv_n_set(n, m, BV, n, cd, nullptr, BW, s);
          op(BW, W);
          bmul(W, BW);
          const double xb = dot(W, BW);
          EIG_CHECK(xb > 0.0, EIG_ERR_BREAKDOWN, "shift-invert: purified Ritz vector has no B-norm");
          launch_scal(n, 1.0 / std::sqrt(xb), W, s);
        }
        EIG_HIP(hipMemcpyAsync(evec_host + (i64)q * n, W, n * 8, hipMemcpyDeviceToHost, s));
        EIG_HIP(hipStreamSynchronize(s));
      }
    }
    if (restarts) *restarts = nrestart;
}

// Block variant (EIG_SI_BLOCK, the default where the basis fits): the same OP, the same wanted
// pairs and the same B-inner product, by block Lanczos with Krylov-Schur (thick) restarts on p
// columns at once.  Why: one application of OP is the block-inverse triangular solve, a chain over
// the factor's 64-row blocks that one workgroup walks per 8 columns -- latency-bound, so p = 16
// columns cost what one column costs (two chains side by side), and a block Krylov space reaches
// the wanted pairs in a fraction of the applications the one-vector recurrence needs (nev = 8 on
// the 200^2 GenEO pencil: 44 applications -> 8).  Basis V (c columns, MultiVector<double,8>
// blocks) and BV = B V; per block step, with V_a the last p columns:
//     W = OP(B V_a);  H = (B V)^T W, W -= V H  (twice: CGS2 in the B-inner product);
//     W = F R (CholQR2 in the B-inner product);  T(:, a) = H, T(next, a) = R.
// Rayleigh-Ritz on T; the residual of Ritz pair i is ||R y_i(a)|| (V_next is B-orthonormal), so the
// convergence test is ||R y_i(a)|| <= tol |theta_i|.  Restart: U = V Y(:, kept) (kk Ritz vectors of
// largest |theta|), T = diag(theta_kept) coupled to F by C = R Y(a, kept) -- again a block Krylov
// decomposition OP [U F] = [U F] T + ..., extended from F.  Eigenvectors purified like the one-vector
// path: x = OP(B V y) / theta, B-normalised (one block solve for all of them).
struct SiBlockShape {
  int nw, p, kk, cmax;
};

SiBlockShape si_block_shape(int nev, int ncv)
{
  SiBlockShape g;
  g.nw = (nev + 7) / 8 * 8;
  g.p = std::max(16, g.nw);
  g.kk = std::max((nev + (nev + 1) / 2 + 7) / 8 * 8, 3 * g.p);
  g.cmax = std::max(g.kk + 3 * g.p, (ncv + 7) / 8 * 8);
  return g;
}

// the block method's reductions within the context's tickets: the projection Gram (cmax x p, partials
// in a buffer sized for the launch), the CholQR Gram (p x p) and the purified vectors' B-norms
// (the projection Gram goes in row slices of 64 when it is larger: see gram_rows)
bool si_block_fits(const SiBlockShape &g)
{
  return gram_mv8_chunks(64, g.p) <= kNumTickets && gram_mv8_chunks(g.p, g.p) <= kNumTickets &&
         g.nw / 8 <= kNumTickets;
}

// H (c x p, row i at H + i p) = Q1(:, 0 .. c)^T Q2: one launch where its output chunks fit the
// tickets, else row slices (each a multiple of 64 rows) in stream order
void gram_rows(eig_ctx_t ctx, i64 n, int c, int p, const double *Q1, const double *Q2, double *H, hipStream_t s)
{
  int rc = c;
  while (gram_mv8_chunks(rc, p) > kNumTickets) rc = std::max(64, (rc / 2 + 63) / 64 * 64);
  for (int r0 = 0; r0 < c; r0 += rc)
    launch_gram_panel(ctx, n, n, std::min(rc, c - r0), p, Q1 + (i64)r0 * n, Q2, H + (size_t)r0 * p, s);
}

void shift_invert_block_core(eig_mat_t A, eig_mat_t B, const LuRef &F, double sigma, int nev, int ncv, double tol,
                             int maxit, unsigned seed, double *eval_host, double *evec_host, int *restarts)
{
  eig_ctx_t ctx = A->ctx;
  EIG_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const i64 n = A->nb_rows;
  const SiBlockShape g = si_block_shape(nev, ncv);
  const int p = g.p, kk = g.kk, cmax = g.cmax, cap = cmax + p;
  EIG_CHECK(nev < n && cap <= n, EIG_ERR_ARG, "shift-invert (block): the block basis does not fit n");
  EIG_CHECK(si_block_fits(g), EIG_ERR_ARG, "shift-invert (block): nev too large for the block method (use EIG_SI_SINGLE)");
  if (tol <= 0.0) tol = 2.220446049250313e-16;
  if (maxit <= 0) maxit = 100 * nev;
  const int wk = std::max(kk, g.nw);
  DevBuf Vb((size_t)cap * n * 8), BVb(B ? (size_t)cap * n * 8 : 8), W1b((size_t)p * n * 8), W2b((size_t)p * n * 8),
      BWb((size_t)p * n * 8), Ub((size_t)wk * n * 8), Hb((size_t)cap * std::max(p, wk) * 8);
  double *V = Vb.d(), *BV = B ? BVb.d() : V, *W = W1b.d(), *Wt = W2b.d(), *BW = BWb.d(), *U = Ub.d(), *dH = Hb.d();
  auto bmul = [&](const double *x, double *y, int cols) {  // y = B x (cols columns)
    if (B) launch_spmm_mv8(*B, cols, x, y, s);
    else if (y != x) EIG_HIP(hipMemcpyAsync(y, x, (size_t)cols * n * 8, hipMemcpyDeviceToDevice, s));
  };
  // y (q columns) = x (px columns) M, M px x q row-major on the host
  std::vector<double> mneg;
  auto mul_small = [&](const double *x, int px, const std::vector<double> &M, int q, double *y) {
    mneg.resize((size_t)px * q);
    for (size_t k = 0; k < mneg.size(); ++k) mneg[k] = -M[k];
    EIG_HIP(hipMemcpyAsync(dH, mneg.data(), mneg.size() * 8, hipMemcpyHostToDevice, s));
    EIG_HIP(hipMemsetAsync(y, 0, (size_t)q * n * 8, s));
    for (int i = 0; i < px / 8; ++i) launch_project(n, q, x + (i64)i * 8 * n, y, dH + (size_t)i * 8 * q, s);
    EIG_HIP(hipStreamSynchronize(s));  // (mneg is reused by the next call)
  };
  // OP on p columns: y = (A - sigma B)^-1 bx (bx is consumed as the solve's scratch)
  auto op = [&](double *bx, double *y, int cols) { lu_inverse_device(F.lu, cols, bx, y, s); };
  // W (p columns, scratch Wt) -> B-orthonormal F at dst / bdst with W = F R; false on a rank loss
  std::vector<double> G((size_t)p * p), R((size_t)p * p), Ri((size_t)p * p), Rtot((size_t)p * p);
  auto bortho = [&](double *dst, double *bdst) -> bool {
    std::fill(Rtot.begin(), Rtot.end(), 0.0);
    for (int i = 0; i < p; ++i) Rtot[(size_t)i * p + i] = 1.0;
    for (int pass = 0; pass < 2; ++pass)
    {
      double *bw = B ? BW : W;
      bmul(W, bw, p);
      launch_gram_panel(ctx, n, n, p, p, W, bw, dH, s);
      EIG_HIP(hipMemcpyAsync(G.data(), dH, G.size() * 8, hipMemcpyDeviceToHost, s));
      EIG_HIP(hipStreamSynchronize(s));
      for (int i = 0; i < p; ++i)
        for (int j = i + 1; j < p; ++j) G[(size_t)j * p + i] = G[(size_t)i * p + j];
      if (!chol_upper(p, G.data(), R.data())) return false;
      tri_upper_inv(p, R.data(), Ri.data());
      mul_small(W, p, Ri, p, Wt);
      std::swap(W, Wt);
      std::vector<double> Rn((size_t)p * p, 0.0);  // Rtot = R Rtot
      for (int i = 0; i < p; ++i)
        for (int k = i; k < p; ++k)
          for (int j = k; j < p; ++j) Rn[(size_t)i * p + j] += R[(size_t)i * p + k] * Rtot[(size_t)k * p + j];
      Rtot.swap(Rn);
    }
    EIG_HIP(hipMemcpyAsync(dst, W, (size_t)p * n * 8, hipMemcpyDeviceToDevice, s));
    bmul(dst, bdst, p);
    return true;
  };
  // start block: normal numbers put into the range of OP (dgetv0 for the generalised modes), then
  // B-orthonormalised
  {
    launch_fill_normal((i64)p * n, seed, Wt, s);
    bmul(Wt, BW, p);
    op(BW, W, p);
    EIG_CHECK(bortho(V, BV), EIG_ERR_BREAKDOWN, "shift-invert (block): start block is rank deficient");
  }
  std::vector<double> T((size_t)cap * cap, 0.0), th, Y, Hh, Ht, Tc;
  int c = p, nrestart = 0;
  std::vector<int> ord;
  for (;;)
  {
    // apply OP to the active block V(:, a .. c), project, B-orthonormalise: F = V(:, c .. c + p)
    const int a = c - p;
    EIG_HIP(hipMemcpyAsync(BW, BV + (i64)a * n, (size_t)p * n * 8, hipMemcpyDeviceToDevice, s));
    op(BW, W, p);
    Ht.assign((size_t)c * p, 0.0);
    for (int pass = 0; pass < 2; ++pass)  // CGS2 against V(:, 0 .. c) in the B-inner product
    {
      gram_rows(ctx, n, c, p, BV, W, dH, s);
      for (int i = 0; i < c / 8; ++i) launch_project(n, p, V + (i64)i * 8 * n, W, dH + (size_t)i * 8 * p, s);
      Hh.resize((size_t)c * p);
      EIG_HIP(hipMemcpyAsync(Hh.data(), dH, Hh.size() * 8, hipMemcpyDeviceToHost, s));
      EIG_HIP(hipStreamSynchronize(s));
      for (size_t k = 0; k < Hh.size(); ++k) Ht[k] += Hh[k];
    }
    for (int i = 0; i < c; ++i)
      for (int j = 0; j < p; ++j) T[(size_t)i * cap + a + j] = T[(size_t)(a + j) * cap + i] = Ht[(size_t)i * p + j];
    EIG_CHECK(bortho(V + (i64)c * n, BV + (i64)c * n), EIG_ERR_BREAKDOWN,
              "shift-invert (block): invariant subspace reached (choose another seed or the one-vector solver)");
    // Rayleigh-Ritz on the c columns: at the end of the first cycle, then after every application
    // (stop as soon as the wanted pairs converged).  Inside the first cycle the wanted pairs have not
    // converged in any run seen, and the host eigen-solve of T costs O(c^3) (~1-2 ms at c = 64-96).
    if (nrestart == 0 && c + p <= cmax)
    {
      for (int i = 0; i < p; ++i)
        for (int j = 0; j < p; ++j)
          T[(size_t)(c + i) * cap + a + j] = T[(size_t)(a + j) * cap + c + i] = Rtot[(size_t)i * p + j];
      c += p;
      continue;
    }
    Tc.resize((size_t)c * c);
    for (int i = 0; i < c; ++i)
      for (int j = 0; j < c; ++j) Tc[(size_t)i * c + j] = T[(size_t)i * cap + j];
    sym_eig(c, Tc, th, Y);  // Y[i * c + j]: component i of Ritz vector j
    // "LM" on OP: the Ritz values of largest magnitude (eigenvalues of the pencil nearest sigma)
    ord.resize(c);
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return std::fabs(th[x]) > std::fabs(th[y]); });
    // coupling of the Ritz vectors to F: C(:, j) = R y_j(a .. a + p)
    auto coupling = [&](int j, int i) {
      double v = 0.0;
      for (int k = i; k < p; ++k) v += Rtot[(size_t)i * p + k] * Y[(size_t)(a + k) * c + j];
      return v;
    };
    bool conv = c >= std::min(nev + 1, cmax);
    for (int q = 0; q < nev && conv; ++q)
    {
      double r2 = 0.0;
      for (int i = 0; i < p; ++i)
      {
        const double v = coupling(ord[q], i);
        r2 += v * v;
      }
      if (std::sqrt(r2) > tol * std::fabs(th[ord[q]])) conv = false;
    }
    if (conv) break;
    if (c + p <= cmax)
    {
      // F joins the basis: T(c .. c + p, a .. c) = R
      for (int i = 0; i < p; ++i)
        for (int j = 0; j < p; ++j)
          T[(size_t)(c + i) * cap + a + j] = T[(size_t)(a + j) * cap + c + i] = Rtot[(size_t)i * p + j];
      c += p;
      continue;
    }
    if (nrestart >= maxit) break;
    // thick restart: U = V Y(:, kept), F moves behind it, T = diag(theta_kept) + the coupling C
    {
      std::vector<double> Ysel((size_t)c * kk);
      for (int r = 0; r < c; ++r)
        for (int q = 0; q < kk; ++q) Ysel[(size_t)r * kk + q] = Y[(size_t)r * c + ord[q]];
      mul_small(V, c, Ysel, kk, U);
      EIG_HIP(hipMemcpyAsync(V, U, (size_t)kk * n * 8, hipMemcpyDeviceToDevice, s));
      EIG_HIP(hipMemcpyAsync(V + (i64)kk * n, V + (i64)c * n, (size_t)p * n * 8, hipMemcpyDeviceToDevice, s));
      if (B)
      {
        EIG_HIP(hipMemcpyAsync(BV + (i64)kk * n, BV + (i64)c * n, (size_t)p * n * 8, hipMemcpyDeviceToDevice, s));
        bmul(V, BV, kk);
      }
      std::fill(T.begin(), T.end(), 0.0);
      for (int q = 0; q < kk; ++q)
      {
        T[(size_t)q * cap + q] = th[ord[q]];
        for (int i = 0; i < p; ++i) T[(size_t)(kk + i) * cap + q] = T[(size_t)q * cap + kk + i] = coupling(ord[q], i);
      }
      c = kk + p;
      ++nrestart;
    }
  }
  // eigenpairs of the pencil: lambda = sigma + 1 / theta, ascending (:636-648)
  std::vector<int> idx(nev);
  std::iota(idx.begin(), idx.end(), 0);
  std::vector<double> lam(nev);
  for (int q = 0; q < nev; ++q) lam[q] = sigma + 1.0 / th[ord[q]];
  std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return lam[x] < lam[y]; });
  for (int q = 0; q < nev; ++q) eval_host[q] = lam[idx[q]];
  if (evec_host)
  {
    const int nw = g.nw;
    std::vector<double> Ysel((size_t)c * nw, 0.0);
    for (int q = 0; q < nev; ++q)
    {
      const int j = ord[idx[q]];
      for (int r = 0; r < c; ++r) Ysel[(size_t)r * nw + q] = Y[(size_t)r * c + j] / th[j];
    }
    mul_small(BV, c, Ysel, nw, U);  // B V y / theta
    op(U, W, nw);                   // x = OP(B V y) / theta
    double *bw = B ? BW : W;
    bmul(W, bw, nw);
    launch_dot_diag_mv8(n, nw, W, bw, dH, 0, s, ctx->red);
    std::vector<double> xb(nw), h((size_t)nw * n);
    EIG_HIP(hipMemcpyAsync(xb.data(), dH, nw * 8, hipMemcpyDeviceToHost, s));
    EIG_HIP(hipMemcpyAsync(h.data(), W, h.size() * 8, hipMemcpyDeviceToHost, s));
    EIG_HIP(hipStreamSynchronize(s));
    for (int q = 0; q < nev; ++q)
    {
      EIG_CHECK(xb[q] > 0.0, EIG_ERR_BREAKDOWN, "shift-invert: purified Ritz vector has no B-norm");
      const double sc = 1.0 / std::sqrt(xb[q]);
      for (i64 i = 0; i < n; ++i) evec_host[(i64)q * n + i] = sc * h[((i64)(q / 8) * n + i) * 8 + q % 8];
    }
  }
  if (restarts) *restarts = nrestart;
}

// EIG_SI_AUTO: the block solver where its basis (cmax + p columns) is at most a quarter of n
bool si_use_block(i64 n, int nev, int ncv, int flags)
{
  if (flags & EIG_SI_SINGLE) return false;
  if (flags & EIG_SI_BLOCK) return true;
  const SiBlockShape g = si_block_shape(nev, ncv);
  // the basis within n / 4, and the reductions within the tickets
  return (i64)(g.cmax + g.p) * 4 <= n && si_block_fits(g);
}

void shift_invert_run(eig_mat_t A, eig_mat_t B, const LuRef &F, double sigma, int nev, int ncv, double tol, int maxit,
                      unsigned seed, double *eval_host, double *evec_host, int *restarts, int flags)
{
  if (si_use_block(A->nb_rows, nev, ncv, flags))
    shift_invert_block_core(A, B, F, sigma, nev, ncv, tol, maxit, seed, eval_host, evec_host, restarts);
  else
    shift_invert_core(A, B, F, sigma, nev, ncv, tol, maxit, seed, eval_host, evec_host, restarts);
}

}  // namespace

extern "C" int eig_shift_invert_solve_ex(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double sigma, int nev, int ncv,
                                         double tol, int maxit, unsigned seed, double *eval_host, double *evec_host,
                                         int *restarts, int flags)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && eval_host && nev > 0, EIG_ERR_ARG, "eig_shift_invert_solve: bad argument");
    EIG_CHECK((flags & ~(EIG_SI_SINGLE | EIG_SI_BLOCK)) == 0 && flags != (EIG_SI_SINGLE | EIG_SI_BLOCK), EIG_ERR_ARG,
              "eig_shift_invert_solve_ex: unknown flags");
    shift_invert_check(A, B);
    EIG_HIP(hipSetDevice(A->ctx->device));
    LuRef F;
    shift_invert_factor(A, B, lu, sigma, F);
    shift_invert_run(A, B, F, sigma, nev, ncv, tol, maxit, seed, eval_host, evec_host, restarts, flags);
  });
}

extern "C" int eig_shift_invert_solve(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double sigma, int nev, int ncv,
                                      double tol, int maxit, unsigned seed, double *eval_host, double *evec_host,
                                      int *restarts)
{
  return eig_shift_invert_solve_ex(A, B, lu, sigma, nev, ncv, tol, maxit, seed, eval_host, evec_host, restarts,
                                   EIG_SI_AUTO);
}

// computeGenSymShiftInvertMinMagnitudeAdaptive (arpack_geneo_wrapper.hh:661-774): solve with nev =
// initial_nev; while the largest returned eigenvalue is below `threshold` and nev < max_nev, grow
// nev to min(max_nev, int(nev * 1.3)) (:770; the comment at :665 says 50 %, the code 1.3) and solve
// again from the same start (ARPACK++'s default initial guess each pass).  One factorisation of
// A - sigma B serves every pass.  ncv = 0 (auto) and maxit = nIterationsMax_ * nev as the reference.
extern "C" int eig_shift_invert_adaptive(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double sigma, double threshold,
                                         int initial_nev, int max_nev, double tol, int maxit_per_nev, unsigned seed,
                                         double *eval_host, double *evec_host, int *nev_out, int *passes)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && eval_host && nev_out && initial_nev > 0 && max_nev > 0, EIG_ERR_ARG,
              "eig_shift_invert_adaptive: bad argument");
    // (arpack_geneo_wrapper.hh:693-694: "initial_nev too large")
    EIG_CHECK(initial_nev <= max_nev, EIG_ERR_ARG, "eig_shift_invert_adaptive: initial_nev too large");
    shift_invert_check(A, B);
    EIG_HIP(hipSetDevice(A->ctx->device));
    LuRef F;
    shift_invert_factor(A, B, lu, sigma, F);
    int nev = initial_nev, pass = 0;
    for (;;)
    {
      const int maxit = maxit_per_nev > 0 ? maxit_per_nev * nev : 0;
      shift_invert_run(A, B, F, sigma, nev, 0, tol, maxit, seed, eval_host, evec_host, nullptr, EIG_SI_AUTO);
      ++pass;
      if (eval_host[nev - 1] >= threshold || nev >= max_nev) break;
      // (:770; for nev <= 3, int(nev * 1.3) == nev and the reference would solve the same problem
      // forever -- there nev grows by one instead; from nev = 4 on the sequences are identical)
      nev = std::min(max_nev, std::max(nev + 1, (int)(nev * 1.3)));
    }
    *nev_out = nev;
    if (passes) *passes = pass;
  });
}

// ============================================================================================
// Non-symmetric modes (arpack_geneo_wrapper.hh:428-578): computeStdNonSymMinMagnitude
// (ARNonSymStdEig on OP = (A - sigma B)^-1 B, "LM", lambda = sigma + 1 / Re(nu)) and
// computeGenNonSymShiftInvertMinMagnitude (ARNonSymGenEig, real shift-invert mode: the same OP in
// the B-inner product, lambda = sigma + 1 / nu).  ARPACK's dnaupd restarts implicitly with exact
// shifts; here the restart is Stewart's Krylov-Schur in its eigenvector-basis form: the projected
// matrix G of the Krylov decomposition  OP V = V G + f c^T  has its wanted eigenvectors (real and
// imaginary parts of complex pairs) orthonormalised into Z (m x kk); span(Z) is G-invariant, so
// OP (V Z) = (V Z)(Z^T G Z) + f (Z^T c)^T is again a Krylov decomposition, extended by Arnoldi
// steps (CGS2 in the chosen inner product) back to m vectors.  The same wanted Ritz values as
// ARPACK's restart filter (the polynomial with the unwanted Ritz values as roots annihilates the
// complement of span(Z)); convergence: ||f|| |c^T y| <= tol |nu| (dnaupd's Ritz estimate).
// ============================================================================================
namespace {

void arnoldi_core(eig_mat_t A, eig_mat_t B, const LuRef &F, double sigma, int nev, int ncv, double tol, int maxit,
                  unsigned seed, bool gen, double *eval_re, double *eval_im, double *evec_host, int *restarts)
{
  typedef std::complex<double> C;
  eig_ctx_t ctx = A->ctx;
  EIG_HIP(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const i64 n = A->nb_rows;
  if (ncv <= 0) ncv = (int)std::min<i64>(n, std::max(2 * nev + 1, 20));  // ARPACK++ ncv = 0 (auto)
  EIG_CHECK(nev + 2 <= ncv && ncv <= n && ncv <= 500, EIG_ERR_ARG, "Arnoldi: need nev + 2 <= ncv <= min(n, 500)");
  if (tol <= 0.0) tol = 2.220446049250313e-16;
  if (maxit <= 0) maxit = 100 * nev;
  const int m = ncv;
  const bool bip = gen && B;  // B-inner product
  DevBuf Vb((size_t)(m + 1) * n * 8), BVb(bip ? (size_t)(m + 1) * n * 8 : 8), Wb(n * 8), BWb(n * 8), X8b(n * 64),
      Y8b(n * 64), Tb((size_t)2 * (m + 1) * n * 8), cb((size_t)(m + 8) * 8 * 2);
  double *V = Vb.d(), *BV = bip ? BVb.d() : Vb.d(), *W = Wb.d(), *BW = BWb.d(), *X8 = X8b.d(), *Y8 = Y8b.d();
  double *cd = cb.d(), *sc = cd + m + 8;
  EIG_HIP(hipMemsetAsync(X8, 0, n * 64, s));
  auto bmul = [&](const double *x, double *y) {  // y = B x
    if (B) launch_spmv(*B, x, y, nullptr, 0, B->nslices, s);
    else if (y != x) EIG_HIP(hipMemcpyAsync(y, x, n * 8, hipMemcpyDeviceToDevice, s));
  };
  auto dot = [&](const double *x, const double *y) {
    launch_dot(n, x, y, sc, 0, s, ctx->red);
    double h = 0.0;
    EIG_HIP(hipMemcpyAsync(&h, sc, 8, hipMemcpyDeviceToHost, s));
    EIG_HIP(hipStreamSynchronize(s));
    return h;
  };
  auto solve = [&](const double *bx, double *y) {  // y = (A - sigma B)^-1 bx
    EIG_HIP(hipMemcpy2DAsync(X8, 64, bx, 8, 8, n, hipMemcpyDeviceToDevice, s));
    lu_inverse_device(F.lu, 8, X8, Y8, s);
    EIG_HIP(hipMemcpy2DAsync(y, 8, Y8, 64, 8, n, hipMemcpyDeviceToDevice, s));
  };
  auto norm_in = [&](double *x, double *bx) {  // ||x|| in the driver's inner product; bx = B x (bip)
    if (bip) bmul(x, bx);
    return std::sqrt(std::max(0.0, dot(x, bip ? bx : x)));
  };
  // start vector: mt19937(seed) normal numbers; the generalised mode puts it into range(OP) first
  // (dgetv0 for mode 3)
  {
    std::vector<double> h(n);
    host_random_normal(n, seed, h.data());
    EIG_HIP(hipMemcpyAsync(W, h.data(), n * 8, hipMemcpyHostToDevice, s));
    if (gen)
    {
      bmul(W, BW);
      solve(BW, V);
    }
    else
      EIG_HIP(hipMemcpyAsync(V, W, n * 8, hipMemcpyDeviceToDevice, s));
    const double nb = norm_in(V, BV);
    EIG_CHECK(nb > 0.0, EIG_ERR_BREAKDOWN, "Arnoldi: zero start vector");
    launch_scal(n, 1.0 / nb, V, s);
    if (bip) launch_scal(n, 1.0 / nb, BV, s);
  }
  std::vector<double> G((size_t)m * m, 0.0), cvec, ctot(m + 1);
  // per step j: the two CGS passes' coefficients and the squared norm of the new vector, on the
  // device; one read-back per extension (as shift_invert_core)
  const i64 cstride = 2 * (i64)(m + 1) + 1;
  DevBuf coefb((size_t)m * cstride * 8);
  double *coef = coefb.d();
  std::vector<double> coefh((size_t)m * cstride);
  std::vector<C> w, Y;
  std::vector<int> ord(m);
  double beta = 0.0;
  int k = 0, nrestart = 0;
  for (;;)
  {
    // extend the Krylov decomposition from k to m vectors (Arnoldi steps)
    for (int j = k; j < m; ++j)
    {
      double *vj = V + (i64)j * n;
      double *cj = coef + (i64)j * cstride;
      bmul(vj, BW);
      solve(BW, W);  // W = OP v_j (the reverse-communication product)
      for (int pass = 0; pass < 2; ++pass)  // CGS2 against v_0 .. v_j in the inner product
      {
        launch_gemv_t(n, j + 1, BV, n, W, cj + pass * (m + 1), 0, s, ctx->red);
        launch_gemv_n_sub(n, j + 1, V, n, cj + pass * (m + 1), nullptr, W, s);
      }
      if (bip) bmul(W, BW);
      launch_dot(n, W, bip ? BW : W, cj + 2 * (m + 1), 0, s, ctx->red);  // beta_j^2
      double *vn = V + (i64)(j + 1) * n;
      EIG_HIP(hipMemcpyAsync(vn, W, n * 8, hipMemcpyDeviceToDevice, s));
      launch_scal_dev(n, cj + 2 * (m + 1), true, vn, s);
      if (bip)
      {
        double *bvn = BV + (i64)(j + 1) * n;
        EIG_HIP(hipMemcpyAsync(bvn, BW, n * 8, hipMemcpyDeviceToDevice, s));
        launch_scal_dev(n, cj + 2 * (m + 1), true, bvn, s);
      }
    }
    EIG_HIP(hipMemcpyAsync(coefh.data() + (size_t)k * cstride, coef + (i64)k * cstride,
                           (size_t)(m - k) * cstride * 8, hipMemcpyDeviceToHost, s));
    EIG_HIP(hipStreamSynchronize(s));
    for (int j = k; j < m; ++j)
    {
      if (j > 0)
        for (int i = 0; i < j; ++i) G[(size_t)j * m + i] = beta * cvec[i];
      const double *ch = coefh.data() + (size_t)j * cstride;
      std::fill(ctot.begin(), ctot.end(), 0.0);
      for (int pass = 0; pass < 2; ++pass)
        for (int i = 0; i <= j; ++i) ctot[i] += ch[pass * (m + 1) + i];
      for (int i = 0; i <= j; ++i) G[(size_t)i * m + j] = ctot[i];
      beta = std::sqrt(std::max(0.0, ch[2 * (m + 1)]));
      double hn = 0.0;
      for (int i = 0; i <= j; ++i) hn = std::max(hn, std::fabs(ctot[i]));
      EIG_CHECK(beta > 1e-14 * hn, EIG_ERR_BREAKDOWN,
                "Arnoldi: invariant subspace reached (choose ncv < n or another seed)");
      cvec.assign(j + 1, 0.0);
      cvec[j] = 1.0;
    }
    EIG_CHECK(gen_eig(m, G, w, Y), EIG_ERR_BREAKDOWN, "Arnoldi: QR iteration of the projected matrix failed");
    // "LM": largest |nu| first (conjugate partners keep their relative order)
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return std::abs(w[a]) > std::abs(w[b]); });
    auto resid = [&](int q) {
      C r = 0.0;
      for (int i = 0; i < m; ++i) r += cvec[i] * Y[(size_t)i * m + q];
      return beta * std::abs(r);
    };
    bool conv = true;
    for (int i = 0; i < nev; ++i)
      if (resid(ord[i]) > tol * std::abs(w[ord[i]])) conv = false;
    if (conv || nrestart >= maxit) break;
    // Krylov-Schur restart: about nev + (m - nev) / 2 wanted vectors, never splitting a conjugate
    // pair.  The kept set is built from whole units in "LM" order -- a real Ritz value (one column)
    // or a conjugate pair (real and imaginary part: two columns; its partner is looked up by value,
    // wherever the sort put it) -- so span(Z) is G-invariant whatever the ordering of equal moduli.
    const int target = std::min(m - 2, nev + (m - nev) / 2);
    std::vector<std::pair<int, bool>> units;  // (eigenvalue index, complex pair)
    int kk = 0;
    {
      std::vector<char> used(m, 0);
      for (int q = 0; q < m && kk < target; ++q)
      {
        const int e = ord[q];
        if (used[e]) continue;
        used[e] = 1;
        const bool cplx = w[e].imag() != 0.0;
        if (cplx)
        {
          int partner = -1;
          for (int q2 = 0; q2 < m; ++q2)
            if (!used[ord[q2]] && w[ord[q2]] == std::conj(w[e]))
            {
              partner = ord[q2];
              break;
            }
          EIG_CHECK(partner >= 0, EIG_ERR_BREAKDOWN, "Arnoldi: complex Ritz value without its conjugate");
          used[partner] = 1;
          if (kk + 2 > m - 1) break;  // a pair that does not fit is dropped whole
        }
        units.push_back({e, cplx});
        kk += cplx ? 2 : 1;
      }
    }
    EIG_CHECK(kk >= 1, EIG_ERR_BREAKDOWN, "Arnoldi: no Ritz vector to keep at restart");
    std::vector<double> Z((size_t)m * kk, 0.0);  // row-major m x kk
    {
      int col = 0;
      for (auto &u : units)
      {
        for (int i = 0; i < m; ++i) Z[(size_t)i * kk + col] = Y[(size_t)i * m + u.first].real();
        ++col;
        if (u.second)
        {
          for (int i = 0; i < m; ++i) Z[(size_t)i * kk + col] = Y[(size_t)i * m + u.first].imag();
          ++col;
        }
      }
      for (int c = 0; c < kk; ++c)  // MGS, twice
        for (int pass = 0; pass < 2; ++pass)
        {
          for (int p = 0; p < c; ++p)
          {
            double d = 0.0;
            for (int i = 0; i < m; ++i) d += Z[(size_t)i * kk + p] * Z[(size_t)i * kk + c];
            for (int i = 0; i < m; ++i) Z[(size_t)i * kk + c] -= d * Z[(size_t)i * kk + p];
          }
          double nr = 0.0;
          for (int i = 0; i < m; ++i) nr += Z[(size_t)i * kk + c] * Z[(size_t)i * kk + c];
          nr = std::sqrt(nr);
          EIG_CHECK(nr > 0.0, EIG_ERR_BREAKDOWN, "Arnoldi: dependent Ritz vectors at restart");
          for (int i = 0; i < m; ++i) Z[(size_t)i * kk + c] /= nr;
        }
    }
    // G <- Z^T G Z, c <- Z^T c; V <- V Z, v_kk <- v_m
    std::vector<double> GZ((size_t)m * kk, 0.0), Gn((size_t)m * m, 0.0), cn(kk, 0.0);
    for (int i = 0; i < m; ++i)
      for (int q = 0; q < kk; ++q)
      {
        double a = 0.0;
        for (int l = 0; l < m; ++l) a += G[(size_t)i * m + l] * Z[(size_t)l * kk + q];
        GZ[(size_t)i * kk + q] = a;
      }
    for (int p = 0; p < kk; ++p)
    {
      for (int q = 0; q < kk; ++q)
      {
        double a = 0.0;
        for (int i = 0; i < m; ++i) a += Z[(size_t)i * kk + p] * GZ[(size_t)i * kk + q];
        Gn[(size_t)p * m + q] = a;
      }
      for (int i = 0; i < m; ++i) cn[p] += Z[(size_t)i * kk + p] * cvec[i];
    }
    {
      // the restarted decomposition is a Krylov decomposition only if span(Z) is G-invariant:
      // ||G Z - Z (Z^T G Z)|| small relative to ||G||
      double gmax = 0.0, rmax = 0.0;
      for (double g : G) gmax = std::max(gmax, std::fabs(g));
      for (int i = 0; i < m; ++i)
        for (int q = 0; q < kk; ++q)
        {
          double a = GZ[(size_t)i * kk + q];
          for (int p = 0; p < kk; ++p) a -= Z[(size_t)i * kk + p] * Gn[(size_t)p * m + q];
          rmax = std::max(rmax, std::fabs(a));
        }
      EIG_CHECK(rmax <= 1e-6 * std::max(gmax, 1e-300), EIG_ERR_BREAKDOWN,
                "Arnoldi: restart subspace is not invariant under the projected matrix");
    }
    G.swap(Gn);
    cvec = cn;
    double *Tmp = Tb.d();
    std::vector<double> coef(m);
    for (int q = 0; q < kk; ++q)
    {
      for (int i = 0; i < m; ++i) coef[i] = Z[(size_t)i * kk + q];
      EIG_HIP(hipMemcpyAsync(cd, coef.data(), m * 8, hipMemcpyHostToDevice, s));
      launch_gemv_n_set(n, m, V, n, cd, nullptr, Tmp + (i64)q * n, s);
      if (bip) launch_gemv_n_set(n, m, BV, n, cd, nullptr, Tmp + (i64)(kk + q) * n, s);
      EIG_HIP(hipStreamSynchronize(s));
    }
    EIG_HIP(hipMemcpyAsync(V, Tmp, (size_t)kk * n * 8, hipMemcpyDeviceToDevice, s));
    EIG_HIP(hipMemcpyAsync(V + (i64)kk * n, V + (i64)m * n, n * 8, hipMemcpyDeviceToDevice, s));
    if (bip)
    {
      EIG_HIP(hipMemcpyAsync(BV, Tmp + (i64)kk * n, (size_t)kk * n * 8, hipMemcpyDeviceToDevice, s));
      EIG_HIP(hipMemcpyAsync(BV + (i64)kk * n, BV + (i64)m * n, n * 8, hipMemcpyDeviceToDevice, s));
    }
    k = kk;
    ++nrestart;
  }
  // eigenvalues of the original problem, ascending by real part (:484-498, :556-571)
  std::vector<C> lam(nev);
  for (int i = 0; i < nev; ++i)
  {
    const C nu = w[ord[i]];
    lam[i] = gen ? C(sigma) + 1.0 / nu : C(sigma + 1.0 / nu.real(), (C(sigma) + 1.0 / nu).imag());
  }
  std::vector<int> idx(nev);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return lam[a].real() < lam[b].real(); });
  for (int i = 0; i < nev; ++i)
  {
    eval_re[i] = lam[idx[i]].real();
    if (eval_im) eval_im[i] = lam[idx[i]].imag();
  }
  if (evec_host)
  {
    // x = V y, unit 2-norm as a complex vector; ARPACK's raw storage of a conjugate pair: the real
    // part for the member with Im(nu) > 0, the imaginary part for its partner
    std::vector<double> coef(m);
    for (int q = 0; q < nev; ++q)
    {
      const int e = ord[idx[q]];
      const bool cplx = w[e].imag() != 0.0;
      int ey = e;
      if (cplx && w[e].imag() < 0.0)
        for (int i = 0; i < m; ++i)
          if (w[i] == std::conj(w[e])) ey = i;
      double nr2 = 0.0;
      for (int part = 0; part < (cplx ? 2 : 1); ++part)
      {
        for (int i = 0; i < m; ++i)
          coef[i] = part == 0 ? Y[(size_t)i * m + ey].real() : Y[(size_t)i * m + ey].imag();
        EIG_HIP(hipMemcpyAsync(cd, coef.data(), m * 8, hipMemcpyHostToDevice, s));
        launch_gemv_n_set(n, m, V, n, cd, nullptr, part == 0 ? W : BW, s);
        nr2 += dot(part == 0 ? W : BW, part == 0 ? W : BW);
      }
      double *x = (cplx && w[e].imag() < 0.0) ? BW : W;
      launch_scal(n, 1.0 / std::sqrt(nr2), x, s);
      EIG_HIP(hipMemcpyAsync(evec_host + (i64)q * n, x, n * 8, hipMemcpyDeviceToHost, s));
      EIG_HIP(hipStreamSynchronize(s));
    }
  }
  if (restarts) *restarts = nrestart;
}

}  // namespace

extern "C" int eig_arnoldi_shift_invert(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double sigma, int nev, int ncv,
                                        double tol, int maxit, unsigned seed, int mode, double *eval_re,
                                        double *eval_im, double *evec_host, int *restarts)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && eval_re && nev > 0, EIG_ERR_ARG, "eig_arnoldi_shift_invert: bad argument");
    EIG_CHECK(mode == EIG_ARNOLDI_STD || mode == EIG_ARNOLDI_GEN, EIG_ERR_ARG, "eig_arnoldi_shift_invert: bad mode");
    shift_invert_check(A, B);
    EIG_HIP(hipSetDevice(A->ctx->device));
    LuRef F;
    shift_invert_factor(A, B, lu, sigma, F);
    arnoldi_core(A, B, F, sigma, nev, ncv, tol, maxit, seed, mode == EIG_ARNOLDI_GEN, eval_re, eval_im, evec_host,
                 restarts);
  });
}

// ============================================================================================
// Lanczos three-term recurrence (DESIGN.md "Lanczos step")
// ============================================================================================
namespace {

struct LanczosBufs {
  DevBuf scal;
  DevBuf ictl;
  LanczosState st;
  double *carry;
  // steps: logical steps; launches: fused launches (a step plus at most one repair each, plus the
  // forced final repair)
  explicit LanczosBufs(int steps, int launches = 0)
      : scal((size_t)(4 * (steps + 2) + 6 * (launches + 2) + 8) * sizeof(double)),
        ictl((size_t)2 * (launches + 2) * sizeof(int))
  {
    double *b = scal.d();
    st.dsum = b;
    st.nsum = b + (steps + 2);
    st.alpha = b + 2 * (steps + 2);
    st.beta = b + 3 * (steps + 2);
    st.fred = b + 4 * (steps + 2);
    st.aux = st.fred + 3 * (launches + 2);
    carry = st.aux + 2 * (launches + 2);
    st.mu2 = carry + 4;
    st.pn = st.mu2 + 4;
    st.ctl = static_cast<int *>(ictl.p);
  }
};

// One step j: t = A u sig - gam up (+ dot), allreduce, u_{j+1} = t - alpha sig u (+ norm), allreduce.
// Optional event timing: ev[0..5] = before K1, after K1, after allreduce 1, after K2, after allreduce 2.
// Halo exchange + SpMV-type launch split into interior slices (no ghost columns) and boundary
// slices.  RCCL: the exchange runs on the comm stream while the interior launch computes; the
// loopback transport exchanges synchronously first (same launches, so its tests cover the split
// and the carry of the partial reductions).  launch(slices, first, count, part): part 0 = the
// only launch of the step, 1 = first of two (writes its partial sums to the carry slot), 2 =
// second (adds the carry).
enum { kPartOnly = 0, kPartFirst = 1, kPartSecond = 2 };
template <class Halo, class Launch>
void halo_split(eig_mat_s &A, hipEvent_t e0, hipEvent_t e1, Halo halo, Launch launch)
{
  eig_ctx_t ctx = A.ctx;
  hipStream_t s = ctx->stream;
  if (!distributed(A) || (A.recvs.empty() && A.sends.empty()))
  {
    launch(nullptr, 0, A.nslices, kPartOnly);
    return;
  }
  if (ctx->loop)
    halo(s);
  else
  {
    EIG_HIP(hipEventRecord(e0, s));
    EIG_HIP(hipStreamWaitEvent(ctx->comm_stream, e0, 0));
    halo(ctx->comm_stream);
    EIG_HIP(hipEventRecord(e1, ctx->comm_stream));
  }
  if (A.tune_halo_whole)
  {
    // EIG_TUNE_HALO = 1: wait for the exchange, then one launch over every owned row
    if (!ctx->loop) EIG_HIP(hipStreamWaitEvent(s, e1, 0));
    launch(nullptr, 0, A.nslices, kPartOnly);
    return;
  }
  if (march_split_active(A))
  {
    // interior planes on the plane march (k_spmv.hip), every other slice after the exchange
    const bool has_bd = A.n_march_bnd > 0;
    launch(&kMarchInteriorTag, 0, 0, has_bd ? kPartFirst : kPartOnly);
    if (!ctx->loop) EIG_HIP(hipStreamWaitEvent(s, e1, 0));
    if (has_bd) launch(A.march_bnd, 0, A.n_march_bnd, kPartSecond);
    return;
  }
  const bool has_in = A.n_interior > 0, has_bd = A.n_boundary > 0;
  if (has_in) launch(A.slice_list, 0, A.n_interior, has_bd ? kPartFirst : kPartOnly);
  if (!ctx->loop) EIG_HIP(hipStreamWaitEvent(s, e1, 0));
  if (has_bd) launch(A.slice_list, A.n_interior, A.n_boundary, has_in ? kPartSecond : kPartOnly);
}

// ev_external: the step is being captured into a hipGraph, so the timing events become external
// event-record nodes (a plain record during capture is only a fork/join marker).
// ev: nullptr, 2 events (K1 bracket) or 5 (detail: + after allreduce 1, after K2, after allreduce 2).
void lanczos_step(eig_mat_s &A, double *u, double *up, double *t, int j, LanczosBufs &lb, hipEvent_t *ev, int nev,
                  hipEvent_t halo_ev0, hipEvent_t halo_ev1, bool ev_external = false)
{
  eig_ctx_t ctx = A.ctx;
  hipStream_t s = ctx->stream;
  const i64 own = A.own_offset;
  const i64 n = A.nb_rows;
  auto mark = [&](int i) {
    if (ev && i < nev)
      EIG_HIP(hipEventRecordWithFlags(ev[i], s, ev_external ? hipEventRecordExternal : hipEventRecordDefault));
  };
  mark(0);
  halo_split(
      A, halo_ev0, halo_ev1, [&](hipStream_t hs) { halo_exchange(A, u, hs); },
      [&](const i32 *sl, i64 first, i64 count, int part) {
        launch_lanczos_spmv(A, u, up, t, j, lb.st, sl, first, count, part == kPartFirst ? lb.carry : lb.st.dsum + j,
                            lb.st.beta + j, part == kPartSecond ? lb.carry : nullptr, 0, s, ctx->red);
      });
  mark(1);
  allreduce_sum(ctx, lb.st.dsum + j, 1, s);
  mark(2);
  launch_lanczos_update(n, u + own, t + own, j, lb.st, 0, s, ctx->red);
  mark(3);
  allreduce_sum(ctx, lb.st.nsum + j + 1, 1, s);
  mark(4);
}

// One fused launch L (k_spmv.hip "Fused one-reduction Lanczos step"; a step or a repair, decided
// on the device): P = interleaved pairs of the previous launch (window layout, ghosts exchanged
// here), the output pairs go to Pout; one allreduce of the launch's three sums.  Events as
// lanczos_step: ev[0] before, ev[1] after the kernel, ev[2..4] after the allreduce.
// xch = kXchPublish (EIG_AR_MAILBOX_STEP, xch_dev.h): the kernel's last workgroup allreduces the
// sums through the peers' mailboxes, no allreduce call here.  (A split step: the boundary launch,
// which completes the sums.)
void lanczos_fused_step(eig_mat_s &A, double *P, double *Pout, int L, int force, LanczosBufs &lb, hipEvent_t *ev,
                        int nev, hipEvent_t halo_ev0, hipEvent_t halo_ev1, bool ev_external, int xch = 0)
{
  eig_ctx_t ctx = A.ctx;
  hipStream_t s = ctx->stream;
  auto mark = [&](int i) {
    if (ev && i < nev)
      EIG_HIP(hipEventRecordWithFlags(ev[i], s, ev_external ? hipEventRecordExternal : hipEventRecordDefault));
  };
  double *out = lb.st.fred + 3 * (i64)L;
  FusedLaunch fl{lb.st, L, force, xch & kXchPublish};
  FusedLaunch fl_first{lb.st, L, force, 0};
  mark(0);
  halo_split(
      A, halo_ev0, halo_ev1, [&](hipStream_t hs) { halo_exchange(A, P, hs, nullptr, 2); },
      [&](const i32 *sl, i64 first, i64 count, int part) {
        launch_lanczos_fused(A, P, Pout, part == kPartFirst ? fl_first : fl, sl, first, count,
                             part == kPartSecond ? lb.carry : nullptr, part == kPartFirst ? lb.carry : out, 0, s,
                             ctx->red);
      });
  mark(1);
  if (!(xch & kXchPublish)) allreduce_sum(ctx, out, 3, s);
  mark(2);
  mark(3);
  mark(4);
}

// Start vector into the owned rows of a zeroed window buffer: u0 (device, window layout) or
// mt19937(seed) normal numbers for the GLOBAL vector, of which this rank keeps its rows.
void init_start(eig_mat_s &A, double *U0, const double *u0, unsigned seed)
{
  eig_ctx_t ctx = A.ctx;
  hipStream_t s = ctx->stream;
  EIG_HIP(hipMemsetAsync(U0, 0, A.window * sizeof(double), s));
  const i64 n = A.nb_rows * A.br;
  if (u0)
  {
    EIG_HIP(hipMemcpyAsync(U0 + A.own_offset, u0 + A.own_offset, n * sizeof(double), hipMemcpyDeviceToDevice, s));
  }
  else
  {
    const i64 first = A.row_begin * A.br;
    std::vector<double> h((size_t)(first + n));
    host_random_normal(first + n, seed, h.data());
    EIG_HIP(hipMemcpyAsync(U0 + A.own_offset, h.data() + first, n * sizeof(double), hipMemcpyHostToDevice, s));
    EIG_HIP(hipStreamSynchronize(s));
  }
}

}  // namespace

struct eig_lanczos_s {
  eig_mat_s *A = nullptr;
  int max_steps = 0, k = 0;
  bool fused = false;  // EIG_LANCZOS_FUSED: B = {P0, P1} (2-wide pair vectors); else B = {u_j rotation of 3}
  // EIG_LANCZOS_PIPELINED (implies fused launch accounting): B = {T, UZ pairs, S}; hp = after the
  // row kernel (main stream), ha = after its allreduce (red_stream, when that overlaps)
  bool pipe = false;
  hipEvent_t hp = nullptr, ha = nullptr;
  // fused: launches issued (a repair is a launch, not a step) and the launch capacity
  int L = 0, max_launches = 0;
  DevBuf *B[4] = {nullptr, nullptr, nullptr, nullptr};
  LanczosBufs *lb = nullptr;
  hipEvent_t h0 = nullptr, h1 = nullptr;
  // pending eig_lanczos_capture batch (graph == nullptr with g_steps > 0: eager fallback)
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  int g_steps = 0, g_flags = 0;
  std::vector<hipEvent_t> g_ev;  // [beg, end, events_per_step(g_flags) per step]
  void drop_graph()
  {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
    for (auto &e : g_ev) (void)hipEventDestroy(e);
    gexec = nullptr;
    graph = nullptr;
    g_ev.clear();
    g_steps = 0;
  }
  ~eig_lanczos_s()
  {
    drop_graph();
    for (auto *b : B) delete b;
    delete lb;
    if (h0) (void)hipEventDestroy(h0);
    if (h1) (void)hipEventDestroy(h1);
    if (hp) (void)hipEventDestroy(hp);
    if (ha) (void)hipEventDestroy(ha);
  }
};

namespace {

void check_lanczos_matrix(const eig_mat_s *A)
{
  EIG_CHECK(A->br == 1 && A->bc == 1, EIG_ERR_BLOCKSIZE, "Lanczos driver: 1x1 blocks only");
  EIG_CHECK(A->nb_rows_global == A->nb_cols, EIG_ERR_SHAPE, "Lanczos needs a square matrix");
}

// Events per step for the timing flags: EIG_LANCZOS_TIME_KERNELS brackets the fused SpMV only (two
// timestamps per step keep the perturbation of the timed loop small), EIG_LANCZOS_TIME_DETAIL adds the
// allreduce / update boundaries.
int events_per_step(int flags)
{
  return (flags & EIG_LANCZOS_TIME_DETAIL) ? 5 : (flags & EIG_LANCZOS_TIME_KERNELS) ? 2 : 0;
}

// Pipelined launch L (k_spmv.hip k_lanczos_pipe): S = A t_{k-1} -- interior planes
// while the halo of T is exchanged, boundary planes after it -- needs nothing from launch L-1's
// allreduce, which is still running on red_stream; only the row kernel waits for it.  Its sums
// then go out on red_stream while launch L+1's SpMV computes.  Without a concurrent transport (one
// rank, loopback) the allreduce runs in line.  wait_prev: launch L-1 was enqueued in the same batch
// (its allreduce event was recorded there; a batch starts after a join).  Events as
// lanczos_fused_step (ev[1]: after the row kernel).
void lanczos_pipe_step(eig_lanczos_s &ws, int L, int force, bool wait_prev, hipEvent_t *ev, int nev,
                       bool ev_external)
{
  eig_mat_s &A = *ws.A;
  eig_ctx_t ctx = A.ctx;
  hipStream_t s = ctx->stream;
  auto mark = [&](int i) {
    if (ev && i < nev)
      EIG_HIP(hipEventRecordWithFlags(ev[i], s, ev_external ? hipEventRecordExternal : hipEventRecordDefault));
  };
  double *T = ws.B[0]->d(), *UZ = ws.B[1]->d(), *S = ws.B[2]->d();
  double *out = ws.lb->st.fred + 3 * (i64)L;
  const bool ovl = allreduce_overlaps(ctx);
  mark(0);
  halo_split(
      A, ws.h0, ws.h1, [&](hipStream_t hs) { halo_exchange(A, T, hs); },
      [&](const i32 *sl, i64 first, i64 count, int) { launch_spmv(A, T, S, sl, first, count, s, true); });
  if (ovl && wait_prev) EIG_HIP(hipStreamWaitEvent(s, ws.ha, 0));  // launch L-1's sums are in
  launch_lanczos_pipe(A, T, UZ, S, FusedLaunch{ws.lb->st, L, force}, out, s, ctx->red);
  mark(1);
  if (ovl)
  {
    EIG_HIP(hipEventRecord(ws.hp, s));
    EIG_HIP(hipStreamWaitEvent(ctx->red_stream, ws.hp, 0));
    allreduce_sum_red(ctx, out, 3, ctx->red_stream);
    EIG_HIP(hipEventRecord(ws.ha, ctx->red_stream));
  }
  else
    allreduce_sum(ctx, out, 3, s);
  mark(2);
  mark(3);
  mark(4);
}

// The library stream waits for the last pipelined allreduce (joins red_stream back, e.g. before a
// synchronisation or the end of a graph capture).
void pipe_join(eig_lanczos_s &ws)
{
  if (ws.pipe && allreduce_overlaps(ws.A->ctx)) EIG_HIP(hipStreamWaitEvent(ws.A->ctx->stream, ws.ha, 0));
}

// ev = [beg, end, nps per step]; enqueues steps k .. k+steps-1 (fused: launches L .. L+steps-1) on
// the library stream.
void enqueue_steps(eig_lanczos_s &ws, int steps, int nps, hipEvent_t *ev, bool external)
{
  eig_mat_s &A = *ws.A;
  hipStream_t s = A.ctx->stream;
  const unsigned fl = external ? hipEventRecordExternal : hipEventRecordDefault;
  EIG_HIP(hipEventRecordWithFlags(ev[0], s, fl));
  for (int i = 0; i < steps; ++i)
  {
    hipEvent_t *e = nps ? ev + 2 + (size_t)nps * i : nullptr;
    if (ws.pipe)
      lanczos_pipe_step(ws, ws.L + i, 0, i > 0, e, nps, external);
    else if (ws.fused)
    {
      const int L = ws.L + i;
      lanczos_fused_step(A, ws.B[L & 1]->d(), ws.B[(L + 1) & 1]->d(), L, 0, *ws.lb, e, nps, ws.h0, ws.h1, external,
                         A.ctx->step_exchange() ? kXchPublish : 0);
    }
    else
    {
      const int j = ws.k + i;
      double *U[3] = {ws.B[0]->d(), ws.B[1]->d(), ws.B[2]->d()};
      lanczos_step(A, U[j % 3], U[(j + 2) % 3], U[(j + 1) % 3], j, *ws.lb, e, nps, ws.h0, ws.h1, external);
    }
  }
  if (steps > 0) pipe_join(ws);
  EIG_HIP(hipEventRecordWithFlags(ev[1], s, fl));
}

// The in-kernel exchange of a fused batch: NaN sums mean a peer's exchange timed out (xch_dev.h:
// then every rank reads NaN -- the same decision on all ranks).  Called after a synchronisation.
void check_step_exchange(eig_lanczos_s &ws)
{
  if (!ws.fused || ws.pipe || ws.L == 0 || !ws.A->ctx->step_exchange()) return;
  double f[3];
  EIG_HIP(hipMemcpy(f, ws.lb->st.fred + 3 * (i64)(ws.L - 1), sizeof(f), hipMemcpyDeviceToHost));
  if (!(std::isfinite(f[0]) && std::isfinite(f[1]) && std::isfinite(f[2])))
    throw Error(EIG_ERR_RCCL, "fused Lanczos: the in-kernel xGMI exchange of the step sums failed (a peer timed "
                              "out, or the recurrence produced NaN)");
}

// Fused workspace: control word of launch L (logical step, mode), read after a synchronisation.
void fused_state(eig_lanczos_s &ws, int &j, int &mode)
{
  int c[2];
  EIG_HIP(hipMemcpy(c, ws.lb->st.ctl + 2 * (i64)ws.L, sizeof(c), hipMemcpyDeviceToHost));
  j = c[0];
  mode = c[1];
}

void read_timing(const std::vector<hipEvent_t> &ev, int steps, int nps, eig_timing *timing, bool accumulate = false);
std::vector<hipEvent_t> make_events(int steps, int nps);

// After `launched` fused launches were enqueued for logical steps up to `target`: synchronise, then
// top up with eager launches until the target step is reached (launches that repaired took no
// step).  Extra batches add to `timing`.  Breakdown (u_j = 0) ends the recurrence at step j.
void fused_settle(eig_lanczos_s &ws, int target, int nps, eig_timing *timing)
{
  eig_ctx_t ctx = ws.A->ctx;
  for (;;)
  {
    int j, mode;
    check_step_exchange(ws);
    fused_state(ws, j, mode);
    ws.k = j;
    if (mode == kFusedModeHalt)
      throw Error(EIG_ERR_BREAKDOWN, "Lanczos breakdown: invariant subspace after " + std::to_string(j) + " steps");
    if (j >= target) return;
    const int more = target - j;
    EIG_CHECK(ws.L + more <= ws.max_launches, EIG_ERR_ARG, "fused Lanczos: launch capacity exhausted");
    std::vector<hipEvent_t> ev = make_events(more, nps);
    try
    {
      enqueue_steps(ws, more, nps, ev.data(), false);
      EIG_HIP(hipStreamSynchronize(ctx->stream));
      ws.L += more;
      read_timing(ev, more, nps, timing, true);
    }
    catch (...)
    {
      for (auto &e : ev) (void)hipEventDestroy(e);
      throw;
    }
    for (auto &e : ev) (void)hipEventDestroy(e);
  }
}

std::vector<hipEvent_t> make_events(int steps, int nps)
{
  std::vector<hipEvent_t> ev(2 + (size_t)nps * steps);
  for (auto &e : ev) EIG_HIP(hipEventCreate(&e));
  return ev;
}

void read_timing(const std::vector<hipEvent_t> &ev, int steps, int nps, eig_timing *timing, bool accumulate)
{
  if (!timing) return;
  if (!accumulate) std::memset(timing, 0, sizeof(*timing));
  float ms = 0.f;
  EIG_HIP(hipEventElapsedTime(&ms, ev[0], ev[1]));
  timing->total_ms += ms;
  if (!nps) return;  // region events only: no per-launch kernel timing
  timing->spmv_launches += steps;
  for (int i = 0; i < steps; ++i)
  {
    const hipEvent_t *e = &ev[2 + (size_t)nps * i];
    float a = 0, b = 0, c = 0, d = 0;
    EIG_HIP(hipEventElapsedTime(&a, e[0], e[1]));
    timing->spmv_ms += a;
    if (nps < 5) continue;
    EIG_HIP(hipEventElapsedTime(&b, e[1], e[2]));
    EIG_HIP(hipEventElapsedTime(&c, e[2], e[3]));
    EIG_HIP(hipEventElapsedTime(&d, e[3], e[4]));
    timing->comm_ms += b + d;
    timing->update_ms += c;
  }
}

}  // namespace

extern "C" int eig_lanczos_create(eig_mat_t A, int max_steps, const double *u0, unsigned seed, eig_lanczos_t *out)
{
  return eig_lanczos_create_ex(A, max_steps, u0, seed, 0, out);
}

extern "C" int eig_lanczos_create_ex(eig_mat_t A, int max_steps, const double *u0, unsigned seed, int flags,
                                     eig_lanczos_t *out)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && out && max_steps >= 0, EIG_ERR_ARG, "eig_lanczos_create: bad argument");
    EIG_CHECK((flags & ~(EIG_LANCZOS_FUSED | EIG_LANCZOS_PIPELINED | EIG_LANCZOS_AUTO)) == 0, EIG_ERR_ARG,
              "eig_lanczos_create_ex: unknown flag");
    EIG_CHECK(__builtin_popcount(flags & (EIG_LANCZOS_FUSED | EIG_LANCZOS_PIPELINED | EIG_LANCZOS_AUTO)) <= 1,
              EIG_ERR_ARG, "eig_lanczos_create_ex: FUSED, PIPELINED and AUTO are exclusive");
    check_lanczos_matrix(A);
    if (flags & EIG_LANCZOS_AUTO) flags = fused_step_pays(*A) ? EIG_LANCZOS_FUSED : 0;
    eig_ctx_t ctx = A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    auto *ws = new eig_lanczos_s();
    try
    {
      ws->A = A;
      ws->max_steps = max_steps;
      ws->pipe = (flags & EIG_LANCZOS_PIPELINED) != 0;
      ws->fused = ws->pipe || (flags & EIG_LANCZOS_FUSED) != 0;
      if (ws->pipe) (void)allreduce_overlaps(ctx);  // creates the reduction stream before any capture
      // worst case: every step repaired, plus one forced repair per eig_lanczos_tridiag call
      ws->max_launches = ws->fused ? 3 * max_steps + 8 : 0;
      const size_t wb = (size_t)A->window * sizeof(double);
      for (int i = 0; i < 3; ++i)
      {
        // fused: B[0], B[1] = pair vectors (2 doubles per row), B[2] = start vector scratch;
        // pipelined: B[0] = T (t_0 = u_0), B[1] = (u, z) pairs, B[2] = S
        const bool pair = ws->pipe ? i == 1 : (ws->fused && i < 2);
        ws->B[i] = new DevBuf(pair ? 2 * wb : wb);
        if (i) EIG_HIP(hipMemsetAsync(ws->B[i]->d(), 0, ws->B[i]->bytes(), s));
      }
      double *U0 = ws->pipe ? ws->B[0]->d() : ws->fused ? ws->B[2]->d() : ws->B[0]->d();
      init_start(*A, U0, u0, seed);
      ws->lb = new LanczosBufs(max_steps, ws->max_launches);
      launch_nrm2sq(A->nb_rows, U0 + A->own_offset, ws->lb->st.nsum, 0, s, ctx->red);
      if (ws->fused)  // P0 = (u_0, 0) interleaved; the whole window (ghosts are refilled per step)
      {
        if (!ws->pipe)
        {
          EIG_HIP(hipMemsetAsync(ws->B[0]->d(), 0, 2 * wb, s));
          EIG_HIP(hipMemcpy2DAsync(ws->B[0]->d(), 2 * sizeof(double), U0, sizeof(double), sizeof(double),
                                   A->window, hipMemcpyDeviceToDevice, s));
        }
        // launch 0 takes step 0; the shift mu = trace / n from every rank's diagonal share
        EIG_HIP(hipMemsetAsync(ws->lb->st.ctl, 0, ws->lb->ictl.bytes(), s));
        const double mu2[2] = {A->diag_sum, (double)A->nb_rows};
        EIG_HIP(hipMemcpyAsync(ws->lb->st.mu2, mu2, sizeof(mu2), hipMemcpyHostToDevice, s));
        allreduce_sum(ctx, ws->lb->st.mu2, 2, s);
      }
      allreduce_sum(ctx, ws->lb->st.nsum, 1, s);
      EIG_HIP(hipEventCreateWithFlags(&ws->h0, hipEventDisableTiming));
      EIG_HIP(hipEventCreateWithFlags(&ws->h1, hipEventDisableTiming));
      EIG_HIP(hipEventCreateWithFlags(&ws->hp, hipEventDisableTiming));
      EIG_HIP(hipEventCreateWithFlags(&ws->ha, hipEventDisableTiming));
      EIG_HIP(hipStreamSynchronize(s));
    }
    catch (...)
    {
      delete ws;
      throw;
    }
    *out = ws;
  });
}

extern "C" int eig_lanczos_step(eig_lanczos_t ws, int steps, int flags, eig_timing *timing)
{
  return guard(ws ? ws->A->ctx : nullptr, [&] {
    EIG_CHECK(ws && steps >= 0, EIG_ERR_ARG, "eig_lanczos_step: bad argument");
    EIG_CHECK(ws->k + steps <= ws->max_steps, EIG_ERR_ARG, "eig_lanczos_step: more steps than max_steps");
    EIG_CHECK((flags & ~(EIG_LANCZOS_TIME_KERNELS | EIG_LANCZOS_TIME_DETAIL)) == 0, EIG_ERR_ARG, "eig_lanczos_step: unknown flag");
    EIG_CHECK(!ws->fused || ws->L + steps <= ws->max_launches, EIG_ERR_ARG, "fused Lanczos: launch capacity exhausted");
    ws->drop_graph();  // a pending capture is for steps that are about to be taken eagerly
    eig_ctx_t ctx = ws->A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    const int nps = events_per_step(flags);
    const int target = ws->k + steps;
    std::vector<hipEvent_t> ev = make_events(steps, nps);
    try
    {
      enqueue_steps(*ws, steps, nps, ev.data(), false);
      EIG_HIP(hipStreamSynchronize(ctx->stream));
      if (ws->fused) ws->L += steps;
      else ws->k += steps;
      read_timing(ev, steps, nps, timing);
    }
    catch (...)
    {
      for (auto &e : ev) (void)hipEventDestroy(e);
      throw;
    }
    for (auto &e : ev) (void)hipEventDestroy(e);
    if (ws->fused) fused_settle(*ws, target, nps, timing);
  });
}

extern "C" int eig_lanczos_ws_info(eig_lanczos_t ws, int *variant, char *name, int name_len, int64_t *bytes)
{
  return guard(ws ? ws->A->ctx : nullptr, [&] {
    EIG_CHECK(ws, EIG_ERR_ARG, "eig_lanczos_ws_info: null workspace");
    if (variant) *variant = ws->pipe ? EIG_LANCZOS_PIPELINED : ws->fused ? EIG_LANCZOS_FUSED : 0;
    std::string nm;
    i64 b = 0;
    if (ws->pipe)
    {
      nm = kernel_for(*ws->A, EIG_OP_SPMV) + "+k_lanczos_pipe";
      b = 0;  // (two launches per step: see bench.py)
    }
    else
      lanczos_kernel_info(*ws->A, ws->fused, nm, b);
    if (name && name_len > 0)
    {
      std::strncpy(name, nm.c_str(), (size_t)name_len - 1);
      name[name_len - 1] = 0;
    }
    if (bytes) *bytes = b;
  });
}

extern "C" int eig_lanczos_capture(eig_lanczos_t ws, int steps, int flags, int *captured)
{
  return guard(ws ? ws->A->ctx : nullptr, [&] {
    EIG_CHECK(ws && steps > 0, EIG_ERR_ARG, "eig_lanczos_capture: bad argument");
    EIG_CHECK(ws->k + steps <= ws->max_steps, EIG_ERR_ARG, "eig_lanczos_capture: more steps than max_steps");
    EIG_CHECK((flags & ~(EIG_LANCZOS_TIME_KERNELS | EIG_LANCZOS_TIME_DETAIL)) == 0, EIG_ERR_ARG, "eig_lanczos_capture: unknown flag");
    EIG_CHECK(!ws->fused || ws->L + steps <= ws->max_launches, EIG_ERR_ARG, "fused Lanczos: launch capacity exhausted");
    ws->drop_graph();
    eig_ctx_t ctx = ws->A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    ws->g_steps = steps;
    ws->g_flags = flags;
    ws->g_ev = make_events(steps, events_per_step(flags));
    if (captured) *captured = 0;
    // the loopback transport synchronises with the host inside the step: eager replay only
    if (ctx->loop) return;
    hipStream_t s = ctx->stream;
    march_prepare(*ws->A);  // (builds a value pack outside the graph, never as a captured node)
    EIG_HIP(hipStreamSynchronize(s));
    EIG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    hipGraph_t g = nullptr;
    bool ok = true;
    try
    {
      enqueue_steps(*ws, steps, events_per_step(flags), ws->g_ev.data(), true);
    }
    catch (...)
    {
      ok = false;
    }
    hipError_t e = hipStreamEndCapture(s, &g);
    if (!ok || e != hipSuccess || !g)
    {
      if (g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
      return;  // capture refused (e.g. by the collective library): eager replay
    }
    ws->graph = g;
    if (hipGraphInstantiate(&ws->gexec, g, nullptr, nullptr, 0) != hipSuccess)
    {
      (void)hipGetLastError();
      (void)hipGraphDestroy(g);
      ws->graph = nullptr;
      ws->gexec = nullptr;
      return;
    }
    if (captured) *captured = 1;
  });
}

extern "C" int eig_lanczos_replay(eig_lanczos_t ws, eig_timing *timing)
{
  return guard(ws ? ws->A->ctx : nullptr, [&] {
    EIG_CHECK(ws && ws->g_steps > 0, EIG_ERR_ARG, "eig_lanczos_replay: nothing captured");
    eig_ctx_t ctx = ws->A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int steps = ws->g_steps;
    const int nps = events_per_step(ws->g_flags);
    const int target = ws->k + steps;
    if (ws->gexec)
      EIG_HIP(hipGraphLaunch(ws->gexec, s));
    else
      enqueue_steps(*ws, steps, nps, ws->g_ev.data(), false);
    EIG_HIP(hipStreamSynchronize(s));
    if (ws->fused) ws->L += steps;
    else ws->k += steps;
    read_timing(ws->g_ev, steps, nps, timing);
    ws->drop_graph();
    if (ws->fused) fused_settle(*ws, target, nps, timing);
  });
}

extern "C" int eig_lanczos_tridiag(eig_lanczos_t ws, int *k, double *alpha_host, double *beta_host)
{
  return guard(ws ? ws->A->ctx : nullptr, [&] {
    EIG_CHECK(ws, EIG_ERR_ARG, "eig_lanczos_tridiag: null workspace");
    eig_ctx_t ctx = ws->A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    EIG_HIP(hipStreamSynchronize(ctx->stream));
    if (ws->fused)
    {
      // alpha[k-1] and an EXACT beta[k]: a forced repair forms u_k and reduces its norm (the
      // prediction is only used to scale a step, never reported), then the tail stores beta[k]
      int j, mode;
      fused_state(*ws, j, mode);
      if (mode == kFusedModeStep && j > 0)
      {
        EIG_CHECK(ws->L + 1 <= ws->max_launches, EIG_ERR_ARG, "fused Lanczos: launch capacity exhausted");
        if (ws->pipe)
        {
          lanczos_pipe_step(*ws, ws->L, 1, false, nullptr, 0, false);
          pipe_join(*ws);
        }
        else
          lanczos_fused_step(*ws->A, ws->B[ws->L & 1]->d(), ws->B[(ws->L + 1) & 1]->d(), ws->L, 1, *ws->lb, nullptr,
                             0, ws->h0, ws->h1, false, ctx->step_exchange() ? kXchPublish : 0);
        ++ws->L;
      }
      launch_fused_tail(ws->lb->st, ws->L, ctx->stream);
    }
    else
      launch_beta_tail(ws->lb->st, ws->k, ctx->stream);
    EIG_HIP(hipStreamSynchronize(ctx->stream));
    check_step_exchange(*ws);  // the forced repair exchanged its sums in-kernel too: a timed-out peer -> EIG_ERR_RCCL
    if (k) *k = ws->k;
    if (alpha_host && ws->k > 0)
      EIG_HIP(hipMemcpy(alpha_host, ws->lb->st.alpha, ws->k * sizeof(double), hipMemcpyDeviceToHost));
    if (beta_host) EIG_HIP(hipMemcpy(beta_host, ws->lb->st.beta, (ws->k + 1) * sizeof(double), hipMemcpyDeviceToHost));
  });
}

extern "C" int eig_lanczos_info(eig_lanczos_t ws, int *steps, int *launches)
{
  return guard(ws ? ws->A->ctx : nullptr, [&] {
    EIG_CHECK(ws, EIG_ERR_ARG, "eig_lanczos_info: null workspace");
    if (steps) *steps = ws->k;
    if (launches) *launches = ws->fused ? ws->L : ws->k;
  });
}

extern "C" int eig_lanczos_destroy(eig_lanczos_t ws)
{
  if (!ws) return EIG_OK;
  (void)hipSetDevice(ws->A->ctx->device);
  (void)hipStreamSynchronize(ws->A->ctx->stream);
  delete ws;
  return EIG_OK;
}

extern "C" int eig_lanczos_run(eig_mat_t A, int steps, const double *u0, unsigned seed, int flags, double *alpha_host,
                               double *beta_host, eig_timing *timing)
{
  eig_lanczos_t ws = nullptr;
  const int kind = EIG_LANCZOS_FUSED | EIG_LANCZOS_PIPELINED;
  int rc = eig_lanczos_create_ex(A, steps, u0, seed, flags & kind, &ws);
  if (rc != EIG_OK) return rc;
  rc = eig_lanczos_step(ws, steps, flags & ~kind, timing);
  if (rc == EIG_OK) rc = eig_lanczos_tridiag(ws, nullptr, alpha_host, beta_host);
  eig_lanczos_destroy(ws);
  return rc;
}

// ============================================================================================
// Lanczos eigensolver with full re-orthogonalisation
// ============================================================================================
extern "C" int eig_lanczos_solve(eig_mat_t A, int nev, int ncv, int which, unsigned seed, double *eval_host,
                                 double *evec_host, double *resid_host)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && eval_host && nev > 0 && ncv >= nev && ncv <= 512, EIG_ERR_ARG,
              "eig_lanczos_solve: need 0 < nev <= ncv <= 512");
    EIG_CHECK(which == EIG_WHICH_LA || which == EIG_WHICH_SA, EIG_ERR_ARG, "eig_lanczos_solve: bad `which`");
    EIG_CHECK(A->br == 1 && A->bc == 1, EIG_ERR_BLOCKSIZE, "Lanczos driver: 1x1 blocks only");
    EIG_CHECK(A->nb_rows_global == A->nb_cols, EIG_ERR_SHAPE, "Lanczos needs a square matrix");
    EIG_CHECK(ncv <= A->nb_rows_global, EIG_ERR_SHAPE, "ncv larger than the matrix");
    eig_ctx_t ctx = A->ctx;
    EIG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const i64 W = A->window, own = A->own_offset, n = A->nb_rows;
    DevBuf Vb((size_t)(ncv + 1) * W * sizeof(double));
    double *V = Vb.d();
    EIG_HIP(hipMemsetAsync(V, 0, (size_t)(ncv + 1) * W * sizeof(double), s));
    init_start(*A, V, nullptr, seed);
    LanczosBufs lb(ncv);
    DevBuf cb((size_t)(ncv + 8) * sizeof(double));
    // ||t||^2 after the passes, newest first: [n3, n2, n1, n0] (n0 before any); the gate of pass
    // q is {n_q, n_(q-1)} = &ng[3 - q], as gated_off reads {after, before}
    DevBuf gate(4 * sizeof(double));
    double *ng = gate.d();
    launch_nrm2sq(n, V + own, lb.st.nsum, 0, s, ctx->red);
    allreduce_sum(ctx, lb.st.nsum, 1, s);
    hipEvent_t h0, h1;
    EIG_HIP(hipEventCreateWithFlags(&h0, hipEventDisableTiming));
    EIG_HIP(hipEventCreateWithFlags(&h1, hipEventDisableTiming));
    for (int j = 0; j < ncv; ++j)
    {
      double *u = V + (i64)j * W, *up = j > 0 ? V + (i64)(j - 1) * W : V + (i64)j * W, *t = V + (i64)(j + 1) * W;
      lanczos_step(*A, u, up, t, j, lb, nullptr, 0, h0, h1);
      // DGKS as ARPACK's dsaitr runs it: a classical Gram-Schmidt pass against v_0..v_j
      // (v_q = u_q / sqrt(nsum[q])); a correction pass only when the previous pass removed a large
      // part of t (||t'|| <= 0.717 ||t||), at most two corrections; when the second one still
      // fails the test, t = 0 (dsaitr: r = 0, rnorm = 0 -- an invariant subspace, T_j exact).
      // Every decision is made on the device from the allreduced norms (gated launches).
      launch_nrm2sq(n, t + own, ng + 3, 0, s, ctx->red);
      allreduce_sum(ctx, ng + 3, 1, s);
      for (int pass = 0; pass < 3; ++pass)
      {
        const double *g = pass ? ng + 3 - pass : nullptr;
        for (int q0 = 0; q0 <= j; q0 += 8 * 48)
        {
          const int kq = std::min(j + 1 - q0, 8 * 48);
          launch_gemv_t(n, kq, V + (i64)q0 * W + own, W, t + own, cb.d() + q0, 0, s, ctx->red, g);
        }
        allreduce_sum(ctx, cb.d(), j + 1, s);  // (after a skipped pass: unused)
        launch_gemv_n_sub(n, j + 1, V + own, W, cb.d(), lb.st.nsum, t + own, s, g);
        // ||t||^2 after this pass (a skipped pass leaves t, so n_q = n_(q-1) and the next gate is off)
        launch_nrm2sq(n, t + own, ng + 2 - pass, 0, s, ctx->red);
        allreduce_sum(ctx, ng + 2 - pass, 1, s);
      }
      launch_zero_gated(n, t + own, ng, s);  // {n3, n2}: the second correction failed too
      launch_nrm2sq(n, t + own, lb.st.nsum + j + 1, 0, s, ctx->red);
      allreduce_sum(ctx, lb.st.nsum + j + 1, 1, s);
    }
    (void)hipEventDestroy(h0);
    (void)hipEventDestroy(h1);
    // T = tridiag(beta_1..beta_{k-1}; alpha_0..alpha_{k-1})
    std::vector<double> alpha(ncv), nsum(ncv + 1);
    EIG_HIP(hipStreamSynchronize(s));
    EIG_HIP(hipMemcpy(alpha.data(), lb.st.alpha, ncv * sizeof(double), hipMemcpyDeviceToHost));
    EIG_HIP(hipMemcpy(nsum.data(), lb.st.nsum, (ncv + 1) * sizeof(double), hipMemcpyDeviceToHost));
    int k = ncv;
    for (int j = 1; j < ncv; ++j)
      if (!(nsum[j] > 1e-28 * nsum[0]) || !std::isfinite(alpha[j]))
      {
        k = j;  // invariant subspace found: T_k is exact
        break;
      }
    EIG_CHECK(k >= nev, EIG_ERR_BREAKDOWN, "Lanczos breakdown before nev Ritz values were available");
    std::vector<double> d(alpha.begin(), alpha.begin() + k), e(k > 0 ? k - 1 : 0), Z;
    for (int j = 1; j < k; ++j) e[j - 1] = std::sqrt(nsum[j]);
    tridiag_eig(k, d, e, Z);
    std::vector<int> pick(nev);
    for (int i = 0; i < nev; ++i) pick[i] = (which == EIG_WHICH_LA) ? k - 1 - i : i;
    for (int i = 0; i < nev; ++i) eval_host[i] = d[pick[i]];
    if (evec_host || resid_host)
    {
      DevBuf Y(W * sizeof(double)), AY(W * sizeof(double)), coef((size_t)(k + 1) * sizeof(double));
      double *r2 = cb.d();
      std::vector<double> zc(k);
      for (int i = 0; i < nev; ++i)
      {
        for (int q = 0; q < k; ++q) zc[q] = Z[(size_t)q * k + pick[i]];
        EIG_HIP(hipMemcpyAsync(coef.d(), zc.data(), k * sizeof(double), hipMemcpyHostToDevice, s));
        EIG_HIP(hipMemsetAsync(Y.d(), 0, W * sizeof(double), s));
        launch_gemv_n_set(n, k, V + own, W, coef.d(), lb.st.nsum, Y.d() + own, s);
        if (evec_host)
          EIG_HIP(hipMemcpyAsync(evec_host + (i64)i * n, Y.d() + own, n * sizeof(double), hipMemcpyDeviceToHost, s));
        if (resid_host)
        {
          mv_device(*A, Y.d(), AY.d());
          launch_resid_sq(n, AY.d() + own, Y.d() + own, d[pick[i]], r2 + i, 0, s, ctx->red);
          allreduce_sum(ctx, r2 + i, 1, s);
        }
        EIG_HIP(hipStreamSynchronize(s));
      }
      if (resid_host)
      {
        EIG_HIP(hipMemcpy(resid_host, r2, nev * sizeof(double), hipMemcpyDeviceToHost));
        for (int i = 0; i < nev; ++i) resid_host[i] = std::sqrt(resid_host[i]);
      }
    }
  });
}
