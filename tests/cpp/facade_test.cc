// facade_test.cc -- the drop-in demonstration: reference-style code (an ISTL-concept BCRS matrix,
// a MultiVector<double,8>-compatible container, the reference's kernel names and the ARPACK++
// operator signature) driven through include/eigmi.hh.
//
// The matrix / multivector types below are this test's own minimal stand-ins for the two
// concepts the reference's templates require (kernels_cpp.hh:629-655, multivector.hh:17-146);
// they are the caller's types, not part of the library.
//
//   facade_test            full run on cuda:0 (GPU tests)
//   facade_test --no-device  expects the library to report "no device" (CPU build check)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <array>
#include <random>
#include <vector>

#include "eigmi.hh"

template <int R, int C>
struct Block {  // FieldMatrix<double,R,C>-like: b[i][j]
  static constexpr int rows = R, cols = C;
  double a[R][C];
  const double *operator[](int i) const { return a[i]; }
  double *operator[](int i) { return a[i]; }
  operator double() const { return a[0][0]; }
};

template <int R, int C>
struct TestBCRS {  // BCRSMatrix-like iteration concept
  using block_type = Block<R, C>;
  std::vector<std::vector<std::pair<std::size_t, block_type>>> rows;
  std::size_t ncols = 0;
  struct ColIter {
    const std::pair<std::size_t, block_type> *p;
    std::size_t index() const { return p->first; }
    const block_type &operator*() const { return p->second; }
    ColIter &operator++() { ++p; return *this; }
    bool operator!=(const ColIter &o) const { return p != o.p; }
  };
  struct Row {
    const std::vector<std::pair<std::size_t, block_type>> *r;
    ColIter begin() const { return {r->data()}; }
    ColIter end() const { return {r->data() + r->size()}; }
  };
  struct RowIter {
    const TestBCRS *m;
    std::size_t i;
    mutable Row row;
    std::size_t index() const { return i; }
    const Row *operator->() const { row.r = &m->rows[i]; return &row; }
    RowIter &operator++() { ++i; return *this; }
    bool operator!=(const RowIter &o) const { return i != o.i; }
  };
  RowIter begin() const { return {this, 0, {}}; }
  RowIter end() const { return {this, rows.size(), {}}; }
  std::size_t N() const { return rows.size(); }
  std::size_t M() const { return ncols; }
};

struct MV8 {  // MultiVector<double,8>-like: block-column-major ((j/8)*n+i)*8 + j%8
  static const std::size_t blocksize = 8;
  std::vector<double> p;
  std::size_t n, m;
  MV8(std::size_t n_, std::size_t m_) : p(n_ * m_), n(n_), m(m_) {}
  double &operator()(std::size_t i, std::size_t j) { return p[((j / 8) * n + i) * 8 + j % 8]; }
  const double &operator()(std::size_t i, std::size_t j) const { return p[((j / 8) * n + i) * 8 + j % 8]; }
  std::size_t rows() const { return n; }
  std::size_t cols() const { return m; }
};

static TestBCRS<1, 1> laplace2d(int N)
{
  TestBCRS<1, 1> A;
  A.rows.resize((std::size_t)N * N);
  A.ncols = (std::size_t)N * N;
  for (std::size_t k = 0; k < A.rows.size(); ++k)
  {
    int x = (int)(k % N), y = (int)(k / N);
    auto put = [&](std::size_t c, double v) { Block<1, 1> b; b.a[0][0] = v; A.rows[k].push_back({c, b}); };
    if (y > 0) put(k - N, -1);
    if (x > 0) put(k - 1, -1);
    put(k, 4);
    if (x < N - 1) put(k + 1, -1);
    if (y < N - 1) put(k + N, -1);
  }
  return A;
}

static int failures = 0;
#define EXPECT(c)                                                        \
  do {                                                                   \
    if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++failures; } \
  } while (0)

int main(int argc, char **argv)
{
  if (argc > 1 && std::strcmp(argv[1], "--no-device") == 0)
  {
    try
    {
      eigmi::Context ctx(0);
      std::printf("unexpected: a device is visible\n");
      return 2;
    }
    catch (const std::runtime_error &e)
    {
      std::printf("no device (expected): %s\n", e.what());
      return 0;
    }
  }
  eigmi::Context ctx(0);
  std::mt19937 g(5);
  std::normal_distribution<double> nd(0.0, 1.0);

  // 1) BCRSMatrix::mv, scalar blocks: bitwise vs the ISTL row loop
  auto A = laplace2d(64);
  auto dA = eigmi::Matrix::upload(ctx, A);
  std::vector<double> x(A.N()), y(A.N()), ref(A.N());
  for (auto &v : x) v = nd(g);
  dA.mv_host(x.data(), y.data());
  for (auto r = A.begin(); r != A.end(); ++r)
  {
    double s = 0.0;
    for (auto c = r->begin(); c != r->end(); ++c) s += (double)(*c) * x[c.index()];
    ref[r.index()] = s;
  }
  EXPECT(std::memcmp(y.data(), ref.data(), y.size() * 8) == 0);

  // 2) 3x3 blocks
  TestBCRS<3, 3> B;
  B.rows.resize(100);
  B.ncols = 100;
  for (std::size_t k = 0; k < 100; ++k)
    for (std::size_t c : {k >= 7 ? k - 7 : k, k, (k + 11) % 100})
    {
      if (!B.rows[k].empty() && B.rows[k].back().first >= c) continue;
      Block<3, 3> b;
      for (auto &row : b.a)
        for (auto &v : row) v = nd(g);
      B.rows[k].push_back({c, b});
    }
  auto dB = eigmi::Matrix::upload(ctx, B);
  std::vector<double> xb(300), yb(300), rb(300, 0.0);
  for (auto &v : xb) v = nd(g);
  dB.mv_host(xb.data(), yb.data());
  for (auto r = B.begin(); r != B.end(); ++r)
    for (auto c = r->begin(); c != r->end(); ++c)
      for (int i = 0; i < 3; ++i)
      {
        double s = rb[r.index() * 3 + i];
        for (int j = 0; j < 3; ++j) s += (*c)[i][j] * xb[c.index() * 3 + j];
        rb[r.index() * 3 + i] = s;
      }
  EXPECT(std::memcmp(yb.data(), rb.data(), 300 * 8) == 0);

  // 2b) an external Lanczos loop on device BlockVectors: w = A v (eig_mv), alpha = v.w (eig_dot), then
  //     the fused update (eig_lanczos_update) and v <- w / beta -- against the same loop in host doubles
  {
    const std::size_t n = A.N();
    const int steps = 20;
    eigmi::DeviceVector dv(ctx, n), dp(ctx, n), dw(ctx, n), da(ctx, 1), db(ctx, 1), dr(ctx, 2);
    std::vector<double> v(n), p(n, 0.0), w(n), hv(n);
    double nv = 0.0;
    for (auto &e : v) e = nd(g), nv += e * e;
    for (auto &e : v) e /= std::sqrt(nv);
    dv.upload(v.data(), n);
    double beta = 0.0, worst = 0.0;
    for (int k = 0; k < steps; ++k)
    {
      // host reference: w = A v, alpha = v.w, w = (w - alpha v) - beta p, beta' = ||w||
      for (auto r = A.begin(); r != A.end(); ++r)
      {
        double s = 0.0;
        for (auto c = r->begin(); c != r->end(); ++c) s += (double)(*c) * v[c.index()];
        w[r.index()] = s;
      }
      double alpha = 0.0;
      for (std::size_t i = 0; i < n; ++i) alpha += v[i] * w[i];
      for (std::size_t i = 0; i < n; ++i) w[i] = (w[i] - alpha * v[i]) - (k ? beta * p[i] : 0.0);
      double bn = 0.0;
      for (double e : w) bn += e * e;
      bn = std::sqrt(bn);
      // device loop
      dA.mv(dv, dw);
      eigmi::check(eig_dot(ctx.get(), (int64_t)n, dv.data(), dw.data(), da.data()), ctx.get());
      eigmi::lanczos_update(ctx, da, k ? &db : nullptr, dv, k ? &dp : nullptr, dw, dr);
      double res[2], ga;
      dr.download(res, 2);
      da.download(&ga, 1);
      worst = std::max({worst, std::fabs(ga - alpha) / std::fabs(alpha), std::fabs(res[0] - bn) / bn,
                        std::fabs(res[1]) / bn});
      // next: p <- v, v <- w / beta'
      eigmi::check(eig_copy(ctx.get(), (int64_t)n, dv.data(), dp.data()), ctx.get());
      eigmi::check(eig_copy(ctx.get(), (int64_t)n, dw.data(), dv.data()), ctx.get());
      eigmi::check(eig_scal(ctx.get(), (int64_t)n, 1.0 / res[0], dv.data()), ctx.get());
      db.upload(&res[0], 1);
      p = v;
      for (std::size_t i = 0; i < n; ++i) v[i] = w[i] * (1.0 / bn);
      beta = bn;
    }
    std::printf("external Lanczos loop through eig_lanczos_update: %d steps, worst rel diff %.2e\n", steps, worst);
    EXPECT(worst < 1e-10);
  }

  // 3) ARPACK++ operator signature
  eigmi::ArpackOperator op(dA);
  EXPECT(op.nrows() == 4096 && op.ncols() == 4096);
  std::vector<double> w(4096);
  op.multMvB(x.data(), w.data());
  EXPECT(std::memcmp(w.data(), ref.data(), 4096 * 8) == 0);

  // 4) MultiVector kernels under the reference names
  const std::size_t n = A.N(), m = 16;
  MV8 Q(n, m), Y(n, m);
  for (auto &v : Q.p) v = nd(g);
  eigmi::matmul_sparse_tallskinny_blocked(Y, dA, Q);
  bool ok = true;
  for (std::size_t j = 0; j < m; ++j)
    for (auto r = A.begin(); r != A.end(); ++r)
    {
      double s = 0.0;
      for (auto c = r->begin(); c != r->end(); ++c) s += (double)(*c) * Q(c.index(), j);
      ok = ok && (s == Y(r.index(), j));
    }
  EXPECT(ok);
  eigmi::orthonormalize_blocked(ctx, Q);
  std::vector<std::vector<double>> G;
  eigmi::dot_products_all_blocked(ctx, G, Q, Q);
  double off = 0.0;
  for (std::size_t i = 0; i < m; ++i)
    for (std::size_t j = 0; j < m; ++j) off = std::max(off, std::fabs(G[i][j] - (i == j ? 1.0 : 0.0)));
  EXPECT(off < 1e-13);
  std::vector<double> dp;
  eigmi::dot_products_diagonal_blocked(ctx, dp, Q, Q);
  EXPECT(dp.size() == m && std::fabs(dp[3] - 1.0) < 1e-13);
  bool threw = false;
  try
  {
    MV8 bad1(n, 8), bad2(n + 1, 8);
    eigmi::dot_products_diagonal_blocked(ctx, dp, bad1, bad2);
  }
  catch (const std::invalid_argument &)
  {
    threw = true;
  }
  EXPECT(threw);

  // 5) StandardLargest: the reference run: 50 iterations, Ritz_0 7.9037
  std::vector<double> eval(4);
  std::vector<std::vector<double>> evec(4, std::vector<double>(n));
  int it = eigmi::StandardLargest(dA, 0.0, 2e-3, 4000, 4, eval, evec, 0, 123);
  EXPECT(it == 50);
  EXPECT(std::fabs(eval[0] - 7.9037) < 5e-5);

  // 6) UMFPackFactorizedMatrix role + matmul_inverse_tallskinny_blocked (kernels_cpp.hh:660-755)
  const int N16 = 16;
  auto A16 = laplace2d(N16);
  const std::size_t n16 = A16.N();
  auto F = eigmi::Factorization::from_istl(ctx, A16);
  EXPECT(F.size() == n16);
  MV8 R(n16, 8), Z(n16, 8), Rc(n16, 8);
  for (auto &v : R.p) v = nd(g);
  Rc = R;
  eigmi::matmul_inverse_tallskinny_blocked(Z, F, R);
  double res = 0.0;
  for (std::size_t j = 0; j < 8; ++j)
    for (auto r = A16.begin(); r != A16.end(); ++r)
    {
      double s = 0.0;
      for (auto c = r->begin(); c != r->end(); ++c) s += (double)(*c) * Z(c.index(), j);
      res = std::max(res, std::fabs(s - Rc(r.index(), j)));
    }
  EXPECT(res < 1e-11);
  {
    // the same factors through an object shaped like UMFPackFactorizedMatrix (IntType long)
    eigmi::Factorization Fh = eigmi::Factorization::from_istl(ctx, A16);
    int64_t nn = 0, lnz = 0, unz = 0;
    int rec = 0;
    eigmi::check(eig_lu_info(Fh.get(), &nn, &lnz, &unz, &rec), ctx.get());
    struct UMFLike {
      long n;
      std::vector<long> lp, lj, up, ui, pp, qq;
      std::vector<double> lx, ux, rs;
      long *Lp, *Lj, *Up, *Ui, *P, *Q;
      double *Lx, *Ux, *Rs;
      long do_recip;
    } u;
    std::vector<int64_t> Lp(nn + 1), Lj(lnz), Up(nn + 1), Ui(unz), P(nn), Q(nn);
    u.lx.resize(lnz);
    u.ux.resize(unz);
    u.rs.resize(nn);
    eigmi::check(eig_lu_export(Fh.get(), Lp.data(), Lj.data(), u.lx.data(), Up.data(), Ui.data(), u.ux.data(), P.data(),
                               Q.data(), u.rs.data()),
                 ctx.get());
    u.n = (long)nn;
    u.lp.assign(Lp.begin(), Lp.end());
    u.lj.assign(Lj.begin(), Lj.end());
    u.up.assign(Up.begin(), Up.end());
    u.ui.assign(Ui.begin(), Ui.end());
    u.pp.assign(P.begin(), P.end());
    u.qq.assign(Q.begin(), Q.end());
    u.Lp = u.lp.data();
    u.Lj = u.lj.data();
    u.Up = u.up.data();
    u.Ui = u.ui.data();
    u.P = u.pp.data();
    u.Q = u.qq.data();
    u.Lx = u.lx.data();
    u.Ux = u.ux.data();
    u.Rs = u.rs.data();
    u.do_recip = rec;
    auto Fu = eigmi::Factorization::from_umfpack(ctx, u);
    MV8 R2 = Rc, Z2(n16, 8);
    eigmi::matmul_inverse_tallskinny_blocked(Z2, Fu, R2);
    // (F's block-inverse image was built on the device from its band factors, Fu's on the host
    // from the exported arrays: the same factors, images that round differently)
    double zmax = 0.0, zd = 0.0;
    for (std::size_t q = 0; q < Z.p.size(); ++q)
    {
      zmax = std::max(zmax, std::fabs(Z.p[q]));
      zd = std::max(zd, std::fabs(Z2.p[q] - Z.p[q]));
    }
    EXPECT(zd <= 1e-13 * zmax);
  }
  bool threw2 = false;
  try
  {
    MV8 a(n16 + 1, 8), b(n16 + 1, 8);
    eigmi::matmul_inverse_tallskinny_blocked(a, F, b);
  }
  catch (const std::invalid_argument &)
  {
    threw2 = true;
  }
  EXPECT(threw2);

  // 7) StandardInverse / GeneralizedInverse: the smallest eigenvalues of the 2-D Dirichlet
  //    Laplacian (the reference's known answer, src/dune-eigensolver.cc:437-446)
  std::vector<double> exact;
  for (int i = 1; i <= N16; ++i)
    for (int j = 1; j <= N16; ++j)
    {
      const double h = M_PI / (N16 + 1);
      exact.push_back(4.0 * std::sin(i * h / 2) * std::sin(i * h / 2) + 4.0 * std::sin(j * h / 2) * std::sin(j * h / 2));
    }
  std::sort(exact.begin(), exact.end());
  {
    auto dA16 = eigmi::Matrix::upload(ctx, A16);
    std::vector<double> ev(4);
    std::vector<std::vector<double>> evv(4, std::vector<double>(n16));
    eigmi::StandardInverse(dA16, 0.0, 1e-12, 2000, 4, ev, evv);
    std::sort(ev.begin(), ev.end());
    for (int i = 0; i < 4; ++i) EXPECT(std::fabs(ev[i] - exact[i]) < 1e-8);
    // B = I on A's pattern
    TestBCRS<1, 1> I16 = A16;
    for (auto &row : I16.rows)
      for (std::size_t q = 0; q < row.size(); ++q) row[q].second.a[0][0] = (row[q].first == (std::size_t)(&row - &I16.rows[0])) ? 1.0 : 0.0;
    auto dI16 = eigmi::Matrix::upload(ctx, I16);
    std::vector<double> gv;
    std::vector<std::vector<double>> gvec;
    eigmi::GeneralizedInverse(dA16, dI16, 0.5, 0.0, 1e-13, 3000, 4, gv, gvec);
    EXPECT(gv.size() == 4 && gvec.size() == 4 && gvec[0].size() == n16);
    std::sort(gv.begin(), gv.end());
    for (int i = 0; i < 4; ++i) EXPECT(std::fabs(gv[i] - exact[i]) < 1e-8);

    // 8) ARPACK++-style shift-invert operator and computeGenSymShiftInvertMinMagnitude
    eigmi::ShiftInvertOperator sop(ctx, A16, dI16);  // sigma = 0: A - 0 B = A
    std::vector<double> v(n16), wv(n16), Av(n16);
    for (auto &e : v) e = nd(g);
    sop.multMv(v.data(), wv.data());
    dA16.mv_host(wv.data(), Av.data());
    double r2 = 0.0;
    for (std::size_t i = 0; i < n16; ++i) r2 = std::max(r2, std::fabs(Av[i] - v[i]));
    EXPECT(r2 < 1e-11);
    std::vector<std::vector<std::array<double, 1>>> xs(4, std::vector<std::array<double, 1>>(n16));
    std::vector<double> lam(4);
    eigmi::computeGenSymShiftInvertMinMagnitude(dA16, dI16, 1e-14, xs, lam, 0.0);
    for (int i = 0; i < 4; ++i) EXPECT(std::fabs(lam[i] - exact[i]) < 1e-10);
    // 9) the adaptive variant (every eigenvalue below a threshold between exact[2] and exact[3]) and
    // the non-symmetric modes on the same (symmetric) pencil
    std::vector<std::vector<std::array<double, 1>>> xa(8);
    std::vector<double> la;
    eigmi::computeGenSymShiftInvertMinMagnitudeAdaptive(dA16, dI16, 1e-14, 0.5 * (exact[2] + exact[3]), xa, la, 0.0, 2);
    EXPECT(la.size() >= 3 && xa.size() == la.size() && xa[0].size() == n16);
    for (int i = 0; i < 3 && i < (int)la.size(); ++i) EXPECT(std::fabs(la[i] - exact[i]) < 1e-10);
    for (int mode = 0; mode < 2; ++mode)
    {
      std::vector<double> ln(4);
      if (mode == 0) eigmi::computeStdNonSymMinMagnitude(dA16, dI16, 1e-13, xs, ln, 0.0);
      else eigmi::computeGenNonSymShiftInvertMinMagnitude(dA16, dI16, 1e-13, xs, ln, 0.0);
      // a one-vector Krylov space holds ONE vector of a multiple eigenspace in exact arithmetic (the
      // Laplacian's lambda_2 = lambda_3); the second copy enters through rounding alone (in ARPACK
      // too), so only the simple leading values and membership in the spectrum are required
      EXPECT(std::fabs(ln[0] - exact[0]) < 1e-10 && std::fabs(ln[1] - exact[1]) < 1e-10);
      for (int i = 0; i < 4; ++i)
      {
        double dmin = 1e300;
        for (double e : exact) dmin = std::min(dmin, std::fabs(ln[i] - e));
        EXPECT(dmin < 1e-10);
      }
    }
  }

  std::printf(failures ? "FAILED %d\n" : "ALL OK\n", failures);
  return failures ? 1 : 0;
}
