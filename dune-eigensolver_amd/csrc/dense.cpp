// dense.cpp -- small dense host linear algebra of the Krylov drivers: the tridiagonal QL
// eigensolver (Lanczos), Householder reduction of a dense symmetric matrix (block Lanczos'
// block-tridiagonal T), Cholesky and triangular inverse (CholQR of 8..32-column blocks), and the
// general real eigenproblem of the Arnoldi drivers' projected matrix (Hessenberg reduction, the
// Francis double-shift QR, inverse-iteration eigenvectors).
#include <algorithm>
#include <cmath>
#include <complex>
#include <numeric>
#include <vector>

#include "internal.h"

namespace eigmi {

// ---------------------------------------------------------------------------------------------
// Symmetric tridiagonal eigenproblem (implicit QL with Wilkinson shifts).  d[k] diagonal,
// e[k-1] off-diagonal; on return d holds the eigenvalues (ascending) and Z (k x k, column j =
// eigenvector j, row-major Z[i*k + j]).  z_identity = false: Z already holds an orthogonal Q
// (A = Q T Q^T, from householder_tridiag) and receives the eigenvectors of A.
// ---------------------------------------------------------------------------------------------
void tridiag_eig(int k, std::vector<double> &d, std::vector<double> e, std::vector<double> &Z, bool z_identity)
{
  if (z_identity)
  {
    Z.assign((size_t)k * k, 0.0);
    for (int i = 0; i < k; ++i) Z[(size_t)i * k + i] = 1.0;
  }
  e.resize(k, 0.0);
  if (k > 0) e[k - 1] = 0.0;
  // the rotations act on pairs of columns of Z: work on Zt = Z^T (row i of Zt = column i of Z), so
  // each rotation updates two contiguous rows (the column-strided form was cache-bound at k ~ 100)
  std::vector<double> Zt((size_t)k * k);
  for (int q = 0; q < k; ++q)
    for (int i = 0; i < k; ++i) Zt[(size_t)i * k + q] = Z[(size_t)q * k + i];
  const double eps = 2.220446049250313e-16;
  for (int l = 0; l < k; ++l)
  {
    int iter = 0, m;
    do
    {
      for (m = l; m < k - 1; ++m)
      {
        const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
        if (std::fabs(e[m]) <= eps * dd) break;
      }
      if (m != l)
      {
        if (iter++ == 100) throw Error(EIG_ERR_BREAKDOWN, "tridiagonal QL did not converge");
        double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
        double r = std::hypot(g, 1.0);
        g = d[m] - d[l] + e[l] / (g + std::copysign(r, g));
        double s = 1.0, c = 1.0, p = 0.0;
        int i;
        for (i = m - 1; i >= l; --i)
        {
          double f = s * e[i], b = c * e[i];
          e[i + 1] = (r = std::hypot(f, g));
          if (r == 0.0)
          {
            d[i + 1] -= p;
            e[m] = 0.0;
            break;
          }
          s = f / r;
          c = g / r;
          g = d[i + 1] - p;
          r = (d[i] - g) * s + 2.0 * c * b;
          d[i + 1] = g + (p = s * r);
          g = c * r - b;
          double *__restrict__ zi = &Zt[(size_t)i * k], *__restrict__ zi1 = &Zt[(size_t)(i + 1) * k];
          for (int q = 0; q < k; ++q)
          {
            const double fz = zi1[q];
            zi1[q] = s * zi[q] + c * fz;
            zi[q] = c * zi[q] - s * fz;
          }
        }
        if (r == 0.0 && i >= l) continue;
        d[l] -= p;
        e[l] = g;
        e[m] = 0.0;
      }
    } while (m != l);
  }
  // sort ascending with vectors
  std::vector<int> idx(k);
  std::iota(idx.begin(), idx.end(), 0);
  std::sort(idx.begin(), idx.end(), [&](int a, int b) { return d[a] < d[b]; });
  std::vector<double> d2(k);
  for (int j = 0; j < k; ++j)
  {
    d2[j] = d[idx[j]];
    const double *zc = &Zt[(size_t)idx[j] * k];
    for (int q = 0; q < k; ++q) Z[(size_t)q * k + j] = zc[q];
  }
  d.swap(d2);
}


// ---------------------------------------------------------------------------------------------
// Householder reduction A = Q T Q^T of a dense symmetric n x n matrix (row-major; only the
// symmetric values are used).  d, e receive T's diagonal / sub-diagonal, Q (row-major) the
// accumulated reflectors.  Reflector k: v zeroes A[k+2.., k]; the trailing block is updated as
// A <- A - v w^T - w v^T with p = tau A v, w = p - (tau/2)(v^T p) v, tau = 2 / v^T v.
// ---------------------------------------------------------------------------------------------
namespace {
// sum_j a[j] b[j] with 4 independent partial sums (vectorisable; the strict-order single
// accumulator kept these O(n^3) loops scalar)
inline double dot4(const double *a, const double *b, int m)
{
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int j = 0;
  for (; j + 4 <= m; j += 4)
  {
    s0 += a[j] * b[j];
    s1 += a[j + 1] * b[j + 1];
    s2 += a[j + 2] * b[j + 2];
    s3 += a[j + 3] * b[j + 3];
  }
  for (; j < m; ++j) s0 += a[j] * b[j];
  return (s0 + s1) + (s2 + s3);
}
}  // namespace

void householder_tridiag(int n, std::vector<double> A, std::vector<double> &d, std::vector<double> &e,
                         std::vector<double> &Q)
{
  Q.assign((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i) Q[(size_t)i * n + i] = 1.0;
  d.assign(n, 0.0);
  e.assign(n > 0 ? n - 1 : 0, 0.0);
  std::vector<double> v(n), p(n), w(n);
  auto a = [&](int i, int j) -> double & { return A[(size_t)i * n + j]; };
  for (int k = 0; k + 2 < n; ++k)
  {
    const int m = n - k - 1;  // length of the column below the diagonal
    double norm2 = 0.0;
    for (int i = 0; i < m; ++i) norm2 += a(k + 1 + i, k) * a(k + 1 + i, k);
    const double x0 = a(k + 1, k);
    const double alpha = (x0 >= 0.0 ? -1.0 : 1.0) * std::sqrt(norm2);
    double vv = 0.0;
    for (int i = 0; i < m; ++i) v[i] = a(k + 1 + i, k);
    v[0] -= alpha;
    for (int i = 0; i < m; ++i) vv += v[i] * v[i];
    if (vv == 0.0) continue;  // column already reduced
    const double tau = 2.0 / vv;
    for (int i = 0; i < m; ++i) p[i] = tau * dot4(&A[(size_t)(k + 1 + i) * n + k + 1], v.data(), m);
    double vp = 0.0;
    for (int i = 0; i < m; ++i) vp += v[i] * p[i];
    for (int i = 0; i < m; ++i) w[i] = p[i] - 0.5 * tau * vp * v[i];
    for (int i = 0; i < m; ++i)
    {
      double *row = &A[(size_t)(k + 1 + i) * n + k + 1];
      for (int j = 0; j < m; ++j) row[j] -= v[i] * w[j] + w[i] * v[j];
    }
    a(k + 1, k) = alpha;
    a(k, k + 1) = alpha;
    for (int i = 1; i < m; ++i) a(k + 1 + i, k) = a(k, k + 1 + i) = 0.0;
    // Q <- Q H on columns k+1..n-1
    for (int r = 0; r < n; ++r)
    {
      double *qr = &Q[(size_t)r * n + k + 1];
      const double s = tau * dot4(qr, v.data(), m);
      for (int j = 0; j < m; ++j) qr[j] -= s * v[j];
    }
  }
  for (int i = 0; i < n; ++i) d[i] = a(i, i);
  for (int i = 0; i + 1 < n; ++i) e[i] = a(i + 1, i);
}

void sym_eig(int n, const std::vector<double> &A, std::vector<double> &w, std::vector<double> &Z)
{
  std::vector<double> e;
  householder_tridiag(n, A, w, e, Z);
  tridiag_eig(n, w, e, Z, false);
}

// G = R^T R with R upper triangular (row-major n x n); false on a non-positive pivot.
bool chol_upper(int n, const double *G, double *R)
{
  std::fill(R, R + (size_t)n * n, 0.0);
  for (int j = 0; j < n; ++j)
  {
    double s = G[(size_t)j * n + j];
    for (int k = 0; k < j; ++k) s -= R[(size_t)k * n + j] * R[(size_t)k * n + j];
    if (!(s > 0.0)) return false;
    const double rjj = std::sqrt(s);
    R[(size_t)j * n + j] = rjj;
    for (int i = j + 1; i < n; ++i)
    {
      double t = G[(size_t)j * n + i];
      for (int k = 0; k < j; ++k) t -= R[(size_t)k * n + j] * R[(size_t)k * n + i];
      R[(size_t)j * n + i] = t / rjj;
    }
  }
  return true;
}

// Rinv = R^{-1} for upper triangular R (row-major), column by column back substitution.
void tri_upper_inv(int n, const double *R, double *Rinv)
{
  std::fill(Rinv, Rinv + (size_t)n * n, 0.0);
  for (int c = 0; c < n; ++c)
  {
    for (int i = c; i >= 0; --i)
    {
      double s = (i == c) ? 1.0 : 0.0;
      for (int k = i + 1; k <= c; ++k) s -= R[(size_t)i * n + k] * Rinv[(size_t)k * n + c];
      Rinv[(size_t)i * n + c] = s / R[(size_t)i * n + i];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// General real eigenproblem of the Arnoldi drivers' m x m projected matrix (m <= a few hundred).
// Eigenvalues: Gaussian-elimination reduction to upper Hessenberg form (a similarity with row
// pivoting), then the Francis double-shift QR iteration (the EISPACK hqr algorithm: deflation on
// negligible subdiagonals, exceptional shifts at iterations 10 and 20).  Eigenvectors: two steps of
// inverse iteration with the ORIGINAL matrix in complex arithmetic (LU with partial pivoting; a
// zero pivot is replaced by eps ||G||), unit 2-norm, phase such that the largest entry is real.
// ---------------------------------------------------------------------------------------------
namespace {

void hess_reduce(int n, std::vector<double> &a)  // row-major, in place; entries below the subdiagonal zeroed
{
  auto A = [&](int i, int j) -> double & { return a[(size_t)i * n + j]; };
  for (int m = 1; m < n - 1; ++m)
  {
    double x = 0.0;
    int piv = m;
    for (int j = m; j < n; ++j)
      if (std::fabs(A(j, m - 1)) > std::fabs(x))
      {
        x = A(j, m - 1);
        piv = j;
      }
    if (piv != m)
    {
      for (int j = m - 1; j < n; ++j) std::swap(A(piv, j), A(m, j));
      for (int j = 0; j < n; ++j) std::swap(A(j, piv), A(j, m));
    }
    if (x != 0.0)
      for (int i = m + 1; i < n; ++i)
      {
        double y = A(i, m - 1);
        if (y == 0.0) continue;
        y /= x;
        A(i, m - 1) = y;
        for (int j = m; j < n; ++j) A(i, j) -= y * A(m, j);
        for (int j = 0; j < n; ++j) A(j, m) += y * A(j, i);
      }
  }
  for (int i = 2; i < n; ++i)
    for (int j = 0; j < i - 1; ++j) A(i, j) = 0.0;
}

// Eigenvalues of the upper Hessenberg matrix a (destroyed).  False when an eigenvalue needed more
// than 60 iterations.
bool hess_eigvals(int n, std::vector<double> &a, std::vector<std::complex<double>> &w)
{
  // 1-based accessor (the algorithm's natural indexing)
  auto A = [&](int i, int j) -> double & { return a[(size_t)(i - 1) * n + (j - 1)]; };
  auto sgn = [](double x, double y) { return y >= 0.0 ? std::fabs(x) : -std::fabs(x); };
  w.assign(n, {0.0, 0.0});
  double anorm = 0.0;
  for (int i = 1; i <= n; ++i)
    for (int j = std::max(i - 1, 1); j <= n; ++j) anorm += std::fabs(A(i, j));
  int nn = n, l = 1;
  double t = 0.0, x, y, z, wv, p = 0, q = 0, r = 0, s, u, v;
  while (nn >= 1)
  {
    int its = 0;
    do
    {
      for (l = nn; l >= 2; --l)
      {
        s = std::fabs(A(l - 1, l - 1)) + std::fabs(A(l, l));
        if (s == 0.0) s = anorm;
        if (std::fabs(A(l, l - 1)) + s == s)
        {
          A(l, l - 1) = 0.0;
          break;
        }
      }
      x = A(nn, nn);
      if (l == nn)
      {
        w[nn - 1] = {x + t, 0.0};
        --nn;
      }
      else
      {
        y = A(nn - 1, nn - 1);
        wv = A(nn, nn - 1) * A(nn - 1, nn);
        if (l == nn - 1)
        {
          p = 0.5 * (y - x);
          q = p * p + wv;
          z = std::sqrt(std::fabs(q));
          x += t;
          if (q >= 0.0)
          {
            z = p + sgn(z, p);
            const double a2 = x + z, a1 = z != 0.0 ? x - wv / z : x + z;
            w[nn - 2] = {a2, 0.0};
            w[nn - 1] = {a1, 0.0};
          }
          else
          {
            w[nn - 2] = {x + p, -z};
            w[nn - 1] = {x + p, z};
          }
          nn -= 2;
        }
        else
        {
          if (its == 60) return false;
          if (its == 10 || its == 20)
          {
            t += x;
            for (int i = 1; i <= nn; ++i) A(i, i) -= x;
            s = std::fabs(A(nn, nn - 1)) + std::fabs(A(nn - 1, nn - 2));
            y = x = 0.75 * s;
            wv = -0.4375 * s * s;
          }
          ++its;
          int m;
          for (m = nn - 2; m >= l; --m)
          {
            z = A(m, m);
            r = x - z;
            s = y - z;
            p = (r * s - wv) / A(m + 1, m) + A(m, m + 1);
            q = A(m + 1, m + 1) - z - r - s;
            r = A(m + 2, m + 1);
            s = std::fabs(p) + std::fabs(q) + std::fabs(r);
            p /= s;
            q /= s;
            r /= s;
            if (m == l) break;
            u = std::fabs(A(m, m - 1)) * (std::fabs(q) + std::fabs(r));
            v = std::fabs(p) * (std::fabs(A(m - 1, m - 1)) + std::fabs(z) + std::fabs(A(m + 1, m + 1)));
            if (u + v == v) break;
          }
          for (int i = m + 2; i <= nn; ++i)
          {
            A(i, i - 2) = 0.0;
            if (i != m + 2) A(i, i - 3) = 0.0;
          }
          for (int k = m; k <= nn - 1; ++k)
          {
            if (k != m)
            {
              p = A(k, k - 1);
              q = A(k + 1, k - 1);
              r = 0.0;
              if (k != nn - 1) r = A(k + 2, k - 1);
              if ((x = std::fabs(p) + std::fabs(q) + std::fabs(r)) != 0.0)
              {
                p /= x;
                q /= x;
                r /= x;
              }
            }
            if ((s = sgn(std::sqrt(p * p + q * q + r * r), p)) != 0.0)
            {
              if (k == m)
              {
                if (l != m) A(k, k - 1) = -A(k, k - 1);
              }
              else
                A(k, k - 1) = -s * x;
              p += s;
              x = p / s;
              y = q / s;
              z = r / s;
              q /= p;
              r /= p;
              for (int j = k; j <= nn; ++j)
              {
                p = A(k, j) + q * A(k + 1, j);
                if (k != nn - 1)
                {
                  p += r * A(k + 2, j);
                  A(k + 2, j) -= p * z;
                }
                A(k + 1, j) -= p * y;
                A(k, j) -= p * x;
              }
              const int mmin = nn < k + 3 ? nn : k + 3;
              for (int i = l; i <= mmin; ++i)
              {
                p = x * A(i, k) + y * A(i, k + 1);
                if (k != nn - 1)
                {
                  p += z * A(i, k + 2);
                  A(i, k + 2) -= p * r;
                }
                A(i, k + 1) -= p * q;
                A(i, k) -= p;
              }
            }
          }
        }
      }
    } while (l < nn - 1);
  }
  return true;
}

// Eigenvector of the real matrix g (row-major n x n) for the eigenvalue theta, orthogonal to the
// vectors `defl` (eigenvectors already found for the same eigenvalue: a multiple eigenvalue gets
// independent vectors of its eigenspace -- otherwise inverse iteration returns the same vector each
// time and the Krylov-Schur restart basis would not span an invariant subspace).
void inverse_iteration(int n, const std::vector<double> &g, std::complex<double> theta,
                       std::vector<std::complex<double>> &y,
                       const std::vector<const std::vector<std::complex<double>> *> &defl = {})
{
  typedef std::complex<double> C;
  double gn = 0.0;
  for (double v : g) gn = std::max(gn, std::fabs(v));
  const double tiny = std::max(gn, 1e-300) * 2.220446049250313e-16;
  std::vector<C> M((size_t)n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) M[(size_t)i * n + j] = g[(size_t)i * n + j] - (i == j ? theta : C(0.0));
  std::vector<int> piv(n);
  for (int k = 0; k < n; ++k)
  {
    int pk = k;
    for (int i = k + 1; i < n; ++i)
      if (std::abs(M[(size_t)i * n + k]) > std::abs(M[(size_t)pk * n + k])) pk = i;
    piv[k] = pk;
    if (pk != k)
      for (int j = 0; j < n; ++j) std::swap(M[(size_t)k * n + j], M[(size_t)pk * n + j]);
    if (std::abs(M[(size_t)k * n + k]) < tiny) M[(size_t)k * n + k] = tiny;
    const C d = M[(size_t)k * n + k];
    for (int i = k + 1; i < n; ++i)
    {
      const C f = M[(size_t)i * n + k] / d;
      M[(size_t)i * n + k] = f;
      if (f != C(0.0))
        for (int j = k + 1; j < n; ++j) M[(size_t)i * n + j] -= f * M[(size_t)k * n + j];
    }
  }
  y.assign(n, C(1.0));
  for (int i = 0; i < n; ++i) y[i] += C(0.0, 1e-3 * (i % 7));  // generic start (not orthogonal to any vector)
  for (int it = 0; it < 3; ++it)
  {
    for (int k = 0; k < n; ++k)
      if (piv[k] != k) std::swap(y[k], y[piv[k]]);
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < i; ++k) y[i] -= M[(size_t)i * n + k] * y[k];
    for (int i = n - 1; i >= 0; --i)
    {
      for (int k = i + 1; k < n; ++k) y[i] -= M[(size_t)i * n + k] * y[k];
      y[i] /= M[(size_t)i * n + i];
    }
    for (int pass = 0; pass < 2; ++pass)
      for (const auto *x : defl)
      {
        C d = 0.0;
        for (int i = 0; i < n; ++i) d += std::conj((*x)[i]) * y[i];
        for (int i = 0; i < n; ++i) y[i] -= d * (*x)[i];
      }
    double nrm = 0.0;
    int big = 0;
    for (int i = 0; i < n; ++i)
    {
      nrm += std::norm(y[i]);
      if (std::abs(y[i]) > std::abs(y[big])) big = i;
    }
    const C ph = std::abs(y[big]) > 0.0 ? std::conj(y[big]) / std::abs(y[big]) : C(1.0);
    nrm = std::sqrt(nrm);
    for (auto &v : y) v = v * ph / nrm;
  }
}

}  // namespace

bool gen_eig(int n, const std::vector<double> &g, std::vector<std::complex<double>> &w,
             std::vector<std::complex<double>> &Y)
{
  std::vector<double> h = g;
  hess_reduce(n, h);
  if (!hess_eigvals(n, h, w)) return false;
  Y.assign((size_t)n * n, 0.0);
  double wmax = 0.0;
  for (const auto &v : w) wmax = std::max(wmax, std::abs(v));
  std::vector<std::vector<std::complex<double>>> found(n);
  for (int j = 0; j < n; ++j)
  {
    if (j > 0 && w[j].imag() != 0.0 && w[j] == std::conj(w[j - 1]))
    {
      found[j].resize(n);
      for (int i = 0; i < n; ++i) found[j][i] = Y[(size_t)i * n + j] = std::conj(Y[(size_t)i * n + j - 1]);
      continue;
    }
    // the vectors of (numerically) the same eigenvalue found so far
    std::vector<const std::vector<std::complex<double>> *> defl;
    for (int i = 0; i < j; ++i)
      if (std::abs(w[i] - w[j]) <= 1e-10 * wmax) defl.push_back(&found[i]);
    inverse_iteration(n, g, w[j], found[j], defl);
    for (int i = 0; i < n; ++i) Y[(size_t)i * n + j] = found[j][i];
  }
  return true;
}

}  // namespace eigmi
