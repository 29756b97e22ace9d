// dense.cpp -- small dense host linear algebra of the Krylov drivers: the tridiagonal QL
// eigensolver (Lanczos), Householder reduction of a dense symmetric matrix (block Lanczos'
// block-tridiagonal T), Cholesky and triangular inverse (CholQR of 8..32-column blocks).
#include <algorithm>
#include <cmath>
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
          for (int q = 0; q < k; ++q)
          {
            f = Z[(size_t)q * k + i + 1];
            Z[(size_t)q * k + i + 1] = s * Z[(size_t)q * k + i] + c * f;
            Z[(size_t)q * k + i] = c * Z[(size_t)q * k + i] - s * f;
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
  std::vector<double> d2(k), Z2((size_t)k * k);
  for (int j = 0; j < k; ++j)
  {
    d2[j] = d[idx[j]];
    for (int q = 0; q < k; ++q) Z2[(size_t)q * k + j] = Z[(size_t)q * k + idx[j]];
  }
  d.swap(d2);
  Z.swap(Z2);
}


// ---------------------------------------------------------------------------------------------
// Householder reduction A = Q T Q^T of a dense symmetric n x n matrix (row-major; only the
// symmetric values are used).  d, e receive T's diagonal / sub-diagonal, Q (row-major) the
// accumulated reflectors.  Reflector k: v zeroes A[k+2.., k]; the trailing block is updated as
// A <- A - v w^T - w v^T with p = tau A v, w = p - (tau/2)(v^T p) v, tau = 2 / v^T v.
// ---------------------------------------------------------------------------------------------
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
    for (int i = 0; i < m; ++i)
    {
      double s = 0.0;
      const double *row = &A[(size_t)(k + 1 + i) * n + k + 1];
      for (int j = 0; j < m; ++j) s += row[j] * v[j];
      p[i] = tau * s;
    }
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
      double s = 0.0;
      for (int j = 0; j < m; ++j) s += qr[j] * v[j];
      s *= tau;
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

}  // namespace eigmi
