// oracle/oracle.cc -- CPU restatement of the dune-eigensolver hot path.
//
// TEST INFRASTRUCTURE ONLY.  Nothing in the product (dune-eigensolver_amd/, include/) links,
// loads or calls this file.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg use it, as the checker / the reported CPU baseline.
//
// Every function restates the reference algorithm in the reference's loop order, citing the
// file:line it follows (paths relative to the reference checkout).  Build flags are
// `-O2 -ffp-contract=off` so that `a += b*c` rounds the product and the sum separately, exactly
// like the reference's portable kernels (kernels_cpp.hh) compiled without FMA contraction.
//
// Parity pinning (see DESIGN.md "Oracle"): the reference itself is unbuildable in this image
// (its kernels need dune-istl / dune-common / SuiteSparse declarations that are absent), so this
// restatement is pinned by the reference's own known-answer test -- the analytic 2-D Dirichlet
// spectrum of src/dune-eigensolver.cc:437-446 -- and by ARPACK (scipy-bundled, the reference's
// Krylov driver dependency) fixtures committed under tests/golden/.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

typedef int64_t i64;
typedef int32_t i32;

static inline i64 mvidx(i64 n, i64 i, i64 j) { return ((j / 8) * n + i) * 8 + (j % 8); }

extern "C" {

// ------------------------------------------------------------------------------------------
// Matrix generators (a15).  dune-istl's setupLaplacian (used at src/dune-eigensolver.cc:98-103)
// builds the 2-D 5-point pattern row-wise with lexicographic k = y*N + x, columns in ascending
// order {k-N, k-1, k, k+1, k+N}, diagonal 4 and off-diagonal -1 (Dirichlet nodes eliminated).
// ------------------------------------------------------------------------------------------
i64 orc_laplace2d_nnz(int N) { return (i64)5 * N * N - 4 * (i64)N; }

void orc_laplace2d(int N, i64 *rowptr, i32 *col, double *val)
{
  i64 p = 0;
  for (i64 k = 0; k < (i64)N * N; ++k)
  {
    rowptr[k] = p;
    int x = (int)(k % N), y = (int)(k / N);
    if (y > 0) { col[p] = (i32)(k - N); val[p++] = -1.0; }
    if (x > 0) { col[p] = (i32)(k - 1); val[p++] = -1.0; }
    col[p] = (i32)k; val[p++] = 4.0;
    if (x < N - 1) { col[p] = (i32)(k + 1); val[p++] = -1.0; }
    if (y < N - 1) { col[p] = (i32)(k + N); val[p++] = -1.0; }
  }
  rowptr[(i64)N * N] = p;
}

// get_laplacian_neumann (src/dune-eigensolver.cc:105-121): diagonal := |sum of off-diagonals|.
void orc_laplace2d_neumann(int N, i64 *rowptr, i32 *col, double *val)
{
  orc_laplace2d(N, rowptr, col, val);
  for (i64 k = 0; k < (i64)N * N; ++k)
  {
    double s = 0.0;
    i64 d = -1;
    for (i64 p = rowptr[k]; p < rowptr[k + 1]; ++p)
      if (col[p] == k) d = p; else s += val[p];
    val[d] = std::fabs(s);
  }
}

// get_laplacian_B (src/dune-eigensolver.cc:124-143): partition-of-unity mask pu[k] = 0 within
// `overlap` of the boundary, 1 inside; a_kl *= pu[k]*pu[l].
void orc_laplace2d_pu(int N, int overlap, i64 *rowptr, i32 *col, double *val)
{
  orc_laplace2d(N, rowptr, col, val);
  std::vector<double> pu((size_t)N * N);
  for (i64 k = 0; k < (i64)N * N; ++k)
  {
    int i = (int)(k / N), j = (int)(k % N);
    pu[k] = (i < overlap || i > N - 1 - overlap || j < overlap || j > N - 1 - overlap) ? 0.0 : 1.0;
  }
  for (i64 k = 0; k < (i64)N * N; ++k)
    for (i64 p = rowptr[k]; p < rowptr[k + 1]; ++p)
      val[p] *= pu[k] * pu[col[p]];
}

// get_identity (src/dune-eigensolver.cc:145-156): Laplacian pattern, values I.
void orc_identity2d(int N, i64 *rowptr, i32 *col, double *val)
{
  orc_laplace2d(N, rowptr, col, val);
  for (i64 k = 0; k < (i64)N * N; ++k)
    for (i64 p = rowptr[k]; p < rowptr[k + 1]; ++p)
      val[p] = (col[p] == k) ? 1.0 : 0.0;
}

// 3-D 7-point Poisson (configs C2/C4): k = (z*N + y)*N + x, sorted columns,
// diagonal 6, off-diagonal -1.  Same construction rule as setupLaplacian, one dimension up.
i64 orc_poisson3d_nnz(int N) { return (i64)7 * N * N * N - (i64)6 * N * N; }

void orc_poisson3d(int N, i64 *rowptr, i32 *col, double *val)
{
  const i64 NN = (i64)N * N, n = NN * N;
  i64 p = 0;
  for (i64 k = 0; k < n; ++k)
  {
    rowptr[k] = p;
    int x = (int)(k % N), y = (int)((k / N) % N), z = (int)(k / NN);
    if (z > 0) { col[p] = (i32)(k - NN); val[p++] = -1.0; }
    if (y > 0) { col[p] = (i32)(k - N); val[p++] = -1.0; }
    if (x > 0) { col[p] = (i32)(k - 1); val[p++] = -1.0; }
    col[p] = (i32)k; val[p++] = 6.0;
    if (x < N - 1) { col[p] = (i32)(k + 1); val[p++] = -1.0; }
    if (y < N - 1) { col[p] = (i32)(k + N); val[p++] = -1.0; }
    if (z < N - 1) { col[p] = (i32)(k + NN); val[p++] = -1.0; }
  }
  rowptr[n] = p;
}

// Config C3: 3x3-block "elasticity" known-answer matrix A = L_Q1 (x) C on N^3 interior nodes.
// L_Q1 = K(x)M(x)M + M(x)K(x)M + M(x)M(x)K with 1-D P1 matrices K = tridiag(-1,2,-1) and
// M = tridiag(1,4,1)/6 (h = 1), C = [[2,1,0],[1,2,1],[0,1,2]].  Block (p,q) = L_pq * C, stored
// row-major (FieldMatrix<double,3,3> layout), block columns sorted.  27-point block pattern.
i64 orc_q1elast_nnzb(int N) { i64 t = 3 * (i64)N - 2; return t * t * t; }

static double k1(int d) { return d == 0 ? 2.0 : -1.0; }
static double m1(int d) { return d == 0 ? 4.0 / 6.0 : 1.0 / 6.0; }

void orc_q1elast(int N, i64 *rowptr, i32 *col, double *val)
{
  const double C[9] = {2, 1, 0, 1, 2, 1, 0, 1, 2};
  const i64 NN = (i64)N * N, nb = NN * N;
  i64 p = 0;
  for (i64 k = 0; k < nb; ++k)
  {
    rowptr[k] = p;
    int x = (int)(k % N), y = (int)((k / N) % N), z = (int)(k / NN);
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx)
        {
          int xx = x + dx, yy = y + dy, zz = z + dz;
          if (xx < 0 || yy < 0 || zz < 0 || xx >= N || yy >= N || zz >= N) continue;
          int ax = std::abs(dx), ay = std::abs(dy), az = std::abs(dz);
          double l = k1(ax) * m1(ay) * m1(az) + m1(ax) * k1(ay) * m1(az) + m1(ax) * m1(ay) * k1(az);
          col[p] = (i32)((zz * (i64)N + yy) * N + xx);
          for (int t = 0; t < 9; ++t) val[p * 9 + t] = l * C[t];
          ++p;
        }
  }
  rowptr[nb] = p;
}

// Analytic eigenvalues of the 2-D Dirichlet 5-point Laplacian, sorted ascending:
// src/dune-eigensolver.cc:437-446 (lambda_ij = 4(sin^2(i pi h/2) + sin^2(j pi h/2)), h=1/(N+1)).
void orc_eig_laplace2d(int N, double *ev)
{
  const double h = 1.0 / (N + 1.0);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j)
    {
      double si = std::sin(0.5 * h * (i + 1) * M_PI), sj = std::sin(0.5 * h * (j + 1) * M_PI);
      ev[(size_t)j * N + i] = 4.0 * (si * si + sj * sj);
    }
  std::sort(ev, ev + (size_t)N * N);
}

// ------------------------------------------------------------------------------------------
// Sparse products
// ------------------------------------------------------------------------------------------

// a3 / BCRSMatrix::mv for 1x1 blocks: y_i = sum over the row in stored (ascending) order,
// starting from 0.0 (kernels_cpp.hh:596-621 inner loop; arpack_geneo_wrapper.hh:269-279).
void orc_csr_mv(i64 n, const i64 *rowptr, const i32 *col, const double *val, const double *x, double *y)
{
  for (i64 i = 0; i < n; ++i)
  {
    double s = 0.0;
    for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
      s += val[p] * x[col[p]];
    y[i] = s;
  }
}

// a4: BCRSMatrix<FieldMatrix<double,br,bc>>::mv.  Blocks row-major; per block row, per
// component r the sum runs over the row's blocks in order and inside a block over c.
void orc_bcsr_mv(i64 nb, int br, int bc, const i64 *rowptr, const i32 *col, const double *val,
                 const double *x, double *y)
{
  for (i64 I = 0; I < nb; ++I)
  {
    for (int r = 0; r < br; ++r)
      y[I * br + r] = 0.0;
    for (i64 p = rowptr[I]; p < rowptr[I + 1]; ++p)
    {
      const double *a = val + p * br * bc;
      const double *xx = x + (i64)col[p] * bc;
      for (int r = 0; r < br; ++r)
      {
        double s = y[I * br + r];
        for (int c = 0; c < bc; ++c)
          s += a[r * bc + c] * xx[c];
        y[I * br + r] = s;
      }
    }
  }
}

// a2: matmul_sparse_tallskinny_blocked (kernels_cpp.hh:626-657) on MultiVector<double,8>.
void orc_spmm_mv8(i64 n, i64 m, const i64 *rowptr, const i32 *col, const double *val,
                  const double *Qin, double *Qout)
{
  for (i64 bj = 0; bj < m; bj += 8)
  {
    const double *pin = Qin + n * bj;
    double *pout = Qout + n * bj;
    for (i64 i = 0; i < n; ++i)
    {
      double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
      {
        const double a = val[p];
        const double *xr = pin + (i64)col[p] * 8;
        for (int j = 0; j < 8; ++j) s[j] += a * xr[j];
      }
      for (int j = 0; j < 8; ++j) pout[i * 8 + j] = s[j];
    }
  }
}

// ------------------------------------------------------------------------------------------
// Dot products on MultiVector<double,8>
// ------------------------------------------------------------------------------------------

// a5: dot_products_diagonal_blocked (kernels_cpp.hh:24-55).
void orc_dot_diag_mv8(i64 n, i64 m, const double *Q1, const double *Q2, double *dp)
{
  for (i64 bj = 0; bj < m; bj += 8)
  {
    double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const double *a = Q1 + n * bj, *b = Q2 + n * bj;
    for (i64 i = 0; i < n; ++i)
      for (int j = 0; j < 8; ++j) s[j] += a[i * 8 + j] * b[i * 8 + j];
    for (int j = 0; j < 8; ++j) dp[bj + j] = s[j];
  }
}

// a6: dot_products_all_blocked (kernels_cpp.hh:58-96).  G is m x m row-major, G[j1][j2] = q1_j1 . q2_j2.
void orc_gram_mv8(i64 n, i64 m, const double *Q1, const double *Q2, double *G)
{
  for (i64 b1 = 0; b1 < m; b1 += 8)
    for (i64 b2 = 0; b2 < m; b2 += 8)
    {
      double s[8][8];
      std::memset(s, 0, sizeof s);
      const double *a = Q1 + n * b1, *b = Q2 + n * b2;
      for (i64 i = 0; i < n; ++i)
        for (int j1 = 0; j1 < 8; ++j1)
          for (int j2 = 0; j2 < 8; ++j2) s[j1][j2] += a[i * 8 + j1] * b[i * 8 + j2];
      for (int j1 = 0; j1 < 8; ++j1)
        for (int j2 = 0; j2 < 8; ++j2) G[(b1 + j1) * m + b2 + j2] = s[j1][j2];
    }
}

// ------------------------------------------------------------------------------------------
// Orthonormalisation
// ------------------------------------------------------------------------------------------

// a8: orthonormalize_naive (kernels_cpp.hh:121-155), column-major (MultiVector<double,1>).
void orc_orthonormalize_naive(i64 n, i64 m, double *q)
{
  for (i64 k = 0; k < m; ++k)
  {
    double *qk = q + k * n;
    double s = 0.0;
    for (i64 i = 0; i < n; ++i) s += qk[i] * qk[i];
    s = 1.0 / std::sqrt(s);
    for (i64 i = 0; i < n; ++i) qk[i] *= s;
    for (i64 j = k + 1; j < m; ++j)
    {
      double *qj = q + j * n;
      double d = 0.0;
      for (i64 i = 0; i < n; ++i) d += qk[i] * qj[i];
      for (i64 i = 0; i < n; ++i) qj[i] -= d * qk[i];
    }
  }
}

// Project the blocks after bk against block bk: S = Q_bk^T Q_bj, Q_bj -= Q_bk S
// (kernels_cpp.hh:309-349; same order of products as the reference: rows outer, k, j).
static void project_later_blocks(i64 n, i64 m, double *q, i64 bk)
{
  for (i64 bj = bk + 8; bj < m; bj += 8)
  {
    double s[8][8];
    std::memset(s, 0, sizeof s);
    const double *qk = q + n * bk;
    double *qj = q + n * bj;
    for (i64 i = 0; i < n; ++i)
      for (int k = 0; k < 8; ++k)
        for (int j = 0; j < 8; ++j) s[k][j] += qk[i * 8 + k] * qj[i * 8 + j];
    for (i64 i = 0; i < n; ++i)
      for (int k = 0; k < 8; ++k)
        for (int j = 0; j < 8; ++j) qj[i * 8 + j] -= s[k][j] * qk[i * 8 + k];
  }
}

// a9: orthonormalize_blocked (kernels_cpp.hh:180-351), the live `if(true)` branch:
// diagonal block by column MGS (:202-229), then single-pass block CGS of later blocks.
void orc_orthonormalize_mv8(i64 n, i64 m, double *q)
{
  for (i64 bk = 0; bk < m; bk += 8)
  {
    double *qb = q + n * bk;
    double s[8][8];
    std::memset(s, 0, sizeof s);
    for (int k = 0; k < 8; ++k)
    {
      for (i64 i = 0; i < n; ++i)
        for (int j = k; j < 8; ++j) s[k][j] += qb[i * 8 + k] * qb[i * 8 + j];
      for (int j = k + 1; j < 8; ++j) s[k][j] /= s[k][k];
      s[k][k] = 1.0 / std::sqrt(s[k][k]);
      for (i64 i = 0; i < n; ++i)
      {
        for (int j = k + 1; j < 8; ++j) qb[i * 8 + j] -= s[k][j] * qb[i * 8 + k];
        qb[i * 8 + k] *= s[k][k];
      }
    }
    project_later_blocks(n, m, q, bk);
  }
}

// Shared CholQR factor used by the AVX2/NEON diagonal block and by B-orthonormalisation:
// LU without pivoting of the symmetric Gram s, D = diag(U)^-1/2, U := L^-T D (upper
// triangular) (kernels_avx2.hh:185-252 == kernels_cpp.hh:474-526).
static void cholqr_factor(const double s[8][8], double U[8][8])
{
  double LU[8][8];
  std::memcpy(LU, s, sizeof LU);
  for (int k = 0; k < 8; ++k)
    for (int i = k + 1; i < 8; ++i)
    {
      LU[i][k] /= LU[k][k];
      for (int j = k + 1; j < 8; ++j) LU[i][j] -= LU[i][k] * LU[k][j];
    }
  double D[8];
  for (int i = 0; i < 8; ++i) D[i] = 1.0 / std::sqrt(LU[i][i]);
  for (int i = 0; i < 8; ++i)
  {
    LU[i][i] = 1.0;
    for (int j = i + 1; j < 8; ++j) LU[i][j] = 0.0;
  }
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) U[i][j] = (i == j) ? 1.0 : 0.0;
  for (int i = 1; i < 8; ++i)
    for (int j = 0; j < i; ++j)
      for (int k = 0; k < 8; ++k) U[i][k] -= LU[i][j] * U[j][k];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < i; ++j) std::swap(U[i][j], U[j][i]);
  for (int i = 0; i < 8; ++i)
    for (int j = i; j < 8; ++j) U[i][j] *= D[j];
}

// v_i := v_i U for an upper-triangular U, in place, j descending (kernels_cpp.hh:556-568).
static void apply_upper(i64 n, double *v, const double U[8][8])
{
  for (i64 i = 0; i < n; ++i)
  {
    double *vi = v + i * 8;
    for (int j = 7; j >= 0; --j)
    {
      double sum = 0.0;
      for (int k = 0; k <= j; ++k) sum += vi[k] * U[k][j];
      vi[j] = sum;
    }
  }
}

// a10: orthonormalize_avx2_b8_v2 / orthonormalize_neon_b8_v2 semantics (kernels_avx2.hh:385-622):
// diagonal block by CholQR on the full 8x8 Gram, then a single 8x8 projection per later block.
// (The SIMD versions use FMA; this restatement rounds products and sums separately.)
void orc_orthonormalize_cholqr_mv8(i64 n, i64 m, double *q)
{
  for (i64 bk = 0; bk < m; bk += 8)
  {
    double *qb = q + n * bk;
    double s[8][8], U[8][8];
    std::memset(s, 0, sizeof s);
    for (i64 i = 0; i < n; ++i)
      for (int k = 0; k < 8; ++k)
        for (int j = 0; j < 8; ++j) s[k][j] += qb[i * 8 + k] * qb[i * 8 + j];
    cholqr_factor(s, U);
    apply_upper(n, qb, U);
    project_later_blocks(n, m, q, bk);
  }
}

// a10, split-half order: orthonormalize_avx2_b8 (kernels_avx2.hh:64-381): the same CholQR of the
// diagonal block, but every later block is projected in two halves -- S1 = Q_bk[:, 0:4]^T Q_bj,
// Q_bj -= Q_bk[:, 0:4] S1, then S2 = Q_bk[:, 4:8]^T Q_bj (the UPDATED block), Q_bj -= Q_bk[:, 4:8] S2
// (:255-381).  (FMA in the SIMD code; separately rounded here.)
void orc_orthonormalize_cholqr_split_mv8(i64 n, i64 m, double *q)
{
  for (i64 bk = 0; bk < m; bk += 8)
  {
    double *qb = q + n * bk;
    double s[8][8], U[8][8];
    std::memset(s, 0, sizeof s);
    for (i64 i = 0; i < n; ++i)
      for (int k = 0; k < 8; ++k)
        for (int j = 0; j < 8; ++j) s[k][j] += qb[i * 8 + k] * qb[i * 8 + j];
    cholqr_factor(s, U);
    apply_upper(n, qb, U);
    for (i64 bj = bk + 8; bj < m; bj += 8)
    {
      double *qj = q + n * bj;
      for (int h = 0; h < 8; h += 4)
      {
        double S[4][8];
        std::memset(S, 0, sizeof S);
        for (i64 i = 0; i < n; ++i)
          for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 8; ++j) S[k][j] += qb[i * 8 + h + k] * qj[i * 8 + j];
        for (i64 i = 0; i < n; ++i)
          for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 8; ++j) qj[i * 8 + j] -= S[k][j] * qb[i * 8 + h + k];
      }
    }
  }
}

// a11: B_orthonormalize_blocked (kernels_cpp.hh:356-591); returns max off-diagonal "R" entry.
double orc_b_orthonormalize_mv8(i64 n, i64 m, const i64 *rowptr, const i32 *col, const double *val, double *q)
{
  double norm = 0.0;
  std::vector<double> p((size_t)n * 8);
  for (i64 bk = 0; bk < m; bk += 8)
  {
    double *qb = q + n * bk;
    // P = B * Q_bk (:378-395)
    for (i64 i = 0; i < n; ++i)
    {
      double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (i64 k = rowptr[i]; k < rowptr[i + 1]; ++k)
        for (int j = 0; j < 8; ++j) s[j] += val[k] * qb[(i64)col[k] * 8 + j];
      for (int j = 0; j < 8; ++j) p[i * 8 + j] = s[j];
    }
    // upper triangle of P^T Q_bk, mirrored (:450-466)
    double s[8][8], U[8][8];
    std::memset(s, 0, sizeof s);
    for (i64 i = 0; i < n; ++i)
      for (int k = 0; k < 8; ++k)
        for (int j = k; j < 8; ++j) s[k][j] += p[i * 8 + k] * qb[i * 8 + j];
    for (int k = 0; k < 8; ++k)
      for (int j = 0; j < k; ++j) s[k][j] = s[j][k];
    for (int k = 0; k < 8; ++k)
      for (int j = k + 1; j < 8; ++j) norm = std::max(norm, s[k][j]);
    cholqr_factor(s, U);
    apply_upper(n, qb, U);
    apply_upper(n, p.data(), U);
    // later blocks: S = P^T Q_bj, Q_bj -= Q_bk S (:543-584)
    for (i64 bj = bk + 8; bj < m; bj += 8)
    {
      double S[8][8];
      std::memset(S, 0, sizeof S);
      double *qj = q + n * bj;
      for (i64 i = 0; i < n; ++i)
        for (int k = 0; k < 8; ++k)
          for (int j = 0; j < 8; ++j) S[k][j] += p[i * 8 + k] * qj[i * 8 + j];
      for (int k = 0; k < 8; ++k)
        for (int j = 0; j < 8; ++j) norm = std::max(norm, S[k][j]);
      for (i64 i = 0; i < n; ++i)
        for (int k = 0; k < 8; ++k)
          for (int j = 0; j < 8; ++j) qj[i * 8 + j] -= S[k][j] * qb[i * 8 + k];
    }
  }
  return norm;
}

// a14: the reference's analytic flop / byte models (kernels_cpp.hh:98-116, :157-175).
double orc_flops_orthonormalize(int n, int m)
{
  double f = 0.0;
  for (int k = m; k > 0; k--) f += 2.0 * n + n + (k - 1) * 4.0 * n;
  return f;
}
double orc_bytes_orthonormalize_naive(int n, int m)
{
  double c = 0.0;
  for (int k = m; k > 0; k--) c += n + 2.0 * n + (k - 1) * (2.0 * n + 3.0 * n);
  return c * 8;
}
double orc_bytes_orthonormalize_blocked(int n, int m, int b)
{
  double c = 0.0;
  for (int bk = 0; bk < m; bk += b)
  {
    for (int k = b; k > 0; k--) c += (double)n * k + (double)n * (1 + (k - 1) + 1);
    for (int bj = bk + b; bj < m; bj += b) c += 5.0 * b * n;
  }
  return c * 8;
}

// ------------------------------------------------------------------------------------------
// Start block and subspace iteration
// ------------------------------------------------------------------------------------------

// eigensolver.hh:49-55: mt19937(seed) + normal_distribution(0,1), fill order (block, row, col).
void orc_random_mv8(i64 n, i64 m, unsigned seed, double *q)
{
  std::mt19937 urbg{seed};
  std::normal_distribution<double> gen{0.0, 1.0};
  for (i64 bj = 0; bj < m; bj += 8)
    for (i64 i = 0; i < n; ++i)
      for (int j = 0; j < 8; ++j) q[mvidx(n, i, bj + j)] = gen(urbg);
}

// Same generator, plain vector (Lanczos start vector).
void orc_random_vec(i64 n, unsigned seed, double *x)
{
  std::mt19937 urbg{seed};
  std::normal_distribution<double> gen{0.0, 1.0};
  for (i64 i = 0; i < n; ++i) x[i] = gen(urbg);
}

// a13: A += shift*I on the diagonal (eigensolver.hh:59-66), 1x1 blocks.
void orc_shift_diag(i64 n, const i64 *rowptr, const i32 *col, double *val, double shift)
{
  for (i64 i = 0; i < n; ++i)
    for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
      if (col[p] == i) val[p] += shift;
}

// a12: StandardLargest (eigensolver.hh:28-112) for 1x1 blocks.  Mutates val when shift != 0,
// like the reference.  eval[nev], evec[nev*n] (vector j contiguous).  Returns iterations (k at exit).
int orc_standard_largest(i64 n, const i64 *rowptr, const i32 *col, double *val, double shift, double tol,
                         int maxiter, int nev, unsigned seed, double *eval, double *evec)
{
  const i64 m = (nev / 8 + std::min(nev % 8, 1)) * 8;
  std::vector<double> Q1((size_t)(n * m)), Q2((size_t)(n * m));
  orc_random_mv8(n, m, seed, Q1.data());
  if (shift != 0.0) orc_shift_diag(n, rowptr, col, val, shift);
  orc_orthonormalize_mv8(n, m, Q1.data());
  std::vector<double> s1(m, 0.0), s2(m, 0.0);
  int kk = 1;
  for (i64 k = 1; k < maxiter; ++k)
  {
    kk = (int)k;
    orc_spmm_mv8(n, m, rowptr, col, val, Q1.data(), Q2.data());
    orc_orthonormalize_mv8(n, m, Q2.data());
    orc_spmm_mv8(n, m, rowptr, col, val, Q2.data(), Q1.data());
    orc_dot_diag_mv8(n, m, Q2.data(), Q1.data(), s1.data());
    for (auto &x : s1) x -= shift;
    double dist = 0.0;
    for (i64 i = 0; i < m; ++i) dist = std::max(dist, std::fabs(s1[i] - s2[i]));
    std::swap(s1, s2);
    std::swap(Q1, Q2);
    if (k > 1 && dist < tol) break;
  }
  for (int j = 0; j < nev; ++j) eval[j] = s2[j];
  for (int j = 0; j < nev; ++j)
    for (i64 i = 0; i < n; ++i) evec[(i64)j * n + i] = Q1[mvidx(n, i, j)];
  return kk;
}

// ------------------------------------------------------------------------------------------
// Inverse subspace iteration: the exported-LU-factor apply and the two
// inverse drivers.  The factors are inputs (UMFPackFactorizedMatrix's public arrays,
// umfpacktools.hh:20-39); whoever computed them, the reference's arithmetic on them is this.
// ------------------------------------------------------------------------------------------

// matmul_inverse_tallskinny_blocked (kernels_cpp.hh:660-755), verbatim loop structure.  Qin is
// overwritten.  L rows: Lp/Lj/Lx with the unit diagonal last; U columns: Up/Ui/Ux with the
// diagonal last.
void orc_inverse_mv8(i64 n, i64 m, const i64 *Lp, const i64 *Lj, const double *Lx, const i64 *Up, const i64 *Ui,
                     const double *Ux, const i64 *P, const i64 *Q, const double *Rs, int do_recip, double *pin,
                     double *pout)
{
  const int bs = 8;
  for (i64 bj = 0; bj < m; bj += bs)
  {
    const i64 nbj = n * bj;
    {  // combined row scaling and permutation (:680-705)
      i64 K = nbj;
      for (i64 k = 0; k < n; ++k)
      {
        const double scaling = do_recip ? Rs[P[k]] : 1.0 / Rs[P[k]];
        const i64 I = nbj + P[k] * bs;
        for (int s = 0; s < bs; ++s) pout[K + s] = scaling * pin[I + s];
        K += bs;
      }
    }
    {  // L (:710-725)
      i64 I = nbj;
      double sum[8];
      for (i64 i = 0; i < n; i++)
      {
        for (int s = 0; s < bs; ++s) sum[s] = pout[I + s];
        for (i64 k = Lp[i]; k < Lp[i + 1] - 1; k++)
        {
          const i64 J = nbj + Lj[k] * bs;
          const double lij = Lx[k];
          for (int s = 0; s < bs; ++s) sum[s] -= lij * pin[J + s];
        }
        for (int s = 0; s < bs; ++s) pin[I + s] = sum[s];
        I += bs;
      }
    }
    {  // U (:727-750)
      i64 J = nbj + (n - 1) * bs;
      double result[8];
      for (i64 j = n - 1; j >= 0; j--)
      {
        double matelem = Ux[Up[j + 1] - 1];
        for (int s = 0; s < bs; ++s) result[s] = pin[J + s] / matelem;
        for (i64 k = Up[j]; k < Up[j + 1] - 1; k++)
        {
          const i64 I = nbj + Ui[k] * bs;
          matelem = Ux[k];
          for (int s = 0; s < bs; ++s) pin[I + s] -= matelem * result[s];
        }
        const i64 K = nbj + Q[j] * bs;
        for (int s = 0; s < bs; ++s) pout[K + s] = result[s];
        J -= bs;
      }
    }
  }
}

// StandardInverse (eigensolver.hh:116-198), 1x1 blocks; val is mutated by the shift like the
// reference; the factors are those of the SHIFTED matrix.  Returns the iterations (k at exit).
int orc_standard_inverse(i64 n, const i64 *rowptr, const i32 *col, double *val, const i64 *Lp, const i64 *Lj,
                         const double *Lx, const i64 *Up, const i64 *Ui, const double *Ux, const i64 *P, const i64 *Q,
                         const double *Rs, int do_recip, double shift, double tol, int maxiter, int nev, unsigned seed,
                         double *eval, double *evec)
{
  const i64 m = (nev / 8 + std::min(nev % 8, 1)) * 8;
  std::vector<double> Q1((size_t)(n * m)), Q2((size_t)(n * m));
  orc_random_mv8(n, m, seed, Q1.data());
  if (shift != 0.0) orc_shift_diag(n, rowptr, col, val, shift);
  orc_orthonormalize_mv8(n, m, Q1.data());
  std::vector<double> s1(m, 0.0), s2(m, 0.0);
  int kk = 1;
  for (i64 k = 1; k < maxiter; ++k)
  {
    kk = (int)k;
    orc_inverse_mv8(n, m, Lp, Lj, Lx, Up, Ui, Ux, P, Q, Rs, do_recip, Q1.data(), Q2.data());  // :168
    orc_orthonormalize_mv8(n, m, Q2.data());                                                 // :171
    orc_spmm_mv8(n, m, rowptr, col, val, Q2.data(), Q1.data());                              // :174
    orc_dot_diag_mv8(n, m, Q2.data(), Q1.data(), s1.data());                                 // :175
    for (auto &x : s1) x -= shift;
    double dist = 0.0;
    for (i64 i = 0; i < m; ++i) dist = std::max(dist, std::fabs(s1[i] - s2[i]));
    std::swap(s1, s2);
    std::swap(Q1, Q2);
    if (k > 1 && dist < tol) break;
  }
  for (int j = 0; j < nev; ++j) eval[j] = s2[j];
  for (int j = 0; j < nev; ++j)
    for (i64 i = 0; i < n; ++i) evec[(i64)j * n + i] = Q1[mvidx(n, i, j)];
  return kk;
}

// GeneralizedInverse (eigensolver.hh:204-351), portable-kernel branch (:268-275, :290-304): A is
// copied and shifted A + shift B + reg I on A's pattern (pattern(B) within pattern(A), :202-203);
// the factors are those of that shifted copy.  Returns the iterations.
int orc_generalized_inverse(i64 n, const i64 *rowptr, const i32 *col, const double *valA, const i64 *browptr,
                            const i32 *bcol, const double *valB, const i64 *Lp, const i64 *Lj, const double *Lx,
                            const i64 *Up, const i64 *Ui, const double *Ux, const i64 *P, const i64 *Q,
                            const double *Rs, int do_recip, double shift, double reg, double tol, int maxiter, int nev,
                            unsigned seed, double *eval, double *evec)
{
  std::vector<double> A(valA, valA + rowptr[n]);
  for (i64 i = 0; i < n; ++i)
  {
    if (shift != 0.0)
      for (i64 q = browptr[i]; q < browptr[i + 1]; ++q)
        for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
          if (col[p] == bcol[q]) A[p] += shift * valB[q];  // A.axpy(shift, B) (:241)
    if (reg != 0.0)
      for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
        if (col[p] == i) A[p] += reg;  // (:244-252)
  }
  const i64 m = (nev / 8 + std::min(nev % 8, 1)) * 8;
  std::vector<double> Q1((size_t)(n * m)), Q2((size_t)(n * m));
  orc_random_mv8(n, m, seed, Q1.data());
  std::vector<double> ra1(m, 0.0), ra2(m, 0.0), sA(m, 0.0);
  orc_b_orthonormalize_mv8(n, m, browptr, bcol, valB, Q1.data());  // :273
  orc_spmm_mv8(n, m, rowptr, col, A.data(), Q1.data(), Q2.data());
  orc_dot_diag_mv8(n, m, Q2.data(), Q1.data(), sA.data());
  for (i64 i = 0; i < m; ++i) ra2[i] = sA[i] - shift;
  int iter = 0;
  while (iter < maxiter)
  {
    orc_spmm_mv8(n, m, browptr, bcol, valB, Q1.data(), Q2.data());                            // :302
    orc_inverse_mv8(n, m, Lp, Lj, Lx, Up, Ui, Ux, P, Q, Rs, do_recip, Q2.data(), Q1.data());  // :303
    orc_b_orthonormalize_mv8(n, m, browptr, bcol, valB, Q1.data());                            // :304
    iter += 1;
    orc_spmm_mv8(n, m, rowptr, col, A.data(), Q1.data(), Q2.data());  // :317
    orc_dot_diag_mv8(n, m, Q2.data(), Q1.data(), sA.data());
    for (i64 i = 0; i < m; ++i) ra1[i] = sA[i] - shift;
    double relerror = 0.0;
    for (i64 i = 0; i < m; ++i) relerror = std::max(relerror, std::fabs(ra1[i] - ra2[i]));
    relerror /= *std::max_element(ra1.begin(), ra1.end());
    std::swap(ra1, ra2);
    if ((iter > 10) & (relerror < tol)) break;
  }
  for (int j = 0; j < nev; ++j) eval[j] = ra2[j];
  for (int j = 0; j < nev; ++j)
    for (i64 i = 0; i < n; ++i) evec[(i64)j * n + i] = Q1[mvidx(n, i, j)];
  return iter;
}

// ------------------------------------------------------------------------------------------
// Lanczos three-term recurrence -- the arithmetic ARPACK's dsaupd performs between the
// multMv callbacks (arpack_geneo_wrapper.hh:257-279; ARPACK dsaitr), written in the exact
// operation order of the device path (DESIGN.md "Lanczos step") so the two can be compared:
//   t      = (A u_j) * sig_j - gam_j * u_{j-1}        gam_j = beta_j * sig_{j-1}
//   alpha_j = sig_j * (t . u_j)
//   u_{j+1} = t - (alpha_j * sig_j) * u_j
//   beta_{j+1} = ||u_{j+1}||,  sig_{j+1} = 1 / beta_{j+1}
// Vectors are kept unnormalised (v_j = u_j * sig_j).  U holds k+1 vectors of length n;
// U[0] is the start vector.  alpha[k], beta[k+1] (beta[0] = ||u_0||).
// ------------------------------------------------------------------------------------------
void orc_lanczos(i64 n, const i64 *rowptr, const i32 *col, const double *val, int k, double *U,
                 double *alpha, double *beta)
{
  double s = 0.0;
  for (i64 i = 0; i < n; ++i) s += U[i] * U[i];
  beta[0] = std::sqrt(s);
  double sig_prev = 0.0, sig = 1.0 / beta[0];
  for (int j = 0; j < k; ++j)
  {
    const double *u = U + (i64)j * n;
    const double *up = j > 0 ? U + (i64)(j - 1) * n : nullptr;
    double *t = U + (i64)(j + 1) * n;
    const double gam = j > 0 ? beta[j] * sig_prev : 0.0;
    double d = 0.0;
    for (i64 i = 0; i < n; ++i)
    {
      double acc = 0.0;
      for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p) acc += val[p] * u[col[p]];
      double ti = acc * sig;
      if (up) ti = ti - gam * up[i];
      t[i] = ti;
      d += ti * u[i];
    }
    const double a = sig * d;
    alpha[j] = a;
    const double as = a * sig;
    double nn = 0.0;
    for (i64 i = 0; i < n; ++i)
    {
      double ui = t[i] - as * u[i];
      t[i] = ui;
      nn += ui * ui;
    }
    beta[j + 1] = std::sqrt(nn);
    sig_prev = sig;
    sig = 1.0 / beta[j + 1];
  }
}

// CPU baseline kernel: `steps` Lanczos steps over three rotating vectors (no basis kept).
// This is the reference CPU path's Lanczos step (a3 SpMV + the BLAS-1 loops ARPACK runs).
void orc_lanczos_rotating(i64 n, const i64 *rowptr, const i32 *col, const double *val, int steps,
                          double *u0, double *u1, double *u2, double *alpha, double *beta)
{
  double *U[3] = {u0, u1, u2};
  double s = 0.0;
  for (i64 i = 0; i < n; ++i) s += u0[i] * u0[i];
  beta[0] = std::sqrt(s);
  double sig_prev = 0.0, sig = 1.0 / beta[0];
  for (int j = 0; j < steps; ++j)
  {
    const double *u = U[j % 3];
    const double *up = U[(j + 2) % 3];
    double *t = U[(j + 1) % 3];
    const double gam = j > 0 ? beta[j] * sig_prev : 0.0;
    double d = 0.0;
    for (i64 i = 0; i < n; ++i)
    {
      double acc = 0.0;
      for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p) acc += val[p] * u[col[p]];
      double ti = acc * sig;
      if (j > 0) ti = ti - gam * up[i];
      t[i] = ti;
      d += ti * u[i];
    }
    const double a = sig * d;
    alpha[j] = a;
    const double as = a * sig;
    double nn = 0.0;
    for (i64 i = 0; i < n; ++i)
    {
      double ui = t[i] - as * u[i];
      t[i] = ui;
      nn += ui * ui;
    }
    beta[j + 1] = std::sqrt(nn);
    sig_prev = sig;
    sig = 1.0 / beta[j + 1];
  }
}

// One-reduction fused Lanczos step, the restatement of the GPU's fused step (k_lanczos_fused_b1 /
// k_lanczos_fused_march, fused_begin in k_spmv.hip).  The same Krylov process as
// orc_lanczos: u_k = t_{k-1} - c u_{k-1} is formed right before the SpMV that needs it, and its
// squared norm is PREDICTED from the previous step's reductions, nt_k = tsq - c dsum with
// c = dsum / m (m = the measured ||u_{k-1}||^2), so a step needs one reduction of (dsum, tsq, m).
// Guard: the step runs on A - mu I (mu = trace / n; alpha reported unshifted), and a launch whose
// prediction keeps no more than kTau of tsq REPAIRS instead of stepping (u_k formed explicitly,
// its exact norm reduced; the next launch takes step k with c = 0 and that norm).  The final beta
// is always exact (a forced repair, as eig_lanczos_tridiag does).  Launch by launch, every scalar
// formula is written exactly as the kernel prologue evaluates it.
static const double kTau = 1e-2;
enum { kStep = 0, kPost = 1, kHalt = 2, kRepair = 3 };

// pipe = false: orc_lanczos_fused; pipe = true: orc_lanczos_pipelined (below).
static void lanczos_onered(i64 n, const i64 *rowptr, const i32 *col, const double *val, int steps, const double *u0,
                           double *alpha, double *beta, int *launches_out, bool pipe)
{
  double dsum = 0.0;
  for (i64 i = 0; i < n; ++i)
    for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p)
      if (col[p] == i) dsum += val[p];
  const double mu = dsum / (double)n;
  std::vector<double> T(u0, u0 + n), U(n, 0.0), Tn(n), Un(n), ux(n), Z(n, 0.0), S(n);
  std::vector<double> nsum(steps + 2, 0.0);
  double s0 = 0.0;
  for (i64 i = 0; i < n; ++i) s0 += u0[i] * u0[i];
  nsum[0] = s0;
  double red[3] = {0.0, 0.0, 0.0}, aux[2] = {0.0, 0.0};
  int j = 0, mode = kStep, L = 0;
  auto launch = [&](bool force) {
    if (pipe)  // S = A t_{k-1}: needs no scalar of the previous launch (issued before its allreduce)
      for (i64 i = 0; i < n; ++i)
      {
        double acc = 0.0;
        for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p) acc += val[p] * T[col[p]];
        S[i] = acc;
      }
    double c = 0.0, nt = 1.0, ap = 0.0, bk = 0.0, gam = 0.0, rn = 0.0, rm = 0.0;
    int act;
    if (mode == kPost)
    {
      const double mex = red[2];
      rn = aux[0];
      rm = aux[1];
      nt = mex;
      if (!(mex > 0.0)) act = kHalt;
      else
      {
        bk = std::sqrt(mex) * rn / rm;
        gam = bk / rm;
        act = kPost;
      }
    }
    else if (j == 0)
    {
      nt = nsum[0];
      act = kStep;
    }
    else
    {
      const double d = red[0], q = red[1], m = red[2];
      rn = std::sqrt(nsum[j - 1]);
      rm = std::sqrt(m);
      c = d / m;
      ap = c * rn + mu;
      nt = q - c * d;
      if (force || !(nt > kTau * q)) act = kRepair;
      else
      {
        bk = std::sqrt(nt) * rn / rm;
        gam = bk / rm;
        act = kStep;
      }
    }
    const double sig = 1.0 / std::sqrt(nt);
    ++L;
    if (act == kHalt)
    {
      nsum[j] = 0.0;
      beta[j] = 0.0;
      mode = kHalt;
      return;
    }
    if (act == kRepair)
    {
      alpha[j - 1] = ap;
      aux[0] = rn;
      aux[1] = rm;
      double m2 = 0.0;
      for (i64 i = 0; i < n; ++i)
      {
        const double u = T[i] - c * U[i];
        T[i] = u;  // pairs (u_j, u_{j-1})
        m2 += u * u;
      }
      red[0] = red[1] = 0.0;
      red[2] = m2;
      mode = kPost;
      return;
    }
    if (act == kPost)
    {
      nsum[j] = nt;
      beta[j] = bk;
    }
    else if (j > 0)
    {
      nsum[j] = nt;
      alpha[j - 1] = ap;
      beta[j] = bk;
    }
    else
      beta[0] = std::sqrt(nt);
    for (i64 i = 0; i < n; ++i) ux[i] = T[i] - c * U[i];
    double d = 0.0, q = 0.0, m = 0.0;
    for (i64 i = 0; i < n; ++i)
    {
      double acc = 0.0;
      if (pipe)
      {
        acc = S[i] - c * Z[i];  // z_k = A u_k = A t_{k-1} - c A u_{k-1}
        Z[i] = acc;
      }
      else
        for (i64 p = rowptr[i]; p < rowptr[i + 1]; ++p) acc += val[p] * ux[col[p]];
      double ti = (acc - mu * ux[i]) * sig;
      if (j > 0) ti = ti - gam * U[i];
      Tn[i] = ti;
      Un[i] = ux[i];
      d += ti * ux[i];
      q += ti * ti;
      m += ux[i] * ux[i];
    }
    red[0] = d;
    red[1] = q;
    red[2] = m;
    std::swap(T, Tn);
    std::swap(U, Un);
    ++j;
    mode = kStep;
  };
  beta[0] = std::sqrt(s0);
  while (j < steps && mode != kHalt) launch(false);
  if (mode == kStep && j > 0) launch(true);  // exact final beta (eig_lanczos_tridiag)
  if (mode == kPost)
  {
    const double mex = red[2];
    nsum[j] = mex;
    beta[j] = mex > 0.0 ? std::sqrt(mex) * aux[0] / aux[1] : 0.0;
  }
  if (launches_out) *launches_out = L;
}

void orc_lanczos_fused(i64 n, const i64 *rowptr, const i32 *col, const double *val, int steps, const double *u0,
                       double *alpha, double *beta, int *launches_out)
{
  lanczos_onered(n, rowptr, col, val, steps, u0, alpha, beta, launches_out, false);
}

// Pipelined one-reduction step, the restatement of the GPU's pipelined step (k_lanczos_pipe in
// k_spmv.hip): the same scalars, modes and repairs as orc_lanczos_fused, but the SpMV of
// a launch multiplies t_{k-1} -- a vector that does not depend on the previous launch's reductions,
// so on N GPUs it overlaps that launch's allreduce -- and A u_k is recovered by the recurrence
// z_k = A t_{k-1} - c z_{k-1} (z_{k-1} = A u_{k-1}, carried per row).  A repair keeps Z; the launch
// after it has c = 0, so z = A u_k exactly.
void orc_lanczos_pipelined(i64 n, const i64 *rowptr, const i32 *col, const double *val, int steps, const double *u0,
                           double *alpha, double *beta, int *launches_out)
{
  lanczos_onered(n, rowptr, col, val, steps, u0, alpha, beta, launches_out, true);
}

} // extern "C"
