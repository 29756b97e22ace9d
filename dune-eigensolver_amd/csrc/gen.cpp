// gen.cpp -- synthetic matrices of the reference harness (src/dune-eigensolver.cc:98-156) and of
// SURVEY 8(d), generated row by row on the host so that a rank can build only its own rows.
//
//   kind 0  2-D Dirichlet 5-point, N*N rows, dune-istl setupLaplacian semantics: k = y N + x,
//           columns ascending {k-N, k-1, k, k+1, k+N}, diagonal 4, off-diagonal -1
//   kind 1  2-D Neumann: diagonal := |sum of off-diagonals|           (.cc:105-121)
//   kind 2  2-D partition-of-unity B: a_kl *= pu_k pu_l               (.cc:124-143)
//   kind 3  2-D identity values on the Laplacian pattern              (.cc:145-156)
//   kind 4  3-D 7-point Poisson, N^3 rows, diagonal 6                  (configs C2 / C4)
//   kind 5  3-D Q1 "elasticity" L_Q1 (x) C on N^3 nodes, 3x3 blocks     (config C3)
//   kind 6  3-D P1 stiffness K on the Kuhn 6-tetrahedra split of the unit cube, N^3 interior
//           nodes, h = 1/(N+1), Dirichlet nodes eliminated, 15-point edge pattern   (config C5)
//   kind 7  3-D P1 consistent mass M on the same mesh and the SAME 15-point pattern (config C5;
//           the reference assumes pattern(A) contains pattern(B), eigensolver.hh:202-203)
//   kind 9, 10  the P1 K / M of kinds 6 / 7 with a coefficient c_e in [0.5, 1.5) per tetrahedron
//           (hashed; contributions summed in element order: bitwise symmetric) -- config C5's
//           variable-coefficient realism variant (no two rows alike: the box-image kernels run)
//   kind 8  3-D 7-point variable-coefficient diffusion (finite volumes, Dirichlet): the 7-point
//           pattern of kind 4 with a positive conductance kappa(e) in [0.5, 1.5) per grid edge e
//           (a hash of the edge, so a(k, q) = a(q, k) = -kappa bit for bit) and the diagonal
//           the sum of the six face conductances (boundary faces included): SPD, no two rows equal
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <utility>

#include "../../include/eigmi.h"

namespace {

typedef int64_t i64;

inline double k1(int d) { return d == 0 ? 2.0 : -1.0; }
inline double m1(int d) { return d == 0 ? 4.0 / 6.0 : 1.0 / 6.0; }

// P1 on the Kuhn split: the cube with lower corner c is cut into 6 tetrahedra, one per axis
// permutation p: v0 = c, v1 = v0 + e_p0, v2 = v1 + e_p1, v3 = c + (1,1,1).  Barycentric gradients
// are -e_p0, e_p0 - e_p1, e_p1 - e_p2, e_p2 (over h), so every element stiffness is the path
// Laplacian (h/6) [1 -1 0 0; -1 2 -1 0; 0 -1 2 -1; 0 0 -1 1] and every element mass is
// (h^3/120)(1 + delta_ab).  Edges are +-e_i, +-(e_i + e_j), +-(1,1,1): 14 neighbours + self.
const int kPerm[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
inline double kappa(i64 k, int a, int side);
// variable coefficients (kinds 9 / 10): element e = (cube corner, tetrahedron) scales its stiffness /
// mass by c_e in [0.5, 1.5) (a hash of e); an entry's element contributions are summed in ascending
// element order, so a(k, q) and a(q, k) round identically (bitwise symmetric)
int gen_p1_row(bool mass, int N, i64 k, int32_t *cols, double *vals, bool var = false)
{
  const i64 NN = (i64)N * N;
  const int P[3] = {(int)(k % N) + 1, (int)((k / N) % N) + 1, (int)(k / NN) + 1};  // grid coords 1..N
  const double h = 1.0 / (N + 1);
  double acc[27] = {0.0};
  bool nb[27] = {false};
  // var: per slot the (element, contribution) pairs, summed in element order below
  int64_t eid[27][24];
  double ev[27][24];
  int ne[27] = {0};
  static const double path[4][4] = {{1, -1, 0, 0}, {-1, 2, -1, 0}, {0, -1, 2, -1}, {0, 0, -1, 1}};
  const double ks = h / 6.0, ms = h * h * h / 120.0;
  for (int dz = 0; dz <= 1; ++dz)
    for (int dy = 0; dy <= 1; ++dy)
      for (int dx = 0; dx <= 1; ++dx)
      {
        const int c[3] = {P[0] - dx, P[1] - dy, P[2] - dz};  // cube lower corner, 0..N
        if (c[0] < 0 || c[1] < 0 || c[2] < 0 || c[0] > N || c[1] > N || c[2] > N) continue;
        for (int t = 0; t < 6; ++t)
        {
          int v[4][3];
          for (int a = 0; a < 3; ++a) v[0][a] = c[a];
          for (int a = 0; a < 3; ++a) v[1][a] = v[0][a] + (kPerm[t][0] == a);
          for (int a = 0; a < 3; ++a) v[2][a] = v[1][a] + (kPerm[t][1] == a);
          for (int a = 0; a < 3; ++a) v[3][a] = c[a] + 1;
          int me = -1;
          for (int a = 0; a < 4; ++a)
            if (v[a][0] == P[0] && v[a][1] == P[1] && v[a][2] == P[2]) me = a;
          if (me < 0) continue;
          for (int b = 0; b < 4; ++b)
          {
            bool interior = true;
            for (int a = 0; a < 3; ++a) interior = interior && v[b][a] >= 1 && v[b][a] <= N;
            if (!interior) continue;
            const int slot = ((v[b][2] - P[2] + 1) * 3 + (v[b][1] - P[1] + 1)) * 3 + (v[b][0] - P[0] + 1);
            const double cv = mass ? ms * (me == b ? 2.0 : 1.0) : ks * path[me][b];
            if (var)
            {
              const int64_t e = (((int64_t)c[2] * (N + 1) + c[1]) * (N + 1) + c[0]) * 6 + t;
              eid[slot][ne[slot]] = e;
              ev[slot][ne[slot]++] = kappa(e, mass ? 1 : 0, 1) * cv;
            }
            else
              acc[slot] += cv;
            nb[slot] = true;
          }
        }
      }
  if (var)
    for (int sl = 0; sl < 27; ++sl)
    {
      for (int i = 1; i < ne[sl]; ++i)  // insertion sort by element
        for (int j = i; j > 0 && eid[sl][j - 1] > eid[sl][j]; --j)
        {
          std::swap(eid[sl][j - 1], eid[sl][j]);
          std::swap(ev[sl][j - 1], ev[sl][j]);
        }
      double a = 0.0;
      for (int i = 0; i < ne[sl]; ++i) a += ev[sl][i];
      acc[sl] = a;
    }
  // the 14 edge neighbours + self that exist (interior), in ascending global column
  int32_t cc[27];
  double vv[27];
  int cnt = 0;
  for (int s = 0; s < 27; ++s)
  {
    if (!nb[s]) continue;
    const int ox = s % 3 - 1, oy = (s / 3) % 3 - 1, oz = s / 9 - 1;
    cc[cnt] = (int32_t)(k + oz * NN + oy * (i64)N + ox);
    vv[cnt] = acc[s];
    ++cnt;
  }
  for (int i = 1; i < cnt; ++i)  // insertion sort by column
    for (int j = i; j > 0 && cc[j - 1] > cc[j]; --j)
    {
      std::swap(cc[j - 1], cc[j]);
      std::swap(vv[j - 1], vv[j]);
    }
  for (int i = 0; i < cnt; ++i)
  {
    if (cols) cols[i] = cc[i];
    if (vals) vals[i] = vv[i];
  }
  return cnt;
}

// kind 8: the conductance of the edge from node k along axis a (0 x, 1 y, 2 z) to its + neighbour;
// boundary faces of the grid hash with side 1 (the - face of node k) so every face has its own value
inline double kappa(i64 k, int a, int side)
{
  uint64_t h = (uint64_t)k * 6u + (uint64_t)a * 2u + (uint64_t)side + 0x9e3779b97f4a7c15ull;
  h = (h ^ (h >> 30)) * 0xbf58476d1ce4e5b9ull;
  h = (h ^ (h >> 27)) * 0x94d049bb133111ebull;
  h ^= h >> 31;
  return 0.5 + (double)(h >> 11) * 0x1.0p-53;
}

// Entries of global block row k; returns the count.  cols/vals may be null (count only).
int gen_row(int kind, int N, int overlap, i64 k, int32_t *cols, double *vals)
{
  int c = 0;
  auto put = [&](i64 col, double v) {
    if (cols) cols[c] = (int32_t)col;
    if (vals) vals[c] = v;
    ++c;
  };
  if (kind >= 0 && kind <= 3)
  {
    const int x = (int)(k % N), y = (int)(k / N);
    auto pu = [&](i64 q) {
      const int i = (int)(q / N), j = (int)(q % N);
      return (i < overlap || i > N - 1 - overlap || j < overlap || j > N - 1 - overlap) ? 0.0 : 1.0;
    };
    const bool nb[5] = {y > 0, x > 0, true, x < N - 1, y < N - 1};
    const i64 off[5] = {-(i64)N, -1, 0, 1, (i64)N};
    int noff = 0;
    for (int t = 0; t < 5; ++t)
      if (nb[t] && t != 2) ++noff;
    for (int t = 0; t < 5; ++t)
    {
      if (!nb[t]) continue;
      const i64 q = k + off[t];
      double v = (t == 2) ? 4.0 : -1.0;
      if (kind == 1 && t == 2) v = std::fabs(-1.0 * noff);       // |sum of off-diagonals|
      if (kind == 2) v *= pu(k) * pu(q);
      if (kind == 3) v = (t == 2) ? 1.0 : 0.0;
      put(q, v);
    }
    return c;
  }
  const i64 NN = (i64)N * N;
  const int x = (int)(k % N), y = (int)((k / N) % N), z = (int)(k / NN);
  if (kind == 4)
  {
    if (z > 0) put(k - NN, -1.0);
    if (y > 0) put(k - N, -1.0);
    if (x > 0) put(k - 1, -1.0);
    put(k, 6.0);
    if (x < N - 1) put(k + 1, -1.0);
    if (y < N - 1) put(k + N, -1.0);
    if (z < N - 1) put(k + NN, -1.0);
    return c;
  }
  if (kind == 8)
  {
    const i64 st[3] = {1, (i64)N, NN};
    const int co[3] = {x, y, z};
    // faces -z, -y, -x, +x, +y, +z: the - face of node k is the + edge of k - st[a] (or a boundary face)
    double kf[6];
    for (int a = 0; a < 3; ++a)
    {
      kf[2 - a] = co[a] > 0 ? kappa(k - st[a], a, 0) : kappa(k, a, 1);
      kf[3 + a] = kappa(k, a, 0);
    }
    const double d = ((((kf[0] + kf[1]) + kf[2]) + kf[3]) + kf[4]) + kf[5];
    if (z > 0) put(k - NN, -kf[0]);
    if (y > 0) put(k - N, -kf[1]);
    if (x > 0) put(k - 1, -kf[2]);
    put(k, d);
    if (x < N - 1) put(k + 1, -kf[3]);
    if (y < N - 1) put(k + N, -kf[4]);
    if (z < N - 1) put(k + NN, -kf[5]);
    return c;
  }
  if (kind == 5)
  {
    static const double C[9] = {2, 1, 0, 1, 2, 1, 0, 1, 2};
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx)
        {
          const int xx = x + dx, yy = y + dy, zz = z + dz;
          if (xx < 0 || yy < 0 || zz < 0 || xx >= N || yy >= N || zz >= N) continue;
          const int ax = std::abs(dx), ay = std::abs(dy), az = std::abs(dz);
          const double l = k1(ax) * m1(ay) * m1(az) + m1(ax) * k1(ay) * m1(az) + m1(ax) * m1(ay) * k1(az);
          if (cols) cols[c] = (int32_t)((zz * (i64)N + yy) * N + xx);
          if (vals)
            for (int t = 0; t < 9; ++t) vals[(i64)c * 9 + t] = l * C[t];
          ++c;
        }
    return c;
  }
  if (kind == 6 || kind == 7) return gen_p1_row(kind == 7, N, k, cols, vals);
  if (kind == 9 || kind == 10) return gen_p1_row(kind == 10, N, k, cols, vals, true);
  return -1;
}

i64 nrows_of(int kind, int N) { return (kind <= 3) ? (i64)N * N : (i64)N * N * N; }
constexpr int kGenKinds = 11;
int blk_of(int kind) { return kind == 5 ? 9 : 1; }

}  // namespace

extern "C" int64_t eig_gen_nnzb_rows(int kind, int N, int64_t row_begin, int64_t nrows)
{
  if (kind < 0 || kind >= kGenKinds || N <= 0) return -1;
  i64 s = 0;
  for (i64 k = row_begin; k < row_begin + nrows; ++k) s += gen_row(kind, N, 0, k, nullptr, nullptr);
  return s;
}

extern "C" int64_t eig_gen_nnzb(int kind, int N)
{
  if (kind == 0 || kind == 1 || kind == 2 || kind == 3) return (i64)5 * N * N - 4 * (i64)N;
  if (kind == 4 || kind == 8) return (i64)7 * N * N * N - (i64)6 * N * N;
  if (kind == 5)
  {
    const i64 t = 3 * (i64)N - 2;
    return t * t * t;
  }
  if (kind == 6 || kind == 7 || kind == 9 || kind == 10)
  {
    const i64 n = N, m = N - 1;
    return n * n * n + 6 * n * n * m + 6 * n * m * m + 2 * m * m * m;
  }
  return -1;
}

extern "C" int eig_gen_matrix_rows(int kind, int N, int64_t row_begin, int64_t nrows, int64_t *rowptr, int32_t *col,
                                   double *vals)
{
  if (kind < 0 || kind >= kGenKinds || N <= 0 || !rowptr || !col || !vals) return EIG_ERR_ARG;
  if (row_begin < 0 || row_begin + nrows > nrows_of(kind, N)) return EIG_ERR_SHAPE;
  const int bb = blk_of(kind);
  i64 p = 0;
  for (i64 r = 0; r < nrows; ++r)
  {
    rowptr[r] = p;
    p += gen_row(kind, N, 3, row_begin + r, col + p, vals + p * bb);
  }
  rowptr[nrows] = p;
  return EIG_OK;
}

extern "C" int eig_gen_matrix(int kind, int N, int overlap, int64_t *rowptr, int32_t *col, double *vals)
{
  if (kind < 0 || kind >= kGenKinds || N <= 0 || !rowptr || !col || !vals) return EIG_ERR_ARG;
  const int bb = blk_of(kind);
  const i64 n = nrows_of(kind, N);
  i64 p = 0;
  for (i64 r = 0; r < n; ++r)
  {
    rowptr[r] = p;
    p += gen_row(kind, N, overlap, r, col + p, vals + p * bb);
  }
  rowptr[n] = p;
  return EIG_OK;
}
