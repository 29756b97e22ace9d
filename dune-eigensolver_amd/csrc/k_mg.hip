// k_mg.hip -- grid transfers of the geometric multigrid inner solve (mg.cpp) on window-layout
// MultiVector<double,8> blocks (gfx950).
//
// Grids are lexicographic boxes, k = (z ny + y) nx + x.  The coarse grid keeps the fine nodes of
// odd index in every direction (coarse c <-> fine 2c + 1, nc = nf / 2), and P is trilinear: per
// direction a fine node of odd index i takes coarse (i - 1) / 2 with weight 1, one of even index
// takes coarse i / 2 - 1 and i / 2 with weight 1/2 each (a neighbour outside the coarse grid is a
// Dirichlet node: dropped).  Restriction is exactly P^T (the same weights, gathered on the coarse
// row), so the V-cycle is symmetric.  One thread per (row, 8-column block): 64-B rows as four 16-B
// loads; the sums run in a fixed order (deterministic).
#include "internal.h"

namespace eigmi {

namespace {

inline int grid_cap(i64 work, i64 per_block, int cap)
{
  i64 g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

__device__ __forceinline__ void add_row(double (&acc)[8], const double *p, double w)
{
  const double2 *q = reinterpret_cast<const double2 *>(p);
#pragma unroll
  for (int h = 0; h < 4; ++h)
  {
    const double2 v = q[h];
    acc[2 * h] += w * v.x;
    acc[2 * h + 1] += w * v.y;
  }
}

}  // namespace

// Bc(I) = sum over the fine 3 x 3 x 3 block around 2 I + 1 of w_x w_y w_z Rf(i)  (w = 1 at the
// centre, 1/2 at +-1 per direction), z, y, x ascending
__global__ __launch_bounds__(256) void k_mg_restrict(int fx, int fy, int fz, int cx, int cy, int cz, int nblk, i64 ldf,
                                                     i64 ldc, const double *__restrict__ Rf, double *__restrict__ Bc)
{
  const i64 nc = (i64)cx * cy * cz, total = nc * nblk;
  for (i64 idx = (i64)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (i64)gridDim.x * 256)
  {
    const i64 b = idx / nc, I = idx - b * nc;
    const int X = (int)(I % cx), Y = (int)((I / cx) % cy), Z = (int)(I / ((i64)cx * cy));
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const double *base = Rf + b * ldf * 8;
    for (int dz = -1; dz <= 1; ++dz)
    {
      const int z = 2 * Z + 1 + dz;
      if (z < 0 || z >= fz) continue;
      const double wz = dz ? 0.5 : 1.0;
      for (int dy = -1; dy <= 1; ++dy)
      {
        const int y = 2 * Y + 1 + dy;
        if (y < 0 || y >= fy) continue;
        const double wzy = wz * (dy ? 0.5 : 1.0);
        for (int dx = -1; dx <= 1; ++dx)
        {
          const int x = 2 * X + 1 + dx;
          if (x < 0 || x >= fx) continue;
          add_row(acc, base + (((i64)z * fy + y) * fx + x) * 8, wzy * (dx ? 0.5 : 1.0));
        }
      }
    }
    double2 *dst = reinterpret_cast<double2 *>(Bc + (b * ldc + I) * 8);
#pragma unroll
    for (int h = 0; h < 4; ++h) dst[h] = make_double2(acc[2 * h], acc[2 * h + 1]);
  }
}

// Xf(i) += sum over the coarse nodes of i of w_x w_y w_z Xc(J)  (z, y, x ascending)
__global__ __launch_bounds__(256) void k_mg_prolong_add(int fx, int fy, int fz, int cx, int cy, int cz, int nblk,
                                                        i64 ldf, i64 ldc, const double *__restrict__ Xc,
                                                        double *__restrict__ Xf)
{
  const i64 nf = (i64)fx * fy * fz, total = nf * nblk;
  for (i64 idx = (i64)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (i64)gridDim.x * 256)
  {
    const i64 b = idx / nf, i = idx - b * nf;
    const int x = (int)(i % fx), y = (int)((i / fx) % fy), z = (int)(i / ((i64)fx * fy));
    // per direction: coarse indices c0 (weight w0) and c1 (weight w1; -1 = none)
    auto split = [](int f, int nc, int &c0, int &c1, double &w0) {
      if (f & 1)
      {
        c0 = (f - 1) >> 1;
        c1 = -1;
        w0 = 1.0;
      }
      else
      {
        c0 = (f >> 1) - 1;
        c1 = (f >> 1) < nc ? (f >> 1) : -1;
        w0 = 0.5;
      }
    };
    int zc[2], yc[2], xc[2];
    double wz, wy, wx;
    split(z, cz, zc[0], zc[1], wz);
    split(y, cy, yc[0], yc[1], wy);
    split(x, cx, xc[0], xc[1], wx);
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const double *base = Xc + b * ldc * 8;
    for (int a = 0; a < 2; ++a)
    {
      if (zc[a] < 0) continue;
      for (int c = 0; c < 2; ++c)
      {
        if (yc[c] < 0) continue;
        for (int e = 0; e < 2; ++e)
        {
          if (xc[e] < 0) continue;
          add_row(acc, base + (((i64)zc[a] * cy + yc[c]) * cx + xc[e]) * 8, wz * wy * wx);
        }
      }
    }
    double2 *dst = reinterpret_cast<double2 *>(Xf + (b * ldf + i) * 8);
#pragma unroll
    for (int h = 0; h < 4; ++h)
    {
      const double2 v = dst[h];
      dst[h] = make_double2(v.x + acc[2 * h], v.y + acc[2 * h + 1]);
    }
  }
}

// Y = a X + b Y over the n owned rows of m columns (window layout, pointers at owned row 0)
__global__ __launch_bounds__(256) void k_mv8_axpby(i64 n, int nblk, i64 ld, double a, const double *__restrict__ X,
                                                   double b, double *__restrict__ Y)
{
  const i64 total = n * nblk * 4;  // 16-B pieces
  for (i64 idx = (i64)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (i64)gridDim.x * 256)
  {
    const i64 row = idx >> 2, blk = row / n, r = row - blk * n;
    const i64 at = (blk * ld + r) * 8 + (idx & 3) * 2;
    const double2 x = *reinterpret_cast<const double2 *>(X + at);
    double2 *y = reinterpret_cast<double2 *>(Y + at);
    const double2 v = *y;
    *y = make_double2(a * x.x + b * v.x, a * x.y + b * v.y);
  }
}

void launch_mg_restrict(const int *fdim, const int *cdim, i64 m, i64 ldf, i64 ldc, const double *Rf, double *Bc,
                        hipStream_t s)
{
  const i64 nc = (i64)cdim[0] * cdim[1] * cdim[2];
  hipLaunchKernelGGL(k_mg_restrict, dim3(grid_cap(nc * (m / 8), 256, kStreamBlocks)), dim3(256), 0, s, fdim[0],
                     fdim[1], fdim[2], cdim[0], cdim[1], cdim[2], (int)(m / 8), ldf, ldc, Rf, Bc);
  EIG_HIP(hipGetLastError());
}

void launch_mg_prolong_add(const int *fdim, const int *cdim, i64 m, i64 ldf, i64 ldc, const double *Xc, double *Xf,
                           hipStream_t s)
{
  const i64 nf = (i64)fdim[0] * fdim[1] * fdim[2];
  hipLaunchKernelGGL(k_mg_prolong_add, dim3(grid_cap(nf * (m / 8), 256, kStreamBlocks)), dim3(256), 0, s, fdim[0],
                     fdim[1], fdim[2], cdim[0], cdim[1], cdim[2], (int)(m / 8), ldf, ldc, Xc, Xf);
  EIG_HIP(hipGetLastError());
}

void launch_mv8_axpby(i64 n, i64 m, i64 ld, double a, const double *X, double b, double *Y, hipStream_t s)
{
  hipLaunchKernelGGL(k_mv8_axpby, dim3(grid_cap(n * (m / 8) * 4, 256, kStreamBlocks)), dim3(256), 0, s, n,
                     (int)(m / 8), ld, a, X, b, Y);
  EIG_HIP(hipGetLastError());
}

}  // namespace eigmi
