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

// Thread layout of the transfers: a workgroup takes 64 consecutive x of one grid line (y, z) and
// one 8-column block (blockIdx.y); thread t handles x = x0 + t / 4 and the 16-B quarter t % 4 of
// that 64-B row.  The prolongation stages the coarse rows it gathers (a 2 x 2 x 33 box) in LDS with
// contiguous 16-B loads, so every row leaves L2 once per workgroup instead of once per thread
// that uses it (sums in the row-by-row order, z, y, x ascending).
constexpr int kMgRows = 64;
constexpr int kMgCoarse = kMgRows / 2 + 1; // coarse rows of one line over 64 fine x

// Bc(I) = sum over the fine 3 x 3 x 3 block around 2 I + 1 of w_x w_y w_z Rf(i)  (w = 1 at the
// centre, 1/2 at +-1 per direction).  Separable: a workgroup takes 32 coarse x of one coarse line;
// its threads first fold the 9 fine lines (dz, dy) of each fine x under them, S(x) = sum (z, y
// ascending) w_z w_y Rf -- coalesced 16-B loads, 9 in flight per thread -- into LDS, then the
// coarse x sums S(2X) / 2 + S(2X + 1) + S(2X + 2) / 2.  (The weights are powers of two, so every
// product is the exact w_x w_y w_z Rf; only the association of the sums differs from row by row.)
constexpr int kMgRX = 32, kMgRFine = 2 * kMgRX + 1;
__global__ __launch_bounds__(256) void k_mg_restrict(int fx, int fy, int fz, int cx, int cy, int cz, i64 ldf, i64 ldc,
                                                     const double *__restrict__ Rf, double *__restrict__ Bc)
{
  __shared__ double2 S[kMgRFine * 4];
  const int xb = (cx + kMgRX - 1) / kMgRX, line = (int)blockIdx.x / xb;
  const int X0 = ((int)blockIdx.x - line * xb) * kMgRX;
  const int Y = line % cy, Z = line / cy;
  const double *base = Rf + (i64)blockIdx.y * ldf * 8;
  const int f0 = 2 * X0;  // fine x of S[0] (the -1 neighbour of X0's centre 2 X0 + 1)
  for (int c = threadIdx.x; c < kMgRFine * 4; c += 256)
  {
    const int x = f0 + (c >> 2), q = c & 3;
    double a0 = 0.0, a1 = 0.0;
    if (x < fx)
      for (int dz = -1; dz <= 1; ++dz)
      {
        const int z = 2 * Z + 1 + dz;
        if (z >= fz) continue;
        const double wz = dz ? 0.5 : 1.0;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
        {
          const int y = 2 * Y + 1 + dy;
          if (y >= fy) continue;
          const double w = wz * (dy ? 0.5 : 1.0);
          const double2 v = *reinterpret_cast<const double2 *>(base + (((i64)z * fy + y) * fx + x) * 8 + q * 2);
          a0 += w * v.x;
          a1 += w * v.y;
        }
      }
    S[c] = make_double2(a0, a1);
  }
  __syncthreads();
  const int X = X0 + (int)(threadIdx.x >> 2), q = threadIdx.x & 3;
  if (threadIdx.x >= kMgRX * 4 || X >= cx) return;
  const int l = (2 * X - f0) * 4 + q;  // S index of fine x = 2 X (the -1 neighbour)
  const double2 sm = S[l], s0 = S[l + 4], sp = S[l + 8];
  const double b0 = 0.5 * sm.x + s0.x + 0.5 * sp.x, b1 = 0.5 * sm.y + s0.y + 0.5 * sp.y;
  *reinterpret_cast<double2 *>(Bc + ((i64)blockIdx.y * ldc + ((i64)Z * cy + Y) * cx + X) * 8 + q * 2) =
      make_double2(b0, b1);
}

// Xf(i) += sum over the coarse nodes of i of w_x w_y w_z Xc(J)  (z, y, x ascending)
__global__ __launch_bounds__(256) void k_mg_prolong_add(int fx, int fy, int fz, int cx, int cy, int cz, i64 ldf,
                                                        i64 ldc, const double *__restrict__ Xc,
                                                        double *__restrict__ Xf)
{
  __shared__ double2 cl[4][kMgCoarse * 4];  // the (zc, yc) coarse line segments, 16-B quarters
  const int xb = (fx + kMgRows - 1) / kMgRows, line = (int)blockIdx.x / xb;
  const int xs = ((int)blockIdx.x - line * xb) * kMgRows;
  const int x = xs + (int)(threadIdx.x >> 2), q = threadIdx.x & 3;
  const int y = line % fy, z = line / fy;
  // per direction: coarse indices c0 (weight w0) and c1 (weight w0; -1 = none)
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
  split(z, cz, zc[0], zc[1], wz);  // (z, y: uniform over the workgroup)
  split(y, cy, yc[0], yc[1], wy);
  split(x, cx, xc[0], xc[1], wx);
  const int c0 = xs / 2 - 1;  // first coarse x staged
  const double *base = Xc + (i64)blockIdx.y * ldc * 8;
  // this thread's fine row quarter, loaded before the staging barrier (its latency overlaps it)
  const bool mine = x < fx && z < fz;
  double2 *dst = reinterpret_cast<double2 *>(Xf + ((i64)blockIdx.y * ldf + ((i64)z * fy + y) * fx + (mine ? x : 0)) * 8 +
                                             q * 2);
  const double2 vf = mine ? *dst : make_double2(0.0, 0.0);
  for (int a = 0; a < 2; ++a)
    for (int c = 0; c < 2; ++c)
    {
      if (zc[a] < 0 || yc[c] < 0) continue;
      const double2 *lp = reinterpret_cast<const double2 *>(base + ((i64)zc[a] * cy + yc[c]) * cx * 8);
      for (int k = threadIdx.x; k < kMgCoarse * 4; k += 256)
      {
        const int X = c0 + (k >> 2);
        cl[2 * a + c][k] = (X >= 0 && X < cx) ? lp[(i64)X * 4 + (k & 3)] : make_double2(0.0, 0.0);
      }
    }
  __syncthreads();
  if (!mine) return;
  const double w = wz * wy * wx;
  double a0 = 0.0, a1 = 0.0;
  for (int a = 0; a < 2; ++a)
  {
    if (zc[a] < 0) continue;
    for (int c = 0; c < 2; ++c)
    {
      if (yc[c] < 0) continue;
      for (int e = 0; e < 2; ++e)
      {
        if (xc[e] < 0) continue;
        const double2 v = cl[2 * a + c][(xc[e] - c0) * 4 + q];
        a0 += w * v.x;
        a1 += w * v.y;
      }
    }
  }
  *dst = make_double2(vf.x + a0, vf.y + a1);
}

// Y = a X + b Y over the n owned rows of m columns (window layout, pointers at owned row 0);
// blockIdx.y = column block, 16-B pieces
__global__ __launch_bounds__(256) void k_mv8_axpby(i64 n, i64 ld, double a, const double *__restrict__ X, double b,
                                                   double *__restrict__ Y)
{
  const i64 off = (i64)blockIdx.y * ld * 8, total = n * 4;
  const double2 *xs = reinterpret_cast<const double2 *>(X + off);
  double2 *ys = reinterpret_cast<double2 *>(Y + off);
  for (i64 idx = (i64)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (i64)gridDim.x * 256)
  {
    const double2 x = xs[idx];
    const double2 v = ys[idx];
    ys[idx] = make_double2(a * x.x + b * v.x, a * x.y + b * v.y);
  }
}

void launch_mg_restrict(const int *fdim, const int *cdim, i64 m, i64 ldf, i64 ldc, const double *Rf, double *Bc,
                        hipStream_t s)
{
  const i64 blocks = (i64)((cdim[0] + kMgRX - 1) / kMgRX) * cdim[1] * cdim[2];
  EIG_CHECK(blocks < (1LL << 31), EIG_ERR_SHAPE, "multigrid restriction: grid too large");
  hipLaunchKernelGGL(k_mg_restrict, dim3((unsigned)blocks, (unsigned)(m / 8)), dim3(256), 0, s, fdim[0], fdim[1],
                     fdim[2], cdim[0], cdim[1], cdim[2], ldf, ldc, Rf, Bc);
  EIG_HIP(hipGetLastError());
}

void launch_mg_prolong_add(const int *fdim, const int *cdim, i64 m, i64 ldf, i64 ldc, const double *Xc, double *Xf,
                           hipStream_t s)
{
  const i64 blocks = (i64)((fdim[0] + kMgRows - 1) / kMgRows) * fdim[1] * fdim[2];
  EIG_CHECK(blocks < (1LL << 31), EIG_ERR_SHAPE, "multigrid prolongation: grid too large");
  hipLaunchKernelGGL(k_mg_prolong_add, dim3((unsigned)blocks, (unsigned)(m / 8)), dim3(256), 0, s, fdim[0], fdim[1],
                     fdim[2], cdim[0], cdim[1], cdim[2], ldf, ldc, Xc, Xf);
  EIG_HIP(hipGetLastError());
}

void launch_mv8_axpby(i64 n, i64 m, i64 ld, double a, const double *X, double b, double *Y, hipStream_t s)
{
  hipLaunchKernelGGL(k_mv8_axpby, dim3(grid_cap(n * 4, 256, 4 * kStreamBlocks / (int)(m / 8) + 1), (unsigned)(m / 8)),
                     dim3(256), 0, s, n, ld, a, X, b, Y);
  EIG_HIP(hipGetLastError());
}

}  // namespace eigmi
