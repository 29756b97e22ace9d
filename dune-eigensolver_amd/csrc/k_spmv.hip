// k_spmv.hip -- sparse matrix x vector on the SELL-64 image (gfx950).
//
// Replaces BCRSMatrix::mv (dune-istl; called at arpack_geneo_wrapper.hh:275 through multMvB)
// and the b = 1 product matmul_sparse_tallskinny_naive (kernels_cpp.hh:596-621).
//
// Layout (internal.h): one wavefront owns one 64-row slice, lane l = block row 64 s + l.  Block
// k of the slice is column-major across lanes, so every wave-instruction that fetches the k-th
// value / column of 64 rows reads 512 B / 256 B contiguous (coalesced), and the row's stored
// (ascending-column) order is kept: each lane accumulates exactly like the ISTL row loop, from
// 0.0, mul then add (built with -ffp-contract=off), so y is bitwise BCRSMatrix::mv.
// Padding entries carry column -1 and are skipped (no 0*x term, no -0.0 / NaN side effects).
//
// Work split: a workgroup of 4 waves walks a CONTIGUOUS chunk of slices (waves interleaved),
// so consecutive rows -- which share x lines -- stay in one CU / one XCD's L2; at 2048
// workgroups (8 per CU) the whole grid is resident.
#include "internal.h"
#include "reduce_dev.h"

namespace eigmi {

constexpr int kWaves = kStreamThreads / 64;

struct SliceRange {
  i64 begin, end;  // slice work items handled by this wave: [begin, end) step kWaves
};

__device__ __forceinline__ void chunk_of(i64 count, i64 &b, i64 &e)
{
  const i64 G = gridDim.x;
  const i64 per = (count + G - 1) / G;
  b = (i64)blockIdx.x * per;
  e = b + per;
  if (e > count) e = count;
}

// One scalar row of a 1x1-block SELL slice: prefetch 8 (val, col) pairs, then gather x.
__device__ __forceinline__ double row_dot_b1(const double *__restrict__ val, const i32 *__restrict__ col,
                                             const double *__restrict__ x, i64 base, int width, int lane)
{
  double acc = 0.0;
  for (int k0 = 0; k0 < width; k0 += 8)
  {
    double a[8];
    i32 c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
    {
      if (k0 + k < width)
      {
        const i64 idx = base + (i64)(k0 + k) * 64 + lane;
        c[k] = __builtin_nontemporal_load(col + idx);
        a[k] = __builtin_nontemporal_load(val + idx);
      }
      else
      {
        c[k] = -1;
        a[k] = 0.0;
      }
    }
    double xv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) xv[k] = (c[k] >= 0) ? x[c[k]] : 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (c[k] >= 0) acc += a[k] * xv[k];
  }
  return acc;
}

// y[own + r] = (A x)[r], 1x1 blocks.
__global__ __launch_bounds__(kStreamThreads) void k_spmv_b1(i64 nrows, const i64 *__restrict__ slice_ptr,
                                                            const i32 *__restrict__ slices, i64 first, i64 count,
                                                            const double *__restrict__ val, const i32 *__restrict__ col,
                                                            const double *__restrict__ x, double *__restrict__ y)
{
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  i64 b, e;
  chunk_of(count, b, e);
  for (i64 it = b + wave; it < e; it += kWaves)
  {
    const i64 s = slices ? (i64)slices[first + it] : first + it;
    const i64 base = slice_ptr[s];
    const int width = (int)((slice_ptr[s + 1] - base) >> 6);
    const double acc = row_dot_b1(val, col, x, base, width, lane);
    const i64 r = s * 64 + lane;
    if (r < nrows) y[r] = acc;
  }
}

// General br x bc blocks: lane = block row, per block br*bc values (column-major over lanes).
template <int BR, int BC>
__global__ __launch_bounds__(kStreamThreads) void k_spmv_blk(i64 nbrows, const i64 *__restrict__ slice_ptr,
                                                             const i32 *__restrict__ slices, i64 first, i64 count,
                                                             const double *__restrict__ val,
                                                             const i32 *__restrict__ col,
                                                             const double *__restrict__ x, double *__restrict__ y)
{
  constexpr int BB = BR * BC;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  i64 b, e;
  chunk_of(count, b, e);
  for (i64 it = b + wave; it < e; it += kWaves)
  {
    const i64 s = slices ? (i64)slices[first + it] : first + it;
    const i64 base = slice_ptr[s];
    const int width = (int)((slice_ptr[s + 1] - base) >> 6);
    double acc[BR];
#pragma unroll
    for (int r = 0; r < BR; ++r) acc[r] = 0.0;
    for (int k = 0; k < width; ++k)
    {
      const i64 ci = base + (i64)k * 64 + lane;
      const i32 c = __builtin_nontemporal_load(col + ci);
      if (c < 0) continue;
      const double *vb = val + (base + (i64)k * 64) * BB + lane;
      double a[BB], xv[BC];
#pragma unroll
      for (int t = 0; t < BB; ++t) a[t] = __builtin_nontemporal_load(vb + t * 64);
#pragma unroll
      for (int cc = 0; cc < BC; ++cc) xv[cc] = x[(i64)c * BC + cc];
#pragma unroll
      for (int r = 0; r < BR; ++r)
      {
        double sacc = acc[r];
#pragma unroll
        for (int cc = 0; cc < BC; ++cc) sacc += a[r * BC + cc] * xv[cc];
        acc[r] = sacc;
      }
    }
    const i64 row = s * 64 + lane;
    if (row < nbrows)
    {
#pragma unroll
      for (int r = 0; r < BR; ++r) y[row * BR + r] = acc[r];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Lanczos step, kernel 1 (DESIGN.md "Lanczos step"):
//   t = (A u_j) * sig_j - gam_j * u_{j-1},  dsum[j] = t . u_j  (grid reduction)
// with beta_j = sqrt(nsum[j]), sig_j = 1/beta_j, gam_j = beta_j / sqrt(nsum[j-1]).
// u, up, t are WINDOW buffers; owned rows at `own`.  `carry` (nullable) is a partial dot from a
// previous launch of the same step (interior slices), added first by the last workgroup.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kStreamThreads) void k_lanczos_spmv_b1(
    i64 nrows, i64 own, const i64 *__restrict__ slice_ptr, const i32 *__restrict__ slices, i64 first, i64 count,
    const double *__restrict__ val, const i32 *__restrict__ col, const double *__restrict__ u,
    const double *__restrict__ up, double *__restrict__ t, int j, const double *__restrict__ nsum,
    double *__restrict__ dot_out, double *__restrict__ beta_out, const double *__restrict__ carry,
    double *partials, unsigned *ticket)
{
  __shared__ double tot[1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double beta = sqrt(nsum[j]);
  const double sig = 1.0 / beta;
  const double gam = (j > 0) ? beta * (1.0 / sqrt(nsum[j - 1])) : 0.0;
  i64 b, e;
  chunk_of(count, b, e);
  double d = 0.0;
  for (i64 it = b + wave; it < e; it += kWaves)
  {
    const i64 s = slices ? (i64)slices[first + it] : first + it;
    const i64 base = slice_ptr[s];
    const int width = (int)((slice_ptr[s + 1] - base) >> 6);
    const double acc = row_dot_b1(val, col, u, base, width, lane);
    const i64 r = s * 64 + lane;
    if (r < nrows)
    {
      double ti = acc * sig;
      if (j > 0) ti = ti - gam * up[own + r];
      t[own + r] = ti;
      d += ti * u[own + r];
    }
  }
  double v[1] = {d};
  if (grid_sum<1, kStreamThreads>(v, partials, ticket, tot))
  {
    if (threadIdx.x == 0)
    {
      dot_out[0] = carry ? (carry[0] + tot[0]) : tot[0];
      if (beta_out) beta_out[0] = beta;
    }
  }
}

void launch_spmv(const eig_mat_s &A, const double *x, double *y, const i32 *slices, i64 first, i64 count,
                 hipStream_t s)
{
  if (count <= 0) return;
  const i64 need = (count + kWaves - 1) / kWaves;
  const int G = (int)(need < kStreamBlocks ? need : kStreamBlocks);
  const double *xw = x;  // window-local columns index x directly
  double *yo = y + A.own_offset;
#define EIG_BLK(R, C)                                                                                  \
  if (A.br == R && A.bc == C)                                                                          \
  {                                                                                                    \
    hipLaunchKernelGGL((k_spmv_blk<R, C>), dim3(G), dim3(kStreamThreads), 0, s, A.nb_rows, A.slice_ptr, \
                       slices, first, count, A.val, A.col, xw, yo);                                    \
    return;                                                                                            \
  }
  if (A.br == 1 && A.bc == 1)
  {
    hipLaunchKernelGGL(k_spmv_b1, dim3(G), dim3(kStreamThreads), 0, s, A.nb_rows, A.slice_ptr, slices, first,
                       count, A.val, A.col, xw, yo);
    return;
  }
  EIG_BLK(1, 2) EIG_BLK(1, 3) EIG_BLK(1, 4)
  EIG_BLK(2, 1) EIG_BLK(2, 2) EIG_BLK(2, 3) EIG_BLK(2, 4)
  EIG_BLK(3, 1) EIG_BLK(3, 2) EIG_BLK(3, 3) EIG_BLK(3, 4)
  EIG_BLK(4, 1) EIG_BLK(4, 2) EIG_BLK(4, 3) EIG_BLK(4, 4)
#undef EIG_BLK
  throw Error(EIG_ERR_BLOCKSIZE, "eig_mv: block size not supported (br, bc must be in 1..4)");
}

void launch_lanczos_spmv(const eig_mat_s &A, const double *u, const double *up, double *t, int j,
                         const LanczosState &st, const i32 *slices, i64 first, i64 count, double *dot_out,
                         double *beta_out, const double *carry, int ticket, hipStream_t s, ReduceWS red)
{
  EIG_CHECK(A.br == 1 && A.bc == 1, EIG_ERR_BLOCKSIZE, "Lanczos driver: 1x1 blocks only");
  const i64 need = (count + kWaves - 1) / kWaves;
  int G = (int)(need < kStreamBlocks ? need : kStreamBlocks);
  if (G < 1) G = 1;
  hipLaunchKernelGGL(k_lanczos_spmv_b1, dim3(G), dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset, A.slice_ptr,
                     slices, first, count, A.val, A.col, u, up, t, j, st.nsum, dot_out, beta_out, carry,
                     red.partials, red.tickets + ticket);
}

}  // namespace eigmi
