// k_block.hip -- window-layout MultiVector<double,8> kernels (gfx950) for the block methods:
//
//   k_sell_mv8        Y = A X over the SELL-64 image, row per lane, 8 columns per column block,
//                     MB column blocks per matrix pass; epilogue kStore (plain SpMM, a2) or kCheb
//                     (one Chebyshev-Jacobi step of the mass solve, fused into the SpMM)
//   k_diag_inv        dinv[r] = 1 / a_rr
//   k_cheb_init       X = gamma * dinv o B
//   k_panel_gram_*    G = Q1^T Q2 for tall-skinny panels on MFMA (v_mfma_f64_16x16x4f64), two
//                     deterministic stages (per-workgroup partials, then a fixed-order sum)
//   k_panel_update    Y = beta Y + alpha Q S (Q: n x m1, S: m1 x m2 with m2 <= 32), FMA with S
//                     in scalar registers
//
// Window layout: column block b of a multivector with leading dimension ld (the matrix window)
// is ld rows of 8 contiguous doubles at Q + 8 b ld; owned row r sits at window row own + r.  On
// one rank ld = n and own = 0, which is the reference's MultiVector<double,8> layout
// (multivector.hh:130-139).
#include "internal.h"

namespace eigmi {

typedef double d4 __attribute__((ext_vector_type(4)));

static inline int grid_cap(i64 work, i64 per_block, int cap)
{
  i64 g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

// ---------------------------------------------------------------------------------------------
// SpMM over 64-row SELL slices (R = 1): lane l computes all 8 columns of slice row l for MB
// column blocks b0 .. b0+nb-1; the slice's value / column (or offset + mask) streams are read once
// per MB blocks, coalesced; each gathered X row is four 16-B loads.  Per column the row sum runs
// over the stored entries in ascending-column order from 0.0 (bitwise the reference's
// matmul_sparse_tallskinny_blocked, kernels_cpp.hh:644-655).
//
// kCheb epilogue (Golub-Varga three-term Chebyshev semi-iteration for M x = b with the Jacobi
// splitting): with acc = (M x_k)_r,
//     x_{k+1}[r] = omega (x_k[r] + gamma dinv[r] (b[r] - acc) - x_{k-1}[r]) + x_{k-1}[r]
// written in place over x_{k-1} (Xold); x_k is the gathered input X.
// ---------------------------------------------------------------------------------------------
enum { kStore = 0, kCheb = 1 };

template <int MB, bool STENCIL, int EPI>
__global__ __launch_bounds__(256) void k_sell_mv8(i64 nrows, i64 nslices, const i64 *__restrict__ slice_ptr,
                                                  const double *__restrict__ val, const i32 *__restrict__ col,
                                                  const i32 *__restrict__ st_delta, const uint8_t *__restrict__ st_mask,
                                                  const double *__restrict__ X, double *__restrict__ Y, i64 ld,
                                                  i64 own, int b0, int nb, const double *__restrict__ Bv,
                                                  const double *__restrict__ dinv, double omega, double gamma)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const i64 per = (nslices + gridDim.x - 1) / gridDim.x;
  const i64 sb = (i64)blockIdx.x * per, se = sb + per < nslices ? sb + per : nslices;
  for (i64 s = sb + wave; s < se; s += 4)
  {
    const i64 base = slice_ptr[s];
    const int width = (int)((slice_ptr[s + 1] - base) >> 6);
    const i64 r = s * 64 + lane;
    unsigned m = 0;
    if (STENCIL) m = st_mask[s * 64 + lane];
    double acc[MB][8];
#pragma unroll
    for (int q = 0; q < MB; ++q)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) acc[q][jj] = 0.0;
    for (int k = 0; k < width; ++k)
    {
      const double a = __builtin_nontemporal_load(val + base + k * 64 + lane);
      i64 c;
      bool ok;
      if (STENCIL)
      {
        ok = (m >> k) & 1u;
        c = own + r + st_delta[8 * s + k];  // window column = own + global row - row_begin + delta
      }
      else
      {
        const i32 cc = __builtin_nontemporal_load(col + base + k * 64 + lane);
        ok = cc >= 0;
        c = cc;
      }
      if (!ok) continue;
#pragma unroll
      for (int q = 0; q < MB; ++q)
      {
        if (q < nb)
        {
          const double2 *xr = reinterpret_cast<const double2 *>(X + ((i64)(b0 + q) * ld + c) * 8);
#pragma unroll
          for (int h = 0; h < 4; ++h)
          {
            const double2 xv = xr[h];
            acc[q][2 * h] += a * xv.x;
            acc[q][2 * h + 1] += a * xv.y;
          }
        }
      }
    }
    if (r < nrows)
    {
      double di = 0.0;
      if (EPI == kCheb) di = dinv[r];
#pragma unroll
      for (int q = 0; q < MB; ++q)
        if (q < nb)
        {
          const i64 row = ((i64)(b0 + q) * ld + own + r) * 8;
          double2 *yr = reinterpret_cast<double2 *>(Y + row);
          if (EPI == kStore)
          {
#pragma unroll
            for (int h = 0; h < 4; ++h) yr[h] = make_double2(acc[q][2 * h], acc[q][2 * h + 1]);
          }
          else
          {
            const double2 *xr = reinterpret_cast<const double2 *>(X + row);
            const double2 *br = reinterpret_cast<const double2 *>(Bv + row);
            const double gd = gamma * di;
#pragma unroll
            for (int h = 0; h < 4; ++h)
            {
              const double2 xk = xr[h], bb = br[h], xo = yr[h];
              const double n0 = omega * (xk.x + gd * (bb.x - acc[q][2 * h]) - xo.x) + xo.x;
              const double n1 = omega * (xk.y + gd * (bb.y - acc[q][2 * h + 1]) - xo.y) + xo.y;
              yr[h] = make_double2(n0, n1);
            }
          }
        }
    }
  }
}

namespace {
bool all_stencil(const eig_mat_s &A) { return A.n_stencil_slices == A.nslices && A.n_stencil_slices > 0; }

template <int EPI>
void sell_mv8(const eig_mat_s &A, i64 m, const double *X, double *Y, const double *Bv, const double *dinv,
              double omega, double gamma, hipStream_t s)
{
  EIG_CHECK(A.br == 1 && A.bc == 1, EIG_ERR_BLOCKSIZE,
            "matmul_sparse_tallskinny_blocked: only implemented for FieldMatrix<..,1,1>");
  EIG_CHECK(A.R == 1, EIG_ERR_ARG, "multivector kernels need the R = 1 SELL image (unset EIGMI_SELL_R)");
  const int nblk = (int)(m / 8);
  constexpr int MB = 2;
  const int gx = grid_cap(A.nslices, 4, kStreamBlocks);
  const bool st = all_stencil(A);
  for (int b0 = 0; b0 < nblk; b0 += MB)
  {
    const int nb = nblk - b0 < MB ? nblk - b0 : MB;
    if (st)
      hipLaunchKernelGGL((k_sell_mv8<MB, true, EPI>), dim3(gx), dim3(256), 0, s, A.nb_rows, A.nslices, A.slice_ptr,
                         A.val, A.col, A.st_delta, A.st_mask, X, Y, A.window, A.own_offset, b0, nb, Bv, dinv, omega,
                         gamma);
    else
      hipLaunchKernelGGL((k_sell_mv8<MB, false, EPI>), dim3(gx), dim3(256), 0, s, A.nb_rows, A.nslices, A.slice_ptr,
                         A.val, A.col, A.st_delta, A.st_mask, X, Y, A.window, A.own_offset, b0, nb, Bv, dinv, omega,
                         gamma);
  }
  EIG_HIP(hipGetLastError());
}
}  // namespace

void launch_sell_mv8(const eig_mat_s &A, i64 m, const double *X, double *Y, hipStream_t s)
{
  sell_mv8<kStore>(A, m, X, Y, nullptr, nullptr, 0.0, 0.0, s);
}

void launch_cheb_step(const eig_mat_s &M, i64 m, const double *Xk, double *Xold, const double *B, const double *dinv,
                      double omega, double gamma, hipStream_t s)
{
  sell_mv8<kCheb>(M, m, Xk, Xold, B, dinv, omega, gamma, s);
}

// ---------------------------------------------------------------------------------------------
// dinv[r] = 1 / a_rr from the SELL image (explicit columns are kept for every slice).
// ---------------------------------------------------------------------------------------------
__global__ void k_diag_inv(i64 nrows, int C, const i64 *__restrict__ slice_ptr, const double *__restrict__ val,
                           const i32 *__restrict__ col, i64 own, double *__restrict__ dinv)
{
  for (i64 r = (i64)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (i64)gridDim.x * blockDim.x)
  {
    const i64 s = r / C, l = r % C;
    const i64 base = slice_ptr[s];
    const i64 w = (slice_ptr[s + 1] - base) / C;
    double d = 0.0;
    for (i64 k = 0; k < w; ++k)
      if (col[base + k * C + l] == own + r) d = val[base + k * C + l];
    dinv[r] = 1.0 / d;
  }
}

void launch_diag_inv(const eig_mat_s &A, double *dinv, hipStream_t s)
{
  EIG_CHECK(A.br == 1 && A.bc == 1, EIG_ERR_BLOCKSIZE, "diagonal extraction: 1x1 blocks only");
  hipLaunchKernelGGL(k_diag_inv, dim3(grid_cap(A.nb_rows, 256, kStreamBlocks)), dim3(256), 0, s, A.nb_rows,
                     (int)(64 * A.R), A.slice_ptr, A.val, A.col, A.own_offset, dinv);
  EIG_HIP(hipGetLastError());
}

// X = gamma * dinv o B on the owned rows of m columns (window layout).
__global__ __launch_bounds__(256) void k_cheb_init(i64 n, i64 ld, i64 own, int nblk, const double *__restrict__ B,
                                                   const double *__restrict__ dinv, double gamma, double *__restrict__ X)
{
  const i64 total = n * nblk;
  for (i64 idx = (i64)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (i64)gridDim.x * 256)
  {
    const i64 b = idx / n, r = idx - b * n;
    const double g = gamma * dinv[r];
    const i64 row = (b * ld + own + r) * 8;
    const double2 *src = reinterpret_cast<const double2 *>(B + row);
    double2 *dst = reinterpret_cast<double2 *>(X + row);
#pragma unroll
    for (int h = 0; h < 4; ++h)
    {
      const double2 v = src[h];
      dst[h] = make_double2(g * v.x, g * v.y);
    }
  }
}

void launch_cheb_init(i64 n, i64 ld, i64 own, i64 m, const double *B, const double *dinv, double gamma, double *X,
                      hipStream_t s)
{
  hipLaunchKernelGGL(k_cheb_init, dim3(grid_cap(n * (m / 8), 256, kStreamBlocks)), dim3(256), 0, s, n, ld, own,
                     (int)(m / 8), B, dinv, gamma, X);
  EIG_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// Panel Gram on MFMA: G (m1 x m2, row-major) = Q1^T Q2 over n rows.  Q1 / Q2 address owned row 0
// of column block 0 (the caller adds own * 8), column blocks ld rows apart.
//
// Workgroup (x, y): output block y = (bi, bj) of TI x TJ 16x16 tiles, row groups of 4 strided by
// x.  Lane l supplies A[i = l&15][k = l>>4] = Q1(r0 + k, c1 + i) and B[k][j = l&15] = Q2(r0 + k,
// c2 + j) per tile; the accumulator holds C[(l>>4) + 4q][l&15].  The Q2 operands of a row group
// are loaded once for all TI tiles and the Q1 operands once for all TJ tiles, so the panel
// streams through HBM ceil(m2 / 16 TJ) (Q1) and ceil(m1 / 16 TI) (Q2) times.  Stage 1 writes
// each workgroup's block (waves summed in LDS) to part[x][y][...]; stage 2 sums the partials in
// x order -- deterministic, bitwise reproducible run to run.
// ---------------------------------------------------------------------------------------------
template <int TI, int TJ>
__global__ __launch_bounds__(256) void k_panel_gram_part(i64 n, i64 ld, int m1, int m2, int nbj,
                                                         const double *__restrict__ Q1, const double *__restrict__ Q2,
                                                         double *__restrict__ part)
{
  constexpr int E = TI * TJ * 256;  // block elements
  __shared__ double sh[4][E];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bi = blockIdx.y / nbj, bj = blockIdx.y % nbj;
  const int kk = lane >> 4, li = lane & 15;
  i64 aoff[TI], boff[TJ];
  bool aok[TI], bok[TJ];
#pragma unroll
  for (int t = 0; t < TI; ++t)
  {
    const int c = bi * 16 * TI + t * 16 + li;
    aok[t] = c < m1;
    aoff[t] = aok[t] ? ((i64)(c >> 3) * ld) * 8 + (c & 7) : 0;
  }
#pragma unroll
  for (int u = 0; u < TJ; ++u)
  {
    const int c = bj * 16 * TJ + u * 16 + li;
    bok[u] = c < m2;
    boff[u] = bok[u] ? ((i64)(c >> 3) * ld) * 8 + (c & 7) : 0;
  }
  d4 acc[TI][TJ];
#pragma unroll
  for (int t = 0; t < TI; ++t)
#pragma unroll
    for (int u = 0; u < TJ; ++u) acc[t][u] = d4{0.0, 0.0, 0.0, 0.0};
  const i64 ngroups = (n + 3) / 4;
  const i64 wstride = (i64)gridDim.x * 4;
  constexpr int U = 2;  // row groups per iteration: all loads issued before the MFMAs
  for (i64 g0 = (i64)blockIdx.x * 4 + wave; g0 < ngroups; g0 += U * wstride)
  {
    double a[U][TI], b[U][TJ];
#pragma unroll
    for (int v = 0; v < U; ++v)
    {
      const i64 r = (g0 + v * wstride) * 4 + kk;
      const bool rok = r < n;
#pragma unroll
      for (int t = 0; t < TI; ++t) a[v][t] = (aok[t] && rok) ? Q1[aoff[t] + r * 8] : 0.0;
#pragma unroll
      for (int u = 0; u < TJ; ++u) b[v][u] = (bok[u] && rok) ? Q2[boff[u] + r * 8] : 0.0;
    }
#pragma unroll
    for (int v = 0; v < U; ++v)
#pragma unroll
      for (int t = 0; t < TI; ++t)
#pragma unroll
        for (int u = 0; u < TJ; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[v][t], b[v][u], acc[t][u], 0, 0, 0);
  }
  // element index inside the block: ((t TJ + u) 16 + row) 16 + col
#pragma unroll
  for (int t = 0; t < TI; ++t)
#pragma unroll
    for (int u = 0; u < TJ; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) sh[wave][((t * TJ + u) * 16 + kk + 4 * q) * 16 + li] = acc[t][u][q];
  __syncthreads();
  double *dst = part + ((size_t)blockIdx.x * gridDim.y + blockIdx.y) * E;
  for (int e = threadIdx.x; e < E; e += 256) dst[e] = ((sh[0][e] + sh[1][e]) + sh[2][e]) + sh[3][e];
}

// Stage 2: workgroup = 64 consecutive block elements; wave w sums the partials of workgroups
// x in [w gx/4, (w+1) gx/4) in x order (16 loads in flight), then the 4 wave sums are added in
// wave order.
template <int TI, int TJ>
__global__ __launch_bounds__(256) void k_panel_gram_reduce(int gx, int ny, int nbj, int m1, int m2,
                                                           const double *__restrict__ part, double *__restrict__ G)
{
  constexpr int E = TI * TJ * 256;
  __shared__ double sh[4][64];
  const i64 total = (i64)ny * E;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const i64 idx = (i64)blockIdx.x * 64 + lane;
  const int x0 = (int)((i64)gx * wave / 4), x1 = (int)((i64)gx * (wave + 1) / 4);
  double s = 0.0;
  if (idx < total)
  {
    for (int x = x0; x < x1; x += 16)
    {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = (x + u < x1) ? part[(size_t)(x + u) * total + idx] : 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
  }
  sh[wave][lane] = s;
  __syncthreads();
  if (wave != 0 || idx >= total) return;
  const double tot = ((sh[0][lane] + sh[1][lane]) + sh[2][lane]) + sh[3][lane];
  const int y = (int)(idx / E), e = (int)(idx % E);
  const int tu = e >> 8, row = (e >> 4) & 15, cl = e & 15;
  const int t = tu / TJ, u = tu % TJ;
  const int gi = (y / nbj) * 16 * TI + t * 16 + row, gj = (y % nbj) * 16 * TJ + u * 16 + cl;
  if (gi < m1 && gj < m2) G[(i64)gi * m2 + gj] = tot;
}

namespace {
template <int TI, int TJ>
void panel_gram(eig_ctx_t ctx, i64 n, i64 ld, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G,
                hipStream_t s)
{
  const int nbi = (int)((m1 + 16 * TI - 1) / (16 * TI)), nbj = (int)((m2 + 16 * TJ - 1) / (16 * TJ));
  const int ny = nbi * nbj;
  EIG_CHECK(ny <= 65535, EIG_ERR_ARG, "panel gram: output too large");
  // about 1024 workgroups in total (4 waves each, row-group loop unrolled for loads in flight),
  // at most 256 per output block so that stage 2 stays short
  const int gx = (int)std::max<i64>(1, std::min<i64>(std::min(256, std::max(1, 1024 / ny)), (n + 255) / 256));
  const size_t E = (size_t)TI * TJ * 256;
  double *part = (double *)ctx_buffer(ctx, 5, (size_t)gx * ny * E * sizeof(double));
  hipLaunchKernelGGL((k_panel_gram_part<TI, TJ>), dim3(gx, ny), dim3(256), 0, s, n, ld, (int)m1, (int)m2, nbj, Q1, Q2,
                     part);
  EIG_HIP(hipGetLastError());
  hipLaunchKernelGGL((k_panel_gram_reduce<TI, TJ>), dim3((unsigned)(((i64)ny * E + 63) / 64)), dim3(256), 0, s, gx, ny,
                     nbj, (int)m1, (int)m2, part, G);
  EIG_HIP(hipGetLastError());
}
}  // namespace

void launch_panel_gram(eig_ctx_t ctx, i64 n, i64 ld, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G,
                       hipStream_t s)
{
  if (m1 <= 32)
    panel_gram<2, 2>(ctx, n, ld, m1, m2, Q1, Q2, G, s);
  else
    panel_gram<4, 2>(ctx, n, ld, m1, m2, Q1, Q2, G, s);
}

// ---------------------------------------------------------------------------------------------
// Y = beta Y + alpha Q S: Q n x m1, S m1 x m2 (row-major, device), m2 = 8 NB2 <= 32.  One thread
// per row, all m2 columns in registers; S is read with uniform addresses (scalar loads, SGPR
// operands of v_fma_f64).  Per output column: acc = sum_k q_k S[k][j] with k ascending (fused
// multiply-add), then y = alpha acc (beta == 0: Y is not read) or beta y + alpha acc.  In place
// (Y == Q) is allowed: a row is fully read before it is written.
// ---------------------------------------------------------------------------------------------
template <int NB2>
__global__ __launch_bounds__(256) void k_panel_update(i64 n, i64 ldq, i64 ldy, int m1, const double *Q,
                                                      const double *__restrict__ S, double alpha, double beta,
                                                      double *Y)
{
  constexpr int M2 = 8 * NB2;
  for (i64 r = (i64)blockIdx.x * 256 + threadIdx.x; r < n; r += (i64)gridDim.x * 256)
  {
    double acc[M2];
#pragma unroll
    for (int j = 0; j < M2; ++j) acc[j] = 0.0;
    const int kb_n = m1 >> 3;
    for (int kb = 0; kb < kb_n; ++kb)
    {
      const double2 *qr = reinterpret_cast<const double2 *>(Q + ((i64)kb * ldq + r) * 8);
      double q[8];
#pragma unroll
      for (int h = 0; h < 4; ++h)
      {
        const double2 v = qr[h];
        q[2 * h] = v.x;
        q[2 * h + 1] = v.y;
      }
      const double *Sk = S + (i64)kb * 8 * M2;
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int j = 0; j < M2; ++j) acc[j] = __builtin_fma(q[k], Sk[k * M2 + j], acc[j]);
    }
#pragma unroll
    for (int ob = 0; ob < NB2; ++ob)
    {
      double2 *yr = reinterpret_cast<double2 *>(Y + ((i64)ob * ldy + r) * 8);
      if (beta == 0.0)
      {
#pragma unroll
        for (int h = 0; h < 4; ++h)
          yr[h] = make_double2(alpha * acc[ob * 8 + 2 * h], alpha * acc[ob * 8 + 2 * h + 1]);
      }
      else
      {
#pragma unroll
        for (int h = 0; h < 4; ++h)
        {
          const double2 y = yr[h];
          yr[h] = make_double2(beta * y.x + alpha * acc[ob * 8 + 2 * h], beta * y.y + alpha * acc[ob * 8 + 2 * h + 1]);
        }
      }
    }
  }
}

void launch_panel_update(i64 n, i64 ldq, i64 ldy, i64 m1, i64 m2, const double *Q, const double *S, double alpha,
                         double beta, double *Y, hipStream_t s)
{
  EIG_CHECK(m1 % 8 == 0 && m2 % 8 == 0 && m2 >= 8 && m2 <= 32, EIG_ERR_ARG,
            "panel update: m1 % 8 == 0 and m2 in {8, 16, 24, 32}");
  if (n <= 0 || m1 <= 0) return;
  const int g = grid_cap(n, 256, kStreamBlocks);
  switch (m2 / 8)
  {
    case 1: hipLaunchKernelGGL(k_panel_update<1>, dim3(g), dim3(256), 0, s, n, ldq, ldy, (int)m1, Q, S, alpha, beta, Y); break;
    case 2: hipLaunchKernelGGL(k_panel_update<2>, dim3(g), dim3(256), 0, s, n, ldq, ldy, (int)m1, Q, S, alpha, beta, Y); break;
    case 3: hipLaunchKernelGGL(k_panel_update<3>, dim3(g), dim3(256), 0, s, n, ldq, ldy, (int)m1, Q, S, alpha, beta, Y); break;
    default: hipLaunchKernelGGL(k_panel_update<4>, dim3(g), dim3(256), 0, s, n, ldq, ldy, (int)m1, Q, S, alpha, beta, Y); break;
  }
  EIG_HIP(hipGetLastError());
}

}  // namespace eigmi
