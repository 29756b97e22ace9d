// k_mv8.hip -- MultiVector<double,8> kernels (gfx950): SpMM, column dots, the tall-skinny Gram
// panel on MFMA, and the building blocks of block Gram-Schmidt / B-Gram-Schmidt.
//
// Layout is the reference's block-column-major MultiVector<double,8> (multivector.hh:130-139):
// column block b of an n x m multivector is n rows of 8 contiguous doubles (64 B) starting at
// Q + b*8*n.  Kernels keep the reference's per-element operation order wherever the result is
// not a reduction, so SpMM / projections are bitwise the reference arithmetic on equal inputs.
#include <algorithm>

#include <cstdlib>

#include "internal.h"
#include "reduce_dev.h"

namespace eigmi {

typedef double d4 __attribute__((ext_vector_type(4)));

static inline int grid_for(i64 work, i64 per_block, int cap)
{
  i64 g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

// ---------------------------------------------------------------------------------------------
// a2: Qout = A Qin (matmul_sparse_tallskinny_blocked, kernels_cpp.hh:626-657).
// A workgroup (4 waves) takes one 64-row SELL slice at a time; lane L of wave w handles row
// 16 w + L/4 of the slice and the column pair 2 (L%4), 2 (L%4)+1 (16-B loads of Qin rows) for up
// to MB column blocks, so the matrix slice is read once for MB column blocks.
// ---------------------------------------------------------------------------------------------
template <int MB>
__global__ __launch_bounds__(256) void k_spmm_mv8(i64 nrows, i64 nslices, const i64 *__restrict__ slice_ptr,
                                                  const double *__restrict__ val, const i32 *__restrict__ col,
                                                  const double *__restrict__ Qin, double *__restrict__ Qout, i64 n,
                                                  int nblk_total, int C)
{
  const int wave = threadIdx.x >> 6, L = threadIdx.x & 63;
  const int cp = L & 3;
  const int b0 = blockIdx.y * MB;
  const i64 nsub = (i64)nslices * (C / 64);  // 64-row sub-slices
  for (i64 ss = blockIdx.x; ss < nsub; ss += gridDim.x)
  {
    const i64 s = ss / (C / 64);
    const int ri = (int)(ss % (C / 64)) * 64 + wave * 16 + (L >> 2);
    const i64 base = slice_ptr[s];
    const int width = (int)((slice_ptr[s + 1] - base) / C);
    double2 acc[MB];
#pragma unroll
    for (int q = 0; q < MB; ++q) acc[q] = make_double2(0.0, 0.0);
    for (int k = 0; k < width; ++k)
    {
      const i32 c = col[base + (i64)k * C + ri];
      if (c < 0) continue;
      const double a = val[base + (i64)k * C + ri];
#pragma unroll
      for (int q = 0; q < MB; ++q)
      {
        if (b0 + q < nblk_total)
        {
          const double2 xv = *reinterpret_cast<const double2 *>(Qin + ((i64)(b0 + q) * n + c) * 8 + 2 * cp);
          acc[q].x += a * xv.x;
          acc[q].y += a * xv.y;
        }
      }
    }
    const i64 r = s * C + ri;
    if (r < nrows)
    {
#pragma unroll
      for (int q = 0; q < MB; ++q)
        if (b0 + q < nblk_total) *reinterpret_cast<double2 *>(Qout + ((i64)(b0 + q) * n + r) * 8 + 2 * cp) = acc[q];
    }
  }
}

void launch_spmm_mv8(const eig_mat_s &A, i64 m, const double *Qin, double *Qout, hipStream_t s)
{
  EIG_CHECK(A.br == 1 && A.bc == 1, EIG_ERR_BLOCKSIZE,
            "matmul_sparse_tallskinny_blocked: only implemented for FieldMatrix<..,1,1>");
  const int nblk = (int)(m / 8);
  if (A.R == 1)
  {
    // row per lane over 64-row slices, window layout (k_block.hip); ld = n on one rank
    launch_sell_mv8(A, m, Qin, Qout, s);
    return;
  }
  const int MB = 4;
  const int gy = (nblk + MB - 1) / MB;
  const int gx = grid_for(A.nslices * A.R, 1, kStreamBlocks);
  // Qin is a window-layout multivector on one rank (window == n); columns index it directly.
  hipLaunchKernelGGL(k_spmm_mv8<MB>, dim3(gx, gy), dim3(256), 0, s, A.nb_rows, A.nslices, A.slice_ptr, A.val, A.col,
                     Qin, Qout, A.nb_rows, nblk, 64 * A.R);
}

void launch_spmm_dot_mv8(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, hipStream_t s,
                         ReduceWS red)
{
  static const bool off = std::getenv("EIGMI_NO_SPMM_DOT") != nullptr;  // A/B: the two launches
  // the same kernel choice as launch_spmm_mv8 -> launch_sell_mv8 (box first, then the band march)
  if (!off && A.R == 1 && A.br == 1 && A.bc == 1)
  {
    if (launch_box_spmm_dot(A, m, X, Y, dp, red, s)) return;
    if (!box_spmm_applies(A, m) && launch_spmm_march_dot(A, m, X, Y, dp, red, s)) return;
  }
  launch_spmm_mv8(A, m, X, Y, s);
  launch_dot_diag_mv8(A.nb_rows, m, X, Y, dp, 0, s, red);
}

bool launch_spmm_dot_gram_mv8(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, double *gram,
                              hipStream_t s, ReduceWS red)
{
  if (m != 8 || A.R != 1 || A.br != 1 || A.bc != 1 || A.ctx->distributed()) return false;
  // the same kernel choice as launch_spmm_dot_mv8 (the row-class box kernel, else the band march);
  // the kernel's last workgroup also zeroes the look-ahead MGS's barrier word, so the MGS of this
  // block that follows (launch_mgs_lookahead_gram with this gram) needs no extra launch
  unsigned *bar = mgs_lookahead_barrier(A.ctx);
  const bool ok = launch_box_spmm_dot_gram(A, m, X, Y, dp, gram, red, s, bar) ||
                  (!box_spmm_applies(A, m) && launch_spmm_march_dot_gram(A, m, X, Y, dp, gram, red, s, bar));
  A.ctx->mgs_bar_clean = ok ? gram : nullptr;
  return ok;
}

// ---------------------------------------------------------------------------------------------
// a5: dp[j] = q1_j . q2_j (dot_products_diagonal_blocked, kernels_cpp.hh:24-55).  grid.y = column
// block; thread t always sees the column pair 2 (t%4) because the grid stride is a multiple of 4.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kStreamThreads) void k_dot_diag_mv8(i64 n, const double *__restrict__ Q1,
                                                                 const double *__restrict__ Q2, double *dp,
                                                                 double *partials, unsigned *tickets)
{
  __shared__ double tot[8];
  const i64 off = (i64)blockIdx.y * n * 8;
  const double2 *a = reinterpret_cast<const double2 *>(Q1 + off);
  const double2 *b = reinterpret_cast<const double2 *>(Q2 + off);
  const i64 n4 = n * 4;
  double sx = 0.0, sy = 0.0;
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n4; i += (i64)gridDim.x * kStreamThreads)
  {
    const double2 x = a[i], y = b[i];
    sx += x.x * y.x;
    sy += x.y * y.y;
  }
  const int cp = threadIdx.x & 3;
  double v[8];
#pragma unroll
  for (int q = 0; q < 4; ++q)
  {
    v[2 * q] = (q == cp) ? sx : 0.0;
    v[2 * q + 1] = (q == cp) ? sy : 0.0;
  }
  if (grid_sum_n<8, kStreamThreads>(v, partials + (size_t)blockIdx.y * gridDim.x * 8, tickets + (size_t)blockIdx.y * kTicketStride, tot,
                                    blockIdx.x, gridDim.x))
  {
    if (threadIdx.x < 8) dp[blockIdx.y * 8 + threadIdx.x] = tot[threadIdx.x];
  }
}

void launch_dot_diag_mv8(i64 n, i64 m, const double *Q1, const double *Q2, double *dp, int ticket, hipStream_t s,
                         ReduceWS red)
{
  const int nb = (int)(m / 8);
  EIG_CHECK(ticket + nb <= kNumTickets, EIG_ERR_ARG, "dot_diag_mv8: too many column blocks");
  int G = grid_for(n * 4, (i64)kStreamThreads * 4, 1024);
  while ((i64)G * nb * 8 > (i64)kMaxRedBlocks * kMaxRedVals) G /= 2;
  hipLaunchKernelGGL(k_dot_diag_mv8, dim3(G, nb), dim3(kStreamThreads), 0, s, n, Q1, Q2, dp, red.partials,
                     red.ticket(ticket));
}

// ---------------------------------------------------------------------------------------------
// a6: G = Q1^T Q2 on MFMA (dot_products_all_blocked, kernels_cpp.hh:58-96), v_mfma_f64_16x16x4f64.
//
// The MFMA tile is 16 columns wide, a MultiVector column block 8.  Two operand forms, neither with
// padding lanes (lane l: k = l>>4, i = l&15; one 8-B load per lane and operand, 512 contiguous
// bytes per wave instruction):
//  * doubled rows (DR = 1; any block count): a "unit" is ONE block and a tile takes 8 ROWS,
//    A[i][k] = Q1(8g + k + 4 (i>>3), i & 7), B[k][j] = Q2(8g + k + 4 (j>>3), j & 7); the products
//    with i>>3 == j>>3 are the two 8x8 quadrants on the tile diagonal (rows 8g..8g+3 and
//    8g+4..8g+7) and the block of G is their sum (the off-diagonal quadrants are discarded);
//  * paired blocks (DR = 0; even block counts): a unit is TWO blocks side by side and a tile takes
//    4 rows, A[i][k] = Q1(4g + k, 16 u + i) -- the whole 16 x 16 tile is output.
// A workgroup takes T1 units of Q1 x T2 units of Q2 over its rows (each operand loaded once for
// T2 / T1 MFMAs: T1 x T2 independent accumulator chains), U row groups per wave iteration with all
// loads issued before the MFMAs; grid.y = chunks of the unit grid (each panel streams once per
// chunk of the other).  Column blocks sit ld rows apart (ld = n for a plain MultiVector, the
// window for the block Lanczos panels).  Reduction: (DR) quadrants folded by a lane shuffle, the 4
// waves summed in LDS, then grid_sum2 across workgroups (two-level, deterministic).
// ---------------------------------------------------------------------------------------------
constexpr int kGramThreads = 256;

template <int DR, int T1, int T2, int U>
__global__ __launch_bounds__(kGramThreads) void k_gram_mv8(i64 n, i64 ld1, i64 ld2, int nb1, int nb2, int ny2, int ny,
                                                           const double *__restrict__ Q1, const double *__restrict__ Q2,
                                                           double *__restrict__ G, double *partials, unsigned *tickets)
{
  constexpr int TE = DR ? 64 : 256;  // output elements per unit pair
  constexpr int E = T1 * T2 * TE;
  constexpr int W = kGramThreads / 64;
  constexpr int RG = DR ? 8 : 4;     // rows per group (one MFMA per unit pair)
  __shared__ double red[E];  // the workgroup's sum of its waves' tiles, then the grid total
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // 1-D grid of gx * ny workgroups (gx a multiple of 8), XCD-aware: workgroups are dealt round-robin
  // over the 8 XCDs, so b, b + 8, b + 16, ... share an XCD; they take the ny output chunks of ONE row
  // range (chunk fastest), run together and read each operand panel's rows once from HBM -- the
  // other chunks' re-reads of it are hits in that XCD's L2
  const int bq = blockIdx.x >> 3;
  const int cy = bq % ny, bx = (bq / ny) * 8 + (blockIdx.x & 7);
  const int gxw = gridDim.x / ny;  // workgroups per chunk
  const int cy1 = cy / ny2, cy2 = cy % ny2;
  const int k = lane >> 4, i = lane & 15;
  const int rl = DR ? k + 4 * (i >> 3) : k;  // row inside the group
  const double *a[T1];
  const double *b[T2];
  bool aok[T1], bok[T2];
#pragma unroll
  for (int t = 0; t < T1; ++t)
  {
    const int blk = DR ? cy1 * T1 + t : 2 * (cy1 * T1 + t) + (i >> 3);
    aok[t] = blk < nb1;
    a[t] = Q1 + (aok[t] ? blk : 0) * ld1 * 8 + (i & 7);
  }
#pragma unroll
  for (int u = 0; u < T2; ++u)
  {
    const int blk = DR ? cy2 * T2 + u : 2 * (cy2 * T2 + u) + (i >> 3);
    bok[u] = blk < nb2;
    b[u] = Q2 + (bok[u] ? blk : 0) * ld2 * 8 + (i & 7);
  }
  d4 acc[T1][T2];
#pragma unroll
  for (int t = 0; t < T1; ++t)
#pragma unroll
    for (int u = 0; u < T2; ++u) acc[t][u] = d4{0.0, 0.0, 0.0, 0.0};
  const i64 ng = (n + RG - 1) / RG;
  const i64 ws = (i64)gxw * W;
  for (i64 g0 = (i64)bx * W + wave; g0 < ng; g0 += U * ws)
  {
    double av[U][T1], bv[U][T2];
#pragma unroll
    for (int v = 0; v < U; ++v)
    {
      const i64 r = (g0 + v * ws) * RG + rl;
      const bool ok = r < n;  // (also false for groups past ng)
      const i64 rr = ok ? r : 0;
#pragma unroll
      for (int t = 0; t < T1; ++t) av[v][t] = a[t][rr * 8];
#pragma unroll
      for (int u = 0; u < T2; ++u) bv[v][u] = b[u][rr * 8];
#pragma unroll
      for (int t = 0; t < T1; ++t) av[v][t] = (ok && aok[t]) ? av[v][t] : 0.0;
#pragma unroll
      for (int u = 0; u < T2; ++u) bv[v][u] = (ok && bok[u]) ? bv[v][u] : 0.0;
    }
#pragma unroll
    for (int v = 0; v < U; ++v)
#pragma unroll
      for (int t = 0; t < T1; ++t)
#pragma unroll
        for (int u = 0; u < T2; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[v][t], bv[v][u], acc[t][u], 0, 0, 0);
  }
  // lane holds C[k + 4q][i] of each tile.  The waves add their tiles into one LDS image in wave
  // order (((w0 + w1) + w2) + w3: a fixed order, E doubles of LDS instead of W E)
  for (int w = 0; w < W; ++w)
  {
    if (wave == w)
    {
#pragma unroll
      for (int t = 0; t < T1; ++t)
#pragma unroll
        for (int u = 0; u < T2; ++u)
        {
          if constexpr (DR)
          {
            // for i < 8, q < 2: C[k + 4q][i] + C[k + 4q + 8][i + 8] (lane + 8, register q + 2)
#pragma unroll
            for (int q = 0; q < 2; ++q)
            {
              const double hi = __shfl_down(acc[t][u][q + 2], 8, 64);
              const int e = (t * T2 + u) * 64 + (k + 4 * q) * 8 + i;
              if (i < 8) red[e] = w == 0 ? acc[t][u][q] + hi : red[e] + (acc[t][u][q] + hi);
            }
          }
          else
          {
#pragma unroll
            for (int q = 0; q < 4; ++q)
            {
              const int e = (t * T2 + u) * 256 + (k + 4 * q) * 16 + i;
              red[e] = w == 0 ? acc[t][u][q] : red[e] + acc[t][u][q];
            }
          }
        }
    }
    __syncthreads();
  }
  double *part = partials + (size_t)cy * gxw * E;
  double *spart = partials + (size_t)ny * gxw * E + (size_t)cy * 8 * E;
  if (!grid_sum2<kGramThreads>(red, E, part, spart, tickets + (size_t)cy * kTicketStride, bx, gxw, red)) return;
  const i64 m1 = (i64)nb1 * 8, m2 = (i64)nb2 * 8;
  for (int e = threadIdx.x; e < E; e += kGramThreads)
  {
    const int tu = e / TE, t = tu / T2, u = tu % T2, el = e % TE;
    const int TW = DR ? 8 : 16;  // tile width in G
    const i64 row = (i64)(cy1 * T1 + t) * TW + el / TW, col = (i64)(cy2 * T2 + u) * TW + el % TW;
    if (row < m1 && col < m2) G[row * m2 + col] = red[e];
  }
}

namespace {
struct GramShape {
  int dr, t1, t2, ny1, ny2;
};
// Operand form and unit tiling of an m1 x m2 Gram: paired blocks when both block counts are even
// (full tiles), doubled rows otherwise; up to 4 x 4 units (doubled) or 4 x 2 pairs per workgroup.
GramShape gram_shape(i64 m1, i64 m2)
{
  const int nb1 = (int)(m1 / 8), nb2 = (int)(m2 / 8);
  GramShape g;
  g.dr = (nb1 % 2 || nb2 % 2) ? 1 : 0;
  const int u1 = std::max(1, g.dr ? nb1 : nb1 / 2), u2 = std::max(1, g.dr ? nb2 : nb2 / 2);
  // at most 4 x 4 units (doubled) / 4 x 2 pairs per workgroup, chunks of equal size
  const int max1 = 4, max2 = g.dr ? 4 : 2;
  g.ny1 = (u1 + max1 - 1) / max1;
  g.ny2 = (u2 + max2 - 1) / max2;
  g.t1 = (u1 + g.ny1 - 1) / g.ny1;
  g.t2 = (u2 + g.ny2 - 1) / g.ny2;
  return g;
}

template <int DR, int T1, int T2>
void gram_launch(i64 n, i64 ld1, i64 ld2, int nb1, int nb2, const GramShape &gs, const double *Q1, const double *Q2,
                 double *G, unsigned *tickets, double *partials, i64 cap, hipStream_t s)
{
  constexpr int U = (T1 + T2) <= 2 ? 8 : (T1 + T2) <= 4 ? 4 : 2;
  constexpr int E = T1 * T2 * (DR ? 64 : 256);
  const int ny = gs.ny1 * gs.ny2;
  const i64 ng = (n + (DR ? 7 : 3)) / (DR ? 8 : 4);
  // about 4 resident workgroups per CU in all, at least one U-group batch per wave; gx a multiple
  // of 8 (the kernel's XCD mapping)
  i64 gx = std::min<i64>(std::max<i64>(8, 1024 / ny), std::max<i64>(1, (ng + 4 * U - 1) / (4 * U)));
  gx = (gx + 7) / 8 * 8;
  while ((gx * ny + 8 * ny) * E > cap && gx > 8) gx -= 8;
  EIG_CHECK((gx * ny + 8 * ny) * E <= cap, EIG_ERR_ARG, "gram: output too large for the reduction workspace");
  hipLaunchKernelGGL((k_gram_mv8<DR, T1, T2, U>), dim3((unsigned)(gx * ny)), dim3(kGramThreads), 0, s, n, ld1, ld2,
                     nb1, nb2, gs.ny2, ny, Q1, Q2, G, partials, tickets);
}

void gram_dispatch(i64 n, i64 ld1, i64 ld2, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G,
                   unsigned *tickets, double *partials, i64 cap, hipStream_t s)
{
  EIG_CHECK(m1 > 0 && m2 > 0 && m1 % 8 == 0 && m2 % 8 == 0, EIG_ERR_ARG, "gram_mv8: m1, m2 multiples of 8");
  const int nb1 = (int)(m1 / 8), nb2 = (int)(m2 / 8);
  const GramShape gs = gram_shape(m1, m2);
#define EIG_GRAM(D_, A_, B_)                                                                           \
  if (gs.dr == D_ && gs.t1 == A_ && gs.t2 == B_)                                                       \
  {                                                                                                    \
    gram_launch<D_, A_, B_>(n, ld1, ld2, nb1, nb2, gs, Q1, Q2, G, tickets, partials, cap, s);          \
    EIG_HIP(hipGetLastError());                                                                        \
    return;                                                                                            \
  }
  EIG_GRAM(1, 1, 1) EIG_GRAM(1, 1, 2) EIG_GRAM(1, 1, 3) EIG_GRAM(1, 1, 4)
  EIG_GRAM(1, 2, 1) EIG_GRAM(1, 2, 2) EIG_GRAM(1, 2, 3) EIG_GRAM(1, 2, 4)
  EIG_GRAM(1, 3, 1) EIG_GRAM(1, 3, 2) EIG_GRAM(1, 3, 3) EIG_GRAM(1, 3, 4)
  EIG_GRAM(1, 4, 1) EIG_GRAM(1, 4, 2) EIG_GRAM(1, 4, 3) EIG_GRAM(1, 4, 4)
  EIG_GRAM(0, 1, 1) EIG_GRAM(0, 1, 2) EIG_GRAM(0, 2, 1) EIG_GRAM(0, 2, 2) EIG_GRAM(0, 3, 1) EIG_GRAM(0, 3, 2)
  EIG_GRAM(0, 4, 1) EIG_GRAM(0, 4, 2)
#undef EIG_GRAM
  throw Error(EIG_ERR_ARG, "gram: no kernel for this shape");
}
}  // namespace

int gram_mv8_chunks(i64 m1, i64 m2)
{
  const GramShape gs = gram_shape(m1, m2);
  return gs.ny1 * gs.ny2;
}

void launch_gram_mv8(i64 n, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G, int ticket,
                     hipStream_t s, ReduceWS red)
{
  EIG_CHECK(ticket + gram_mv8_chunks(m1, m2) <= kNumTickets, EIG_ERR_ARG, "gram_mv8: too many output chunks");
  gram_dispatch(n, n, n, m1, m2, Q1, Q2, G, red.ticket(ticket), red.partials, (i64)kMaxRedBlocks * kMaxRedVals, s);
}

// Window-layout panels (block Lanczos, blanczos.cpp): column blocks ld rows apart; partials in a
// context buffer sized for the launch, tickets from the context pool (the panel products run alone
// on the stream, like every other reduction)
void launch_gram_panel(eig_ctx_t ctx, i64 n, i64 ld, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G,
                       hipStream_t s)
{
  const int chunks = gram_mv8_chunks(m1, m2);
  EIG_CHECK(chunks <= kNumTickets, EIG_ERR_ARG, "panel gram: too many output chunks");
  const GramShape gs = gram_shape(m1, m2);
  const i64 E = (i64)gs.t1 * gs.t2 * (gs.dr ? 64 : 256);
  const i64 cap = (std::max<i64>(8, 1024 / chunks) + 8 + 8) * (i64)chunks * E;
  double *part = (double *)ctx_buffer(ctx, 8, (size_t)cap * sizeof(double));  // slot 8: panel partials
  gram_dispatch(n, ld, ld, m1, m2, Q1, Q2, G, ctx->red.ticket(0), part, cap, s);
}

// ---------------------------------------------------------------------------------------------
// a9 diagonal block, fused column MGS (kernels_cpp.hh:202-229).  Pass k (0..8) over the n x 8
// block Qb, four lanes per row.  Ssum (8x8) holds the RAW sums s[k][j] = q_k . q_j of each pass
// (so a distributed run can allreduce them between passes); pass k first finalises row k-1
// exactly like the reference,  S[k-1][j] = s/s[k-1][k-1] (j > k-1), S[k-1][k-1] = 1/sqrt(s),
// then applies it:  q_j -= S[k-1][j] q_{k-1} (j > k-1), q_{k-1} *= S[k-1][k-1], and (k < 8)
// accumulates the new sums s[k][j] (j >= k) on the updated row.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kStreamThreads) void k_mgs_pass(i64 n, double *__restrict__ Qb, int k,
                                                             double *__restrict__ Ssum, double *partials,
                                                             unsigned *ticket)
{
  // quad mapping: 4 lanes per row, lane ql holds columns 2 ql, 2 ql + 1 (one 16-B load: a wave
  // instruction reads 16 whole 64-B rows); the pivot columns are broadcast inside the quad
  __shared__ double tot[8];
  const int ql = threadIdx.x & 3;
  const int c0 = 2 * ql, c1 = c0 + 1;
  const int qbase = (threadIdx.x & 63) & ~3;
  double sp0 = 0.0, sp1 = 0.0;  // this lane's S[k-1][c] (0 for c < k-1, 1/sqrt for c = k-1)
  const int kp = k - 1;
  if (k > 0)
  {
    const double skk = Ssum[kp * 8 + kp];
    sp0 = (c0 > kp) ? Ssum[kp * 8 + c0] / skk : ((c0 == kp) ? 1.0 / sqrt(skk) : 0.0);
    sp1 = (c1 > kp) ? Ssum[kp * 8 + c1] / skk : ((c1 == kp) ? 1.0 / sqrt(skk) : 0.0);
  }
  double a0 = 0.0, a1 = 0.0;
  const i64 stride = (i64)gridDim.x * (kStreamThreads / 4);
  for (i64 i = ((i64)blockIdx.x * kStreamThreads + threadIdx.x) >> 2; i < n; i += stride)
  {
    double2 *row = reinterpret_cast<double2 *>(Qb + i * 8) + ql;
    double2 v = *row;
    if (k > 0)
    {
      // q_j -= S[kp][j] q_kp (j > kp) with the OLD q_kp, then q_kp *= S[kp][kp]
      const double qkp = __shfl((kp & 1) ? v.y : v.x, qbase + (kp >> 1), 64);
      if (c0 > kp) v.x -= sp0 * qkp;
      if (c1 > kp) v.y -= sp1 * qkp;
      if (c0 == kp) v.x *= sp0;
      if (c1 == kp) v.y *= sp1;
      *row = v;
    }
    if (k < 8)
    {
      const double qk = __shfl((k & 1) ? v.y : v.x, qbase + (k >> 1), 64);
      if (c0 >= k) a0 += qk * v.x;
      if (c1 >= k) a1 += qk * v.y;
    }
  }
  if (k >= 8) return;
  double vals[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) vals[j] = (j == c0) ? a0 : ((j == c1) ? a1 : 0.0);
  if (grid_sum<8, kStreamThreads>(vals, partials, ticket, tot))
  {
    if (threadIdx.x < 8) Ssum[k * 8 + threadIdx.x] = (threadIdx.x >= (unsigned)k) ? tot[threadIdx.x] : 0.0;
  }
}

// ---------------------------------------------------------------------------------------------
// The same MGS with read-only passes (the default): pass K reads the ORIGINAL block and replays
// the row updates of steps 0 .. K-1 in registers (the S coefficients of every finished step come
// from Ssum) before the sums of step K -- per row exactly the operations, in the same order, that
// the in-place passes above apply one per launch.
// Only pass 8 writes the block.  Traffic: 9 reads + 1 write of the n x 8 block instead of 9 reads
// + 9 writes, and the unmodified block stays resident in the 256 MB memory-side cache (MALL) across
// the passes wherever it fits (plain loads and stores, no streaming hints).  (The rows a lane sums
// differ from the in-place passes', so the sums agree to rounding, not bitwise.)
// ---------------------------------------------------------------------------------------------
// Lane P of each quad (4 lanes = one row) broadcast to the quad: a DPP quad_perm move (VALU, no LDS
// traffic), two 32-bit halves.
template <int P>
__device__ __forceinline__ double quad_bcast(double v)
{
  constexpr int ctrl = P | (P << 2) | (P << 4) | (P << 6);  // quad_perm [P, P, P, P]
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), ctrl, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Steps KP .. K-1 of the row update on one lane's two columns (compile-time pivot: DPP control)
template <int KP, int K, int N>
__device__ __forceinline__ void mgs_replay_steps(double2 &v, const double (&sp0)[N], const double (&sp1)[N], int c0,
                                                 int c1)
{
  if constexpr (KP < K)
  {
    const double qkp = quad_bcast<(KP >> 1)>((KP & 1) ? v.y : v.x);
    if (c0 > KP) v.x -= sp0[KP] * qkp;
    if (c1 > KP) v.y -= sp1[KP] * qkp;
    if (c0 == KP) v.x *= sp0[KP];
    if (c1 == KP) v.y *= sp1[KP];
    mgs_replay_steps<KP + 1, K>(v, sp0, sp1, c0, c1);
  }
}

template <int K>
__global__ __launch_bounds__(kStreamThreads) void k_mgs_replay(i64 n, double *__restrict__ Qb,
                                                               double *__restrict__ Ssum, double *partials,
                                                               unsigned *ticket)
{
  // quad mapping as k_mgs_pass (4 lanes per row, lane ql holds columns 2 ql, 2 ql + 1: one 16-B
  // load), the pivot column broadcast inside the quad by DPP instead of LDS shuffles
  __shared__ double tot[8];
  const int ql = threadIdx.x & 3;
  const int c0 = 2 * ql, c1 = c0 + 1;
  double sp0[K > 0 ? K : 1], sp1[K > 0 ? K : 1];  // this lane's S[kp][c] of every finished step kp
#pragma unroll
  for (int kp = 0; kp < K; ++kp)
  {
    const double skk = Ssum[kp * 8 + kp];
    sp0[kp] = (c0 > kp) ? Ssum[kp * 8 + c0] / skk : ((c0 == kp) ? 1.0 / sqrt(skk) : 0.0);
    sp1[kp] = (c1 > kp) ? Ssum[kp * 8 + c1] / skk : ((c1 == kp) ? 1.0 / sqrt(skk) : 0.0);
  }
  double a0 = 0.0, a1 = 0.0;
  constexpr int U = 8;  // rows per lane per round, loads issued together
  const i64 stride = (i64)gridDim.x * (kStreamThreads / 4);
  for (i64 i0 = ((i64)blockIdx.x * kStreamThreads + threadIdx.x) >> 2; i0 < n; i0 += U * stride)
  {
    double2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const i64 i = i0 + u * stride;
      v[u] = i < n ? reinterpret_cast<const double2 *>(Qb + i * 8)[ql] : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      // q_j -= S[kp][j] q_kp (j > kp) with the old q_kp, then q_kp *= S[kp][kp] (kernels_cpp.hh:218-228)
      mgs_replay_steps<0, K>(v[u], sp0, sp1, c0, c1);
      if constexpr (K == 8)
      {
        const i64 i = i0 + u * stride;
        if (i < n) reinterpret_cast<double2 *>(Qb + i * 8)[ql] = v[u];
      }
      else
      {
        // (rows past n are zero: they add nothing)
        const double qk = quad_bcast<(K >> 1)>((K & 1) ? v[u].y : v[u].x);
        if (c0 >= K) a0 += qk * v[u].x;
        if (c1 >= K) a1 += qk * v[u].y;
      }
    }
  }
  if constexpr (K < 8)
  {
    double vals[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) vals[j] = (j == c0) ? a0 : ((j == c1) ? a1 : 0.0);
    if (grid_sum<8, kStreamThreads>(vals, partials, ticket, tot))
    {
      if (threadIdx.x < 8) Ssum[K * 8 + threadIdx.x] = (threadIdx.x >= (unsigned)K) ? tot[threadIdx.x] : 0.0;
    }
  }
}

void launch_mgs_pass(i64 n, double *Qb, int k, double *Ssum, int ticket, hipStream_t s, ReduceWS red)
{
  int G = grid_for(n * 4, kStreamThreads * 4, 1024);
  static const bool inplace = std::getenv("EIGMI_MGS_INPLACE") != nullptr;  // (A/B measurements)
  if (inplace)
  {
    hipLaunchKernelGGL(k_mgs_pass, dim3(G), dim3(kStreamThreads), 0, s, n, Qb, k, Ssum, red.partials,
                       red.ticket(ticket));
    return;
  }
  // read-only passes: fewer, longer-lived workgroups with 8 rows per lane in flight (the reduction
  // tail and the prologue amortised over more rows)
  static const int gmax = [] {
    const char *e = std::getenv("EIGMI_MGS_GRID");
    return e ? std::max(64, std::atoi(e)) : 512;
  }();
  G = grid_for(n * 4, kStreamThreads * 4, gmax);
#define EIG_MGS_K(K_)                                                                                        \
  case K_:                                                                                                   \
    hipLaunchKernelGGL(k_mgs_replay<K_>, dim3(G), dim3(kStreamThreads), 0, s, n, Qb, Ssum, red.partials,     \
                       red.ticket(ticket));                                                                  \
    break;
  switch (k)
  {
    EIG_MGS_K(0) EIG_MGS_K(1) EIG_MGS_K(2) EIG_MGS_K(3) EIG_MGS_K(4) EIG_MGS_K(5) EIG_MGS_K(6) EIG_MGS_K(7)
    EIG_MGS_K(8)
    default:
      throw Error(EIG_ERR_ARG, "mgs pass: k outside 0..8");
  }
#undef EIG_MGS_K
}

// ---------------------------------------------------------------------------------------------
// The read-only MGS passes in ONE cooperative launch (one rank, opt-in: EIGMI_MGS_COOP=1): every
// workgroup stays resident through the 9 passes, and a pass ends in a grid barrier instead of a
// kernel boundary and a last-workgroup tail.  Each workgroup stores its 8 block sums (write-through),
// arrives at the barrier, and after it EVERY workgroup sums the grid's partials itself, in the same
// fixed order (so all hold the bitwise same row of S; workgroup 0 also stores it to Ssum for the
// host).  Rows and per-row operations as k_mgs_replay.  Needs all workgroups co-resident
// (hipLaunchCooperativeKernel refuses the launch otherwise and the per-pass launches run); the
// barrier spin is bounded (1 s of s_memrealtime: err = 1, and the host falls back) so a broken
// co-residency promise cannot hang the GPU.
// ---------------------------------------------------------------------------------------------
constexpr unsigned long long kMgsBarrierTimeout = 100000000ull;

// grid barrier number b (1, 2, ...) of the launch on a counter zeroed before it
__device__ __forceinline__ bool mgs_grid_barrier(unsigned *bar, unsigned b, int *err)
{
  __shared__ int s_late;
  __syncthreads();  // (this workgroup's partial stores were drained by each storing thread)
  if (threadIdx.x == 0)
  {
    s_late = 0;
    // relaxed, as the grid reduction's ticket (reduce_dev.h): the partials went out write-through
    // and are read with coherent loads, so no release / acquire fence (at agent scope those write
    // back / invalidate the whole L2 of every XCD -- measured 2x slower per pass)
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = b * gridDim.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
    {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kMgsBarrierTimeout)
      {
        s_late = 1;
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  return s_late == 0;
}

__global__ __launch_bounds__(kStreamThreads) void k_mgs_coop(i64 n, double *__restrict__ Qb, double *__restrict__ Ssum,
                                                             double *__restrict__ partials, unsigned *bar, int *err)
{
  __shared__ double S[8][8];  // raw sums s[k][j] of the finished steps (bitwise the same in every workgroup)
  const int ql = threadIdx.x & 3;
  const int c0 = 2 * ql, c1 = c0 + 1;
  const i64 stride = (i64)gridDim.x * (kStreamThreads / 4);
  const i64 i00 = ((i64)blockIdx.x * kStreamThreads + threadIdx.x) >> 2;
  constexpr int U = 8;
  auto pass = [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    double sp0[K > 0 ? K : 1], sp1[K > 0 ? K : 1];
#pragma unroll
    for (int kp = 0; kp < K; ++kp)
    {
      const double skk = S[kp][kp];
      sp0[kp] = (c0 > kp) ? S[kp][c0] / skk : ((c0 == kp) ? 1.0 / sqrt(skk) : 0.0);
      sp1[kp] = (c1 > kp) ? S[kp][c1] / skk : ((c1 == kp) ? 1.0 / sqrt(skk) : 0.0);
    }
    double a0 = 0.0, a1 = 0.0;
    for (i64 i0 = i00; i0 < n; i0 += U * stride)
    {
      double2 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
      {
        const i64 i = i0 + u * stride;
        v[u] = i < n ? reinterpret_cast<const double2 *>(Qb + i * 8)[ql] : make_double2(0.0, 0.0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
      {
        mgs_replay_steps<0, K>(v[u], sp0, sp1, c0, c1);
        if constexpr (K == 8)
        {
          const i64 i = i0 + u * stride;
          if (i < n) reinterpret_cast<double2 *>(Qb + i * 8)[ql] = v[u];
        }
        else
        {
          const double qk = quad_bcast<(K >> 1)>((K & 1) ? v[u].y : v[u].x);
          if (c0 >= K) a0 += qk * v[u].x;
          if (c1 >= K) a1 += qk * v[u].y;
        }
      }
    }
    if constexpr (K < 8)
    {
      // block sums of the 8 values -> partials[block][8] (write-through), grid barrier, then every
      // workgroup sums all blocks' partials in block order
      double vals[8], bs[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) vals[j] = (j == c0) ? a0 : ((j == c1) ? a1 : 0.0);
      block_sum<8, kStreamThreads>(vals, bs);
      // two partial buffers by pass parity: pass K + 2's stores come after barrier K + 2, which every
      // workgroup reaches only after reading pass K's partials -- so pass K + 2 may reuse the buffer
      double *part = partials + (size_t)(K & 1) * gridDim.x * 8;
      if (threadIdx.x == 0)
      {
#pragma unroll
        for (int j = 0; j < 8; ++j) st_sc1(&part[(size_t)blockIdx.x * 8 + j], bs[j]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!mgs_grid_barrier(bar, K + 1, err)) return false;
      {
        // thread t: value j = t & 7 over the 16 blocks b = (t >> 3) + 32 u (all loads in one round
        // trip), then the 32 slices of value j summed in slice order through LDS (a fixed order:
        // identical in every workgroup).  G <= 512 blocks.
        __shared__ double sred[32][8];
        const int j = threadIdx.x & 7, sl = threadIdx.x >> 3;
        const unsigned G = gridDim.x;
        double t[16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
        {
          const unsigned b = (unsigned)sl + 32u * u;
          t[u] = b < G ? ld_sc1(&part[(size_t)b * 8 + j]) : 0.0;
        }
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += t[u];
        sred[sl][j] = acc;
        __syncthreads();
        if (threadIdx.x < 8)
        {
          double r = 0.0;
#pragma unroll
          for (int q = 0; q < 32; ++q) r += sred[q][threadIdx.x];
          r = (threadIdx.x >= (unsigned)K) ? r : 0.0;
          S[K][threadIdx.x] = r;
          if (blockIdx.x == 0) Ssum[K * 8 + threadIdx.x] = r;
        }
      }
      __syncthreads();
    }
    return true;
  };
  if (!pass(std::integral_constant<int, 0>{})) return;
  if (!pass(std::integral_constant<int, 1>{})) return;
  if (!pass(std::integral_constant<int, 2>{})) return;
  if (!pass(std::integral_constant<int, 3>{})) return;
  if (!pass(std::integral_constant<int, 4>{})) return;
  if (!pass(std::integral_constant<int, 5>{})) return;
  if (!pass(std::integral_constant<int, 6>{})) return;
  if (!pass(std::integral_constant<int, 7>{})) return;
  pass(std::integral_constant<int, 8>{});
}

// One cooperative launch of the 9 passes; false when the runtime refuses it (co-residency) or a
// barrier timed out -- the caller then runs the per-pass launches (Qb is written only by the last
// pass, after the last barrier, so a failed attempt leaves it untouched).
bool launch_mgs_coop(eig_ctx_t ctx, i64 n, double *Qb, double *Ssum, hipStream_t s)
{
  // opt-in (EIGMI_MGS_COOP=1): measured slower than the 9 launches -- 411 vs ~330 us of kernel time at
  // 128^3, m = 8 (profiles/r05m_ortho_*): the persistent passes stream at ~46 us each against ~33 us
  // for a fresh launch, which the saved launch gaps (~2 us each) do not repay
  static const bool on = std::getenv("EIGMI_MGS_COOP") != nullptr;
  if (!on || n <= 0) return false;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_mgs_coop, kStreamThreads, 0) != hipSuccess || per_cu < 1)
  {
    (void)hipGetLastError();
    return false;
  }
  const int G = std::min<int>({per_cu * ctx->num_cu, 512, grid_for(n * 4, kStreamThreads * 4, 512)});
  // scratch: 2 x G x 8 partials, the barrier counter, the error word (context buffer slot 10)
  char *buf = (char *)ctx_buffer(ctx, 10, (size_t)16 * G * 8 + 256);
  double *part = reinterpret_cast<double *>(buf);
  unsigned *bar = reinterpret_cast<unsigned *>(buf + (size_t)16 * G * 8);
  int *err = reinterpret_cast<int *>(buf + (size_t)16 * G * 8 + 128);
  EIG_HIP(hipMemsetAsync(bar, 0, 256, s));
  void *args[] = {&n, &Qb, &Ssum, &part, &bar, &err};
  if (hipLaunchCooperativeKernel(reinterpret_cast<const void *>(k_mgs_coop), dim3(G), dim3(kStreamThreads), args, 0,
                                 s) != hipSuccess)
  {
    (void)hipGetLastError();
    return false;
  }
  int e = 0;
  EIG_HIP(hipMemcpyAsync(&e, err, sizeof(int), hipMemcpyDeviceToHost, s));
  EIG_HIP(hipStreamSynchronize(s));
  return e == 0;
}

// ---------------------------------------------------------------------------------------------
// The same column MGS with Gram LOOK-AHEAD (the default on one rank; EIG_ORTHO_LOOKAHEAD(L)).
// A pass that starts with F finished steps replays them on each row (as k_mgs_replay) and sums,
// besides step F's own row  s[F][j] = q_F . q_j  (j >= F), the rows a = F+1 .. F+W-1 of the same
// Gram (W = min(L, 8 - F)).  The pass's tail then finishes step F exactly as the stepwise passes
// do, and steps F+1 .. from the Schur complement of the window: after step b the sums of the
// updated columns are  s'[a][j] = s[a][j] - (s[b][a] / s[b][b]) s[b][j]  -- in exact arithmetic the
// very sums the next stepwise pass would form, so ONE pass finishes up to W steps and m = 8 takes
// ceil(8 / L) read passes plus the write pass instead of 8 + 1.
// Rounding: every term of s' is bounded by |q_a| |q_j| of the window's columns (Cauchy-Schwarz), so
// the absolute error of s'[a][j] is O(W eps |q_a| |q_j|) where the stepwise pass has O(eps |q'_a|
// |q'_j|): relative to the step's own scale that is an amplification of 1/r with r = s'[a][a] /
// s[a][a], the fraction of q_a's squared norm left after projecting out the window's earlier
// columns.  A look-ahead step is taken only while r >= kMgsLaTau (1/16: at most 16 W eps, well inside
// the 1e-12 of the restatement); at the first column below it the pass stops and the next pass
// starts there with a DIRECT row, so nearly dependent columns get exactly the stepwise arithmetic.
// (The reference's own fast diagonal block, orthonormalize_avx2_b8_v2 (kernels_avx2.hh:385-622),
// is CholQR: the whole 8 x 8 Gram in one pass, ungated.)
// Layout: the read passes hold ONE ROW PER LANE (four 16-B loads; the window's <= 36 products per
// row with no cross-lane traffic), the write pass the quad layout of k_mgs_replay (coalesced 16-B
// stores).  Both replay a row with the same operations in the same order.
// Launches: ceil(8 / L) read launches (a ticketed tail finishes the window), then ONE last launch
// that writes the block -- and, only when a look-ahead was refused, first runs the missing read
// passes in-kernel between grid barriers (its grid fits the device at one workgroup per CU; bounded
// spins: on a timeout the workgroup poisons its rows with NaN and records the failure, so nothing
// hangs and nothing passes silently).  EIG_ORTHO_NO_COOP instead enqueues the worst case, 9
// launches, whose surplus ones only copy the state word forward.
// State (context scratch, slot 11): Sfin[8][8] the finished S rows (S[k][k] = 1/sqrt, S[k][j] =
// s'/s'[k][k], 0 below); words st[0..1] by launch parity (bits 0-3 F, bit 4 written, bits 8-15 read
// passes so far: launch l reads word l & 1, exactly one thread writes word (l + 1) & 1), st[2] the
// last call's final word, st[32] the last launch's barrier counter; the error flag is a host-mapped word
// (eig_ctx_s::mgs_err_dev, sticky until the host reads it at a synchronisation).
// ---------------------------------------------------------------------------------------------
constexpr int kMgsLaThreads = 512;
constexpr int kMgsLaGrid = 256;  // one workgroup per CU: the tails sum 256 x 8 W partials
constexpr double kMgsLaTau = 1.0 / 16;
constexpr unsigned kMgsLaWritten = 16u;
constexpr int kMgsLaBar = 32, kMgsLaLast = 2;  // st[] word indices

struct MgsLaArgs {
  i64 n;
  double *Qb;
  int launch;
  unsigned *st;
  double *Sfin;
  double *partials;
  unsigned *ticket;
  int *err;  // sticky error word (host-mapped: eig_ctx_s::mgs_err_dev)
};

template <int L>
struct MgsLaShared {
  double red[kMgsLaThreads / 64][8 * L];  // wave totals
  double fin[8][8 * L];                   // the tail's 8 slices
  double Rw[L][8];                        // the window's grid sums
  double S[64];                           // (last launch) the S rows
  unsigned word, last;
};

// Steps 0 .. F-1 on one row held whole (S rows wave-uniform): per element the operations of
// mgs_replay_steps, in its order -- q_j -= S[kp][j] q_kp (j > kp) with the old q_kp, then
// q_kp *= S[kp][kp] (kernels_cpp.hh:218-228)
template <int F>
__device__ __forceinline__ void mgs_row_replay(double (&q)[8], const double (&S)[F > 0 ? F : 1][8])
{
#pragma unroll
  for (int kp = 0; kp < F; ++kp)
  {
#pragma unroll
    for (int j = kp + 1; j < 8; ++j) q[j] -= S[kp][j] * q[kp];
    q[kp] *= S[kp][kp];
  }
}

// a wave-uniform double into scalar registers (the S rows of the LDS copy: no VGPRs held)
__device__ __forceinline__ double mgs_uniform(double x)
{
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// The read pass over this lane's rows: replay F steps, accumulate the window's Gram rows
// acc[w][c] = sum q_{F+w} q_c (c >= F + w; the other slots stay 0)
template <int F, int W, int U>  // U: rows per lane per batch; two batches in flight (ping-pong)
__device__ __forceinline__ void mgs_la_rows(i64 n, const double *__restrict__ Qb, const double *S, double (&acc)[W][8])
{
#pragma unroll
  for (int w = 0; w < W; ++w)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[w][c] = 0.0;
  double Sr[F > 0 ? F : 1][8];
#pragma unroll
  for (int kp = 0; kp < F; ++kp)
#pragma unroll
    for (int j = 0; j < 8; ++j) Sr[kp][j] = j < kp ? 0.0 : mgs_uniform(S[kp * 8 + j]);
  const i64 stride = (i64)gridDim.x * kMgsLaThreads;
  auto load = [&](double (&q)[U][8], i64 i0) {
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const i64 i = i0 + u * stride;
      const double2 *r = reinterpret_cast<const double2 *>(Qb + (i < n ? i : 0) * 8);
#pragma unroll
      for (int h = 0; h < 4; ++h)
      {
        const double2 x = i < n ? r[h] : make_double2(0.0, 0.0);  // (rows past n add nothing)
        q[u][2 * h] = x.x;
        q[u][2 * h + 1] = x.y;
      }
    }
  };
  auto work = [&](double (&q)[U][8]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      mgs_row_replay<F>(q[u], Sr);
#pragma unroll
      for (int w = 0; w < W; ++w)
#pragma unroll
        for (int c = F + w; c < 8; ++c) acc[w][c] += q[u][F + w] * q[u][c];
    }
  };
  const i64 step = (i64)U * stride;
  i64 i0 = (i64)blockIdx.x * kMgsLaThreads + threadIdx.x;
  double qa[U][8], qb[U][8];
  load(qa, i0);
  while (i0 < n)
  {
    load(qb, i0 + step);
    work(qa);
    i0 += step;
    if (i0 >= n) break;
    load(qa, i0 + step);
    work(qb);
    i0 += step;
  }
}

// Workgroup sums of the 8 W slots (slot e = w 8 + c): a reduce-scatter by recursive halving inside
// each wave (P - 1 shuffles for P slots, lane l ending with slot bitrev(l)), the lane groups summed
// by xor shuffles, the waves' totals through LDS in wave order.  Threads < 8 W return their slot.
template <int W, int L>
__device__ __forceinline__ double mgs_la_block(double (&acc)[W][8], MgsLaShared<L> &sh)
{
  constexpr int E = 8 * W;
  constexpr int P = E <= 8 ? 8 : (E <= 16 ? 16 : (E <= 32 ? 32 : 64));
  constexpr int LOG = P == 8 ? 3 : (P == 16 ? 4 : (P == 32 ? 5 : 6));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double v[P];
#pragma unroll
  for (int e = 0; e < P; ++e) v[e] = e < E ? acc[e / 8][e % 8] : 0.0;
  int slot = 0;
#pragma unroll
  for (int s = 0; s < LOG; ++s)
  {
    const int half = P >> (s + 1);
    const bool hi = (lane >> s) & 1;
#pragma unroll
    for (int i = 0; i < half; ++i)
    {
      const double send = hi ? v[i] : v[half + i];
      const double keep = hi ? v[half + i] : v[i];
      v[i] = keep + __shfl_xor(send, 1 << s, 64);
    }
    slot += hi ? half : 0;
  }
  double x = v[0];
#pragma unroll
  for (int m = P; m < 64; m <<= 1) x += __shfl_xor(x, m, 64);
  if (lane < P) sh.red[wave][slot] = x;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x < E)
  {
#pragma unroll
    for (int q = 0; q < kMgsLaThreads / 64; ++q) t += sh.red[q][threadIdx.x];
  }
  return t;
}

// Grid sums of the 8 W slots from nblk workgroups' partials (block b's slot e at part[b ld + e]):
// value e over the blocks g, g + 8, ... (16 loads in flight per round), then the 8 slices in slice
// order -- a fixed order, independent of arrival.  Into sh.Rw (every thread may call; all must).
template <int W, int L>
__device__ __forceinline__ void mgs_la_gather(const double *part, int ld, unsigned nblk, MgsLaShared<L> &sh)
{
  constexpr int E = 8 * W;
  if (threadIdx.x < 8 * E)
  {
    const int e = threadIdx.x % E, g = threadIdx.x / E;
    double x = 0.0;
    for (unsigned b0 = (unsigned)g; b0 < nblk; b0 += 8u * 16u)
    {
      double t[16];
#pragma unroll
      for (int u = 0; u < 16; ++u)
      {
        const unsigned b = b0 + 8u * u;
        t[u] = b < nblk ? ld_sc1(&part[(size_t)b * ld + e]) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) x += t[u];
    }
    sh.fin[g][e] = x;
  }
  __syncthreads();
  if (threadIdx.x < E)
  {
    double x = 0.0;
#pragma unroll
    for (int g = 0; g < 8; ++g) x += sh.fin[g][threadIdx.x];
    sh.Rw[threadIdx.x / 8][threadIdx.x % 8] = x;
  }
  __syncthreads();
}

// Lanes 0..7 of wave 0 (lane j holds column j of the window rows, col[w] = s[F + w][j]): finish
// steps F .. into S; returns the new F (wave-uniform).  The pivot and the multipliers come by
// shuffle, so every index is compile-time and the arithmetic is that of one thread doing
// s'[b][j] -= (s[a][b] / s[a][a]) s[a][j] row by row.
template <int F, int W>
__device__ int mgs_la_finish(double (&col)[W], double *S)
{
  const int j = threadIdx.x & 63;
  double r0[W];
#pragma unroll
  for (int w = 0; w < W; ++w) r0[w] = __shfl(col[w], F + w, 64);
  int Fn = F;
  bool go = true;  // (a predicate, not a break: every index stays compile-time)
#pragma unroll
  for (int w = 0; w < W; ++w)
  {
    const int a = F + w;
    const double d = __shfl(col[w], a, 64);
    if (w > 0) go = go && d >= kMgsLaTau * r0[w];  // (NaN refuses too)
    if (!go) continue;
    // S[a][j] = s[a][j] / s[a][a] (j > a), S[a][a] = 1 / sqrt(s[a][a]) (kernels_cpp.hh:214-228)
    if (j < 8) S[a * 8 + j] = j < a ? 0.0 : (j == a ? 1.0 / sqrt(d) : col[w] / d);
    Fn = a + 1;
    // eliminate step a from the later window rows: s'[b][j] -= (s[a][b] / s[a][a]) s[a][j]
#pragma unroll
    for (int w2 = w + 1; w2 < W; ++w2)
    {
      const int b = F + w2;
      const double f = __shfl(col[w], b, 64) / d;
      if (j >= b) col[w2] -= f * col[w];
    }
  }
  return Fn;
}

// wave 0: the window sums of sh.Rw -> S rows, new state word (returned in every lane of wave 0)
template <int F, int W, int L>
__device__ __forceinline__ unsigned mgs_la_close(MgsLaShared<L> &sh, double *S, unsigned word)
{
  const int j = threadIdx.x & 63;
  double col[W];
#pragma unroll
  for (int w = 0; w < W; ++w) col[w] = j < 8 ? sh.Rw[w][j] : 0.0;
  const int Fn = mgs_la_finish<F, W>(col, S);
  return (unsigned)Fn | ((((word >> 8) & 255u) + 1u) << 8);
}

// An ordinary read launch: rows, workgroup partials, ticket; the last workgroup finishes the window.
template <int F, int L>
__device__ __forceinline__ void mgs_la_read(const MgsLaArgs a, unsigned word, MgsLaShared<L> &sh)
{
  constexpr int W = (8 - F) < L ? (8 - F) : L;
  constexpr int E = 8 * W;
  double acc[W][8];
  mgs_la_rows<F, W, 2>(a.n, a.Qb, a.Sfin, acc);
  const double part = mgs_la_block<W, L>(acc, sh);
  const unsigned bid = blockIdx.x, nblk = gridDim.x;
  if (threadIdx.x < E) st_sc1(&a.partials[(size_t)bid * E + threadIdx.x], part);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sh.last = ticket_arrive(a.ticket, bid, nblk) ? 1u : 0u;
  __syncthreads();
  if (!sh.last) return;
  mgs_la_gather<W, L>(a.partials, E, nblk, sh);
  if (threadIdx.x < 64)
  {
    const unsigned nw = mgs_la_close<F, W, L>(sh, a.Sfin, word);
    if (threadIdx.x == 0)
    {
      a.st[(a.launch + 1) & 1] = nw;
      ticket_reset(a.ticket);
    }
  }
}

// The write pass, quad layout (as k_mgs_replay<8>): replay the 8 steps, store the rows.
__device__ __forceinline__ void mgs_la_write(i64 n, double *__restrict__ Qb, const double *S)
{
  constexpr int U = 8;
  const int ql = threadIdx.x & 3;
  const int c0 = 2 * ql, c1 = c0 + 1;
  double sp0[8], sp1[8];
#pragma unroll
  for (int kp = 0; kp < 8; ++kp)
  {
    sp0[kp] = S[kp * 8 + c0];
    sp1[kp] = S[kp * 8 + c1];
  }
  const i64 stride = (i64)gridDim.x * (kMgsLaThreads / 4);
  auto load = [&](double2 (&v)[U], i64 i0) {
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const i64 i = i0 + u * stride;
      v[u] = i < n ? reinterpret_cast<const double2 *>(Qb + i * 8)[ql] : make_double2(0.0, 0.0);
    }
  };
  auto work = [&](double2 (&v)[U], i64 i0) {
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      mgs_replay_steps<0, 8>(v[u], sp0, sp1, c0, c1);
      const i64 i = i0 + u * stride;
      if (i < n) reinterpret_cast<double2 *>(Qb + i * 8)[ql] = v[u];
    }
  };
  const i64 step = (i64)U * stride;
  i64 i0 = ((i64)blockIdx.x * kMgsLaThreads + threadIdx.x) >> 2;
  double2 va[U], vb[U];
  load(va, i0);
  while (i0 < n)
  {
    load(vb, i0 + step);
    work(va, i0);
    i0 += step;
    if (i0 >= n) break;
    load(va, i0 + step);
    work(vb, i0);
    i0 += step;
  }
}

template <int L>
__global__ __launch_bounds__(kMgsLaThreads) void k_mgs_la(MgsLaArgs a)
{
  __shared__ MgsLaShared<L> sh;  // (one copy for the nine pass bodies)
  const unsigned word = a.launch == 0 ? 0u : a.st[a.launch & 1];
  if (a.launch == 0 && blockIdx.x == 0 && threadIdx.x == 0)
    a.st[kMgsLaBar] = 0u;  // for the last launch of this call (the error word is sticky: the host clears it)
  if (word & kMgsLaWritten)
  {
    if (blockIdx.x == 0 && threadIdx.x == 0) a.st[(a.launch + 1) & 1] = word;
    return;
  }
  switch (word & 15u)
  {
    case 0: mgs_la_read<0, L>(a, word, sh); break;
    case 1: mgs_la_read<1, L>(a, word, sh); break;
    case 2: mgs_la_read<2, L>(a, word, sh); break;
    case 3: mgs_la_read<3, L>(a, word, sh); break;
    case 4: mgs_la_read<4, L>(a, word, sh); break;
    case 5: mgs_la_read<5, L>(a, word, sh); break;
    case 6: mgs_la_read<6, L>(a, word, sh); break;
    case 7: mgs_la_read<7, L>(a, word, sh); break;
    default:
      mgs_la_write(a.n, a.Qb, a.Sfin);
      if (blockIdx.x == 0 && threadIdx.x == 0)
      {
        a.st[(a.launch + 1) & 1] = word | kMgsLaWritten;
        a.st[kMgsLaLast] = word | kMgsLaWritten;
      }
      break;
  }
}

// A read pass inside the last launch: workgroup partials into the pass's parity buffer, a
// grid barrier, then EVERY workgroup sums all partials in the same fixed order and finishes the
// window itself (bitwise the same S rows in each).  False when the barrier timed out.
template <int F, int L>
__device__ __forceinline__ bool mgs_la_read_coop(const MgsLaArgs a, MgsLaShared<L> &sh, unsigned &nb)
{
  constexpr int W = (8 - F) < L ? (8 - F) : L;
  constexpr int E = 8 * W;
  double acc[W][8];
  mgs_la_rows<F, W, 1>(a.n, a.Qb, sh.S, acc);  // (the rare path: fewer rows in flight, no spills)
  const double part = mgs_la_block<W, L>(acc, sh);
  // two buffers by pass parity: pass nb + 2 stores only after barrier nb + 1, which every
  // workgroup reaches after reading pass nb's partials
  double *buf = a.partials + (size_t)(nb & 1u) * gridDim.x * 64;
  if (threadIdx.x < E) st_sc1(&buf[(size_t)blockIdx.x * 64 + threadIdx.x], part);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ++nb;
  if (!mgs_grid_barrier(a.st + kMgsLaBar, nb, a.err)) return false;
  mgs_la_gather<W, L>(buf, 64, gridDim.x, sh);
  if (threadIdx.x < 64)
  {
    const unsigned nw = mgs_la_close<F, W, L>(sh, sh.S, sh.word);
    if (threadIdx.x == 0) sh.word = nw;
  }
  __syncthreads();
  return true;
}

// The last launch of a call (every workgroup resident: G <= CUs, one workgroup fits a CU).
// G (or null): the block's window Gram, summed by the product that wrote the block (StandardLargest,
// launch_mgs_lookahead_gram): every workgroup finishes the window from it itself -- the same close
// as the read pass's tail, so the same S rows in every workgroup -- instead of a first read pass.
template <int L>
__global__ __launch_bounds__(kMgsLaThreads) void k_mgs_la_final(MgsLaArgs a, const double *__restrict__ G = nullptr)
{
  __shared__ MgsLaShared<L> sh;
  if (G)
  {
    if (threadIdx.x < 64)
    {
      const int w = threadIdx.x / 8, c = threadIdx.x % 8;
      sh.Rw[w][c] = c >= w ? G[threadIdx.x] : 0.0;
    }
    __syncthreads();
    if (threadIdx.x < 64)
    {
      const unsigned nw = mgs_la_close<0, 8, L>(sh, sh.S, 0u);
      if (threadIdx.x == 0) sh.word = nw;
    }
  }
  else
  {
    if (threadIdx.x < 64) sh.S[threadIdx.x] = a.Sfin[threadIdx.x];
    if (threadIdx.x == 0) sh.word = a.st[a.launch & 1];
  }
  __syncthreads();
  unsigned nb = 0;
  while ((sh.word & 15u) < 8u)  // (uniform: sh.word changes only between barriers)
  {
    bool ok = true;
    switch (sh.word & 15u)
    {
      case 0: ok = mgs_la_read_coop<0, L>(a, sh, nb); break;
      case 1: ok = mgs_la_read_coop<1, L>(a, sh, nb); break;
      case 2: ok = mgs_la_read_coop<2, L>(a, sh, nb); break;
      case 3: ok = mgs_la_read_coop<3, L>(a, sh, nb); break;
      case 4: ok = mgs_la_read_coop<4, L>(a, sh, nb); break;
      case 5: ok = mgs_la_read_coop<5, L>(a, sh, nb); break;
      case 6: ok = mgs_la_read_coop<6, L>(a, sh, nb); break;
      default: ok = mgs_la_read_coop<7, L>(a, sh, nb); break;
    }
    if (!ok)
    {
      // a peer workgroup never arrived: poison this workgroup's rows (loud, never silent)
      const double nan = __builtin_nan("");
      for (i64 i = (i64)blockIdx.x * kMgsLaThreads + threadIdx.x; i < a.n; i += (i64)gridDim.x * kMgsLaThreads)
      {
        double2 *r = reinterpret_cast<double2 *>(a.Qb + i * 8);
#pragma unroll
        for (int h = 0; h < 4; ++h) r[h] = make_double2(nan, nan);
      }
      return;
    }
  }
  mgs_la_write(a.n, a.Qb, sh.S);
  if (blockIdx.x == 0)
  {
    if (threadIdx.x < 64) a.Sfin[threadIdx.x] = sh.S[threadIdx.x];
    if (threadIdx.x == 0)
    {
      a.st[(a.launch + 1) & 1] = sh.word | kMgsLaWritten;
      a.st[kMgsLaLast] = sh.word | kMgsLaWritten;
    }
  }
}

// The first read pass from a Gram computed elsewhere (StandardLargest: the SpMM that wrote the
// block summed its window Gram in its epilogue, k_boxc_mv8 / k_spmm8_march GRAM): ONE workgroup
// finishes the window from G (row-major 8 x 8, upper triangle used) exactly as the read pass's tail
// does from its grid sums, and hands the state word to launch 1 (k_mgs_la_final).
__global__ __launch_bounds__(kMgsLaThreads) void k_mgs_la_gram(MgsLaArgs a, const double *__restrict__ G)
{
  __shared__ MgsLaShared<8> sh;
  if (threadIdx.x < 64)
  {
    const int w = threadIdx.x / 8, c = threadIdx.x % 8;
    sh.Rw[w][c] = c >= w ? G[threadIdx.x] : 0.0;
  }
  __syncthreads();
  if (threadIdx.x < 64)
  {
    const unsigned nw = mgs_la_close<0, 8, 8>(sh, a.Sfin, 0u);
    if (threadIdx.x == 0)
    {
      a.st[kMgsLaBar] = 0u;  // for the last launch of this call
      a.st[1] = nw;          // launch 1's word
    }
  }
}

static int *mgs_err_word(eig_ctx_t ctx);

int mgs_lookahead_default()
{
  static const int L = [] {
    const char *e = std::getenv("EIGMI_MGS_LOOKAHEAD");
    const int v = e ? std::atoi(e) : kMgsLookaheadDefault;
    return std::min(8, std::max(1, v));
  }();
  return L;
}

namespace {
template <int L>
void mgs_la_enqueue(MgsLaArgs a, int G, bool coop, hipStream_t s)
{
  const int reads = (8 + L - 1) / L;  // read launches when every look-ahead is taken
  for (int l = 0; l < reads; ++l)
  {
    a.launch = l;
    hipLaunchKernelGGL(k_mgs_la<L>, dim3(G), dim3(kMgsLaThreads), 0, s, a);
  }
  EIG_HIP(hipGetLastError());
  a.launch = reads;
  if (coop)
  {
    // an ordinary launch: G <= the CU count and one workgroup fits a CU (VGPRs, LDS), so on an idle
    // device every workgroup is resident at once, and beside other streams' kernels the ones not
    // yet resident only wait for CUs those kernels release -- the barriers need no cooperative
    // launch (whose host call measured ~30 us per orthonormalisation, profiles/r05r_ortho.jsonl)
    hipLaunchKernelGGL(k_mgs_la_final<L>, dim3(G), dim3(kMgsLaThreads), 0, s, a, (const double *)nullptr);
    EIG_HIP(hipGetLastError());
    return;
  }
  // the worst case in ordinary launches: every look-ahead refused -> 8 read launches + the write
  for (int l = reads; l < 9; ++l)
  {
    a.launch = l;
    hipLaunchKernelGGL(k_mgs_la<L>, dim3(G), dim3(kMgsLaThreads), 0, s, a);
  }
  EIG_HIP(hipGetLastError());
}
}  // namespace

bool launch_mgs_lookahead(eig_ctx_t ctx, i64 n, double *Qb, int L, bool coop, hipStream_t s)
{
  if (L <= 1 || n <= 0) return false;
  const size_t bytes = 64 * sizeof(double) + 64 * sizeof(unsigned);
  const bool fresh = (int)ctx->pool.size() <= 11 || ctx->pool[11].second < bytes;
  char *buf = (char *)ctx_buffer(ctx, 11, bytes);
  if (fresh) EIG_HIP(hipMemsetAsync(buf, 0, bytes, s));  // (the sticky error word starts clear)
  if (coop) ctx->mgs_la_armed = true;
  ctx->mgs_bar_clean = nullptr;  // (this call's last launch leaves the barrier word set)
  MgsLaArgs a{n, Qb, 0, reinterpret_cast<unsigned *>(buf + 64 * sizeof(double)), reinterpret_cast<double *>(buf),
              ctx->red.partials, ctx->red.ticket(0), mgs_err_word(ctx)};
  const int G = grid_for(n, kMgsLaThreads * 2, std::min(kMgsLaGrid, ctx->num_cu > 0 ? ctx->num_cu : kMgsLaGrid));
  if (L >= 8) mgs_la_enqueue<8>(a, G, coop, s);
  else if (L >= 4) mgs_la_enqueue<4>(a, G, coop, s);
  else mgs_la_enqueue<2>(a, G, coop, s);
  return true;
}

static int *mgs_err_word(eig_ctx_t ctx)
{
  if (!ctx->mgs_err_host)
  {
    EIG_HIP(hipHostMalloc(reinterpret_cast<void **>(&ctx->mgs_err_host), sizeof(int), hipHostMallocMapped));
    *ctx->mgs_err_host = 0;
    EIG_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->mgs_err_dev), ctx->mgs_err_host, 0));
  }
  return ctx->mgs_err_dev;
}

unsigned *mgs_lookahead_barrier(eig_ctx_t ctx)
{
  const size_t bytes = 64 * sizeof(double) + 64 * sizeof(unsigned);
  const bool fresh = (int)ctx->pool.size() <= 11 || ctx->pool[11].second < bytes;
  char *buf = (char *)ctx_buffer(ctx, 11, bytes);
  if (fresh) EIG_HIP(hipMemsetAsync(buf, 0, bytes, ctx->stream));  // (the sticky error word starts clear)
  return reinterpret_cast<unsigned *>(buf + 64 * sizeof(double)) + kMgsLaBar;
}

bool launch_mgs_lookahead_gram(eig_ctx_t ctx, i64 n, double *Qb, const double *G, hipStream_t s)
{
  if (n <= 0 || !G) return false;
  unsigned *bar = mgs_lookahead_barrier(ctx);
  char *buf = reinterpret_cast<char *>(bar - kMgsLaBar) - 64 * sizeof(double);
  ctx->mgs_la_armed = true;
  MgsLaArgs a{n, Qb, 1, bar - kMgsLaBar, reinterpret_cast<double *>(buf), ctx->red.partials, ctx->red.ticket(0),
              mgs_err_word(ctx)};
  const int G8 = grid_for(n, kMgsLaThreads * 2, std::min(kMgsLaGrid, ctx->num_cu > 0 ? ctx->num_cu : kMgsLaGrid));
  if (ctx->mgs_bar_clean == G)
  {
    // the product that summed G zeroed the last launch's barrier word (its last workgroup): the
    // window is finished in the last launch's prologue, ONE launch per block
    ctx->mgs_bar_clean = nullptr;
    hipLaunchKernelGGL(k_mgs_la_final<8>, dim3(G8), dim3(kMgsLaThreads), 0, s, a, G);
  }
  else
  {
    hipLaunchKernelGGL(k_mgs_la_gram, dim3(1), dim3(kMgsLaThreads), 0, s, a, G);
    hipLaunchKernelGGL(k_mgs_la_final<8>, dim3(G8), dim3(kMgsLaThreads), 0, s, a, (const double *)nullptr);
  }
  EIG_HIP(hipGetLastError());
  return true;
}

// read passes of the last look-ahead call on this context (diagnostics; synchronises the stream):
// -1 none finished, -2 the last launch's grid barrier timed out
int mgs_lookahead_passes(eig_ctx_t ctx)
{
  char *buf = (char *)ctx_buffer(ctx, 11, 64 * sizeof(double) + 64 * sizeof(unsigned));
  unsigned w[64] = {};
  EIG_HIP(hipMemcpyAsync(w, buf + 64 * sizeof(double), sizeof(w), hipMemcpyDeviceToHost, ctx->stream));
  EIG_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->mgs_err_host && *reinterpret_cast<volatile int *>(ctx->mgs_err_host)) return -2;
  return (w[kMgsLaLast] & kMgsLaWritten) ? (int)((w[kMgsLaLast] >> 8) & 255u) : -1;
}

void mgs_lookahead_check(eig_ctx_t ctx)
{
  // (called after a synchronisation of the stream: the word is host memory, no copy, no launch)
  if (!ctx->mgs_la_armed) return;
  ctx->mgs_la_armed = false;
  volatile int *e = ctx->mgs_err_host;
  if (!e || !*e) return;
  *e = 0;
  EIG_CHECK(false, EIG_ERR_HIP,
            "orthonormalize_blocked: a look-ahead MGS grid barrier timed out (workgroups not co-resident); "
            "the block was poisoned with NaN");
}

// ---------------------------------------------------------------------------------------------
// The same column MGS for a small block (n <= 512 R rows, one rank), in ONE workgroup: the 512
// threads keep their R rows in registers for all 8 passes, and each pass's sums meet in a
// workgroup reduction (a xor-shuffle tree per wave, the 8 wave partials summed in wave order by
// every thread), so the block is read and written once and the 9 grid-wide launches with their
// reduction tails (10 us each at n = 4096, launch-bound) become one launch.  Per row the
// operations are those of k_mgs_pass; only the sums' order differs (tolerance, as there).
// ---------------------------------------------------------------------------------------------
constexpr int kMgsSmallThreads = 512;

template <int R>
__global__ __launch_bounds__(kMgsSmallThreads) void k_mgs_small(i64 n, double *__restrict__ Qb)
{
  __shared__ double red[2][kMgsSmallThreads / 64][8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double q[R][8];
#pragma unroll
  for (int t = 0; t < R; ++t)
  {
    const i64 i = tid + (i64)t * kMgsSmallThreads;
    const double2 *row = reinterpret_cast<const double2 *>(Qb + (i < n ? i : 0) * 8);
#pragma unroll
    for (int h = 0; h < 4; ++h)
    {
      const double2 v = i < n ? row[h] : make_double2(0.0, 0.0);
      q[t][2 * h] = v.x;
      q[t][2 * h + 1] = v.y;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k)
  {
    double acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.0;
#pragma unroll
    for (int t = 0; t < R; ++t)
#pragma unroll
      for (int j = k; j < 8; ++j) acc[j] += q[t][k] * q[t][j];  // (rows past n are zero)
#pragma unroll
    for (int j = k; j < 8; ++j)
    {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) acc[j] += __shfl_xor(acc[j], o, 64);
      if (lane == 0) red[k & 1][wave][j] = acc[j];
    }
    __syncthreads();
    double sk[8];
#pragma unroll
    for (int j = k; j < 8; ++j)
    {
      double v = red[k & 1][0][j];
#pragma unroll
      for (int w = 1; w < kMgsSmallThreads / 64; ++w) v += red[k & 1][w][j];
      sk[j] = v;
    }
    // S[k][j] = s[k][j] / s[k][k] (j > k), S[k][k] = 1 / sqrt(s[k][k]) (kernels_cpp.hh:214-228)
    const double skk = sk[k];
#pragma unroll
    for (int t = 0; t < R; ++t)
    {
#pragma unroll
      for (int j = k + 1; j < 8; ++j) q[t][j] -= (sk[j] / skk) * q[t][k];
      q[t][k] *= 1.0 / sqrt(skk);
    }
  }
#pragma unroll
  for (int t = 0; t < R; ++t)
  {
    const i64 i = tid + (i64)t * kMgsSmallThreads;
    if (i < n)
    {
      double2 *row = reinterpret_cast<double2 *>(Qb + i * 8);
#pragma unroll
      for (int h = 0; h < 4; ++h) row[h] = make_double2(q[t][2 * h], q[t][2 * h + 1]);
    }
  }
}

bool launch_mgs_small(i64 n, double *Qb, hipStream_t s)
{
  if (n <= 0 || n > 8 * kMgsSmallThreads) return false;
  const dim3 g(1), b(kMgsSmallThreads);
  if (n <= kMgsSmallThreads) hipLaunchKernelGGL(k_mgs_small<1>, g, b, 0, s, n, Qb);
  else if (n <= 2 * kMgsSmallThreads) hipLaunchKernelGGL(k_mgs_small<2>, g, b, 0, s, n, Qb);
  else if (n <= 4 * kMgsSmallThreads) hipLaunchKernelGGL(k_mgs_small<4>, g, b, 0, s, n, Qb);
  else hipLaunchKernelGGL(k_mgs_small<8>, g, b, 0, s, n, Qb);
  return true;
}

// ---------------------------------------------------------------------------------------------
// CholQR factor of an 8x8 Gram (kernels_avx2.hh:185-252 / kernels_cpp.hh:474-526), one thread:
// LU without pivoting, D = diag^-1/2, U = L^-T D.  flags & 1: take the UPPER triangle of G and
// mirror it (B_orthonormalize_blocked :457-459), and fold max_{k<j} G[k][j] into *normmax.
// Writes U (8x8 row-major).  A non-positive pivot yields NaN/inf like the reference.
// ---------------------------------------------------------------------------------------------
__global__ void k_cholqr_factor(const double *__restrict__ G, double *__restrict__ U, double *normmax, int flags)
{
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s[8][8], LU[8][8], UU[8][8], D[8];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) s[i][j] = G[i * 8 + j];
  if (flags & 1)
  {
    for (int k = 0; k < 8; ++k)
      for (int j = 0; j < k; ++j) s[k][j] = s[j][k];
    double nm = normmax[0];
    for (int k = 0; k < 8; ++k)
      for (int j = k + 1; j < 8; ++j) nm = fmax(nm, s[k][j]);
    normmax[0] = nm;
  }
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) LU[i][j] = s[i][j];
  for (int k = 0; k < 8; ++k)
    for (int i = k + 1; i < 8; ++i)
    {
      LU[i][k] /= LU[k][k];
      for (int j = k + 1; j < 8; ++j) LU[i][j] -= LU[i][k] * LU[k][j];
    }
  for (int i = 0; i < 8; ++i) D[i] = 1.0 / sqrt(LU[i][i]);
  for (int i = 0; i < 8; ++i)
  {
    LU[i][i] = 1.0;
    for (int j = i + 1; j < 8; ++j) LU[i][j] = 0.0;
  }
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) UU[i][j] = (i == j) ? 1.0 : 0.0;
  for (int i = 1; i < 8; ++i)
    for (int j = 0; j < i; ++j)
      for (int k = 0; k < 8; ++k) UU[i][k] -= LU[i][j] * UU[j][k];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < i; ++j)
    {
      double tmp = UU[i][j];
      UU[i][j] = UU[j][i];
      UU[j][i] = tmp;
    }
  for (int i = 0; i < 8; ++i)
    for (int j = i; j < 8; ++j) UU[i][j] *= D[j];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) U[i * 8 + j] = UU[i][j];
}

void launch_cholqr_factor(const double *G, double *U, double *normmax, int flags, hipStream_t s)
{
  hipLaunchKernelGGL(k_cholqr_factor, dim3(1), dim3(64), 0, s, G, U, normmax, flags);
}

// v_i := v_i U in place, j descending, sum over k <= j (kernels_cpp.hh:556-568).
__global__ __launch_bounds__(kStreamThreads) void k_apply_upper(i64 n, double *__restrict__ Qb,
                                                                const double *__restrict__ Ug)
{
  __shared__ double U[64];
  if (threadIdx.x < 64) U[threadIdx.x] = Ug[threadIdx.x];
  __syncthreads();
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
  {
    double v[8];
    double2 *row = reinterpret_cast<double2 *>(Qb + i * 8);
#pragma unroll
    for (int h = 0; h < 4; ++h)
    {
      const double2 x = row[h];
      v[2 * h] = x.x;
      v[2 * h + 1] = x.y;
    }
#pragma unroll
    for (int j = 7; j >= 0; --j)
    {
      double sum = 0.0;
#pragma unroll
      for (int k = 0; k <= j; ++k) sum += v[k] * U[k * 8 + j];
      v[j] = sum;
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) row[h] = make_double2(v[2 * h], v[2 * h + 1]);
  }
}

void launch_apply_upper(i64 n, double *Qb, const double *U, hipStream_t s)
{
  hipLaunchKernelGGL(k_apply_upper, dim3(grid_for(n, kStreamThreads * 4, kStreamBlocks)), dim3(kStreamThreads), 0, s,
                     n, Qb, U);
}

// ---------------------------------------------------------------------------------------------
// Later-block projection (kernels_cpp.hh:335-348): Q_rest(i, j) -= sum_k S[k][j] Q_k(i, k), k
// ascending, element by element in the reference order.  S is 8 x mrest row-major (the Gram
// Q_k^T Q_rest).  One thread per row: Q_k's row is loaded once and every later block is updated in
// turn, so S is read with wave-uniform addresses (scalar loads, SGPR operands).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kStreamThreads) void k_project(i64 n, int nb, const double *__restrict__ Qk,
                                                            double *__restrict__ Qrest, const double *__restrict__ S)
{
  const int mrest = nb * 8;
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
  {
    double qk[8];
    const double2 *rk = reinterpret_cast<const double2 *>(Qk + i * 8);
#pragma unroll
    for (int h = 0; h < 4; ++h)
    {
      const double2 x = rk[h];
      qk[2 * h] = x.x;
      qk[2 * h + 1] = x.y;
    }
    for (int b = 0; b < nb; ++b)
    {
      double qj[8];
      double2 *rj = reinterpret_cast<double2 *>(Qrest + ((i64)b * n + i) * 8);
#pragma unroll
      for (int h = 0; h < 4; ++h)
      {
        const double2 y = rj[h];
        qj[2 * h] = y.x;
        qj[2 * h + 1] = y.y;
      }
      const double *Sb = S + b * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k)
      {
#pragma unroll
        for (int j = 0; j < 8; ++j) qj[j] -= Sb[k * mrest + j] * qk[k];
      }
#pragma unroll
      for (int h = 0; h < 4; ++h) rj[h] = make_double2(qj[2 * h], qj[2 * h + 1]);
    }
  }
}

void launch_project(i64 n, i64 mrest, const double *Qk, double *Qrest, const double *S, hipStream_t s)
{
  if (mrest <= 0) return;
  hipLaunchKernelGGL(k_project, dim3(grid_for(n, kStreamThreads * 2, kStreamBlocks)), dim3(kStreamThreads), 0, s, n,
                     (int)(mrest / 8), Qk, Qrest, S);
}

// *normmax = max(*normmax, max over S (rows x cols, row-major) [strict upper triangle only]).
__global__ void k_max_offdiag(const double *S, i64 rows, i64 cols, int upper_only, double *normmax)
{
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double nm = normmax[0];
  for (i64 k = 0; k < rows; ++k)
    for (i64 j = upper_only ? k + 1 : 0; j < cols; ++j) nm = fmax(nm, S[k * cols + j]);
  normmax[0] = nm;
}
void launch_max_offdiag(const double *S, i64 rows, i64 cols, bool upper_only, double *normmax, hipStream_t s)
{
  hipLaunchKernelGGL(k_max_offdiag, dim3(1), dim3(64), 0, s, S, rows, cols, upper_only ? 1 : 0, normmax);
}

}  // namespace eigmi
