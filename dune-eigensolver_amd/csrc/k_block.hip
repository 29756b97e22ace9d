// k_block.hip -- window-layout MultiVector<double,8> kernels (gfx950) for the block methods:
//
//   k_sell_mv8g       Y = A X over the SELL-64 image, one column block (m = 8): a wave per slice,
//                     lane = column pair x 4 rows
//   k_sell_mv8q       the same for m >= 16: 4 lanes per row, up to 4 column blocks per matrix pass;
//                     epilogue kStore (plain SpMM, a2) or kCheb (one Chebyshev-Jacobi step of the
//                     mass solve, fused into the SpMM)
//   k_diag_inv        dinv[r] = 1 / a_rr
//   k_cheb_init       X = gamma * dinv o B
//   k_panel_gram_*    G = Q1^T Q2 for tall-skinny panels on MFMA (v_mfma_f64_16x16x4f64), two
//                     deterministic stages (per-workgroup partials, then a fixed-order sum)
//   k_panel_update    Y = beta Y + alpha Q S (Q: n x m1, S: m1 x m2 with m2 <= 32), FMA with S
//                     in scalar registers
//   k_cholqr_fold     CholQR2's middle step for 32 columns: Z <- Z S and G = (Z S)^T (MZ S) in one
//                     pass, MFMA for both products
//
// Window layout: column block b of a multivector with leading dimension ld (the matrix window)
// is ld rows of 8 contiguous doubles at Q + 8 b ld; owned row r sits at window row own + r.  On
// one rank ld = n and own = 0, which is the reference's MultiVector<double,8> layout
// (multivector.hh:130-139).
#include <cstdlib>
#include <string>

#include "internal.h"
#include "reduce_dev.h"

namespace eigmi {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double dv2 __attribute__((ext_vector_type(2)));

static inline int grid_cap(i64 work, i64 per_block, int cap)
{
  i64 g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

// ---------------------------------------------------------------------------------------------
// SpMM over 64-row SELL slices.  Per column the row sum runs over the stored entries in
// ascending-column order from 0.0 (bitwise the reference's matmul_sparse_tallskinny_blocked,
// kernels_cpp.hh:644-655).
//
// kCheb epilogue (Golub-Varga three-term Chebyshev semi-iteration for M x = b with the Jacobi
// splitting): with acc = (M x_k)_r,
//     x_{k+1}[r] = omega (x_k[r] + gamma dinv[r] (b[r] - acc) - x_{k-1}[r]) + x_{k-1}[r]
// written in place over x_{k-1} (Xold); x_k is the gathered input X.
// (Measured and dropped: a lane-per-row mapping with 16 columns per matrix pass -- 131 vs 119 us
// for the 7-point SpMM at 128^3 -- and 2 column blocks per quad pass.)
// ---------------------------------------------------------------------------------------------
enum { kStore = 0, kCheb = 1, kResid = 2 };  // kResid: Y = B - A X (multigrid residual)

// Quad mapping: 4 lanes per row (lane owns column pair 2 (l & 3), 2 (l & 3) + 1 of every column
// block), 16 rows per wave, a workgroup (4 waves) per 64-row slice, MB column blocks per matrix
// pass.  Entries are consumed U at a time: the U columns / values are loaded first, then all U * MB
// 16-B gathers are issued before the multiply-adds (memory-level parallelism without holding
// whole 64-B rows per lane).  Per column, ascending-column order from 0.0 as above.
//
// XCD-aware plane-slab schedule.  A unit is 16 W rows (W waves of 16 rows; W = 2: two units per
// 64-row slice).  The rows are cut into "planes" of P8 units (P8 = the matrix bandwidth -- N^2
// rows for the 3-D grids -- rounded up to 8 segments) and every plane into 8 segments; the
// workgroups on XCD x (b % 8 == x: blocks are dealt round-robin over the XCDs -- a speed
// assumption only, any placement gives the same result) sweep segment x of plane 0, then of plane
// 1, ..., interleaved unit by unit, so the XCD's front of resident workgroups moves through one
// contiguous slab.  A row's x / y neighbours lie in the front, its z - 1 neighbours in the
// previous plane's segment the same XCD just streamed: both are read from the XCD's own L2, and
// each X row comes from HBM about once.
template <int MB, int U, int W, bool STENCIL, int EPI>
__global__ __launch_bounds__(64 * W) void k_sell_mv8q(i64 nrows, i64 nslices, const i64 *__restrict__ slice_ptr,
                                                      const double *__restrict__ val, const i32 *__restrict__ col,
                                                      const i32 *__restrict__ st_delta,
                                                      const uint8_t *__restrict__ st_mask, const double *__restrict__ X,
                                                      double *__restrict__ Y, i64 ld, i64 own, int b0,
                                                      const double *__restrict__ Bv, const double *__restrict__ dinv,
                                                      double omega, double gamma, i64 per)
{
  constexpr int UPS = 4 / W;  // units per slice
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cp = lane & 3;
  const i64 nunits = nslices * UPS;
  const i64 seg = per;  // units per plane segment; plane = 8 segments
  const int xcd = blockIdx.x & 7;
  const i64 nloc = gridDim.x >> 3;  // workgroups per XCD (grid is a multiple of 8)
  const double *Xc = X + (i64)b0 * ld * 8 + 2 * cp;  // column pair cp of column block b0
  for (i64 t = blockIdx.x >> 3;; t += nloc)
  {
    const i64 pl = t / seg;
    const i64 un = pl * 8 * seg + xcd * seg + (t - pl * seg);
    if (pl * 8 * seg >= nunits) break;
    if (un >= nunits) continue;  // tail of the last plane
    const i64 s = un / UPS;
    const int ri = (int)(un % UPS) * 16 * W + wave * 16 + (lane >> 2);
    const i64 base = slice_ptr[s];
    const int width = (int)((slice_ptr[s + 1] - base) >> 6);
    const i64 r = s * 64 + ri;
    // entries that are not stored gather the row's own element; padding rows of the last slice
    // (r >= nrows) the last owned row's, so no gather leaves the window (tiny matrices: n < 64)
    const i64 rs = r < nrows ? r : nrows - 1;
    unsigned m = 0;
    if (STENCIL) m = st_mask[s * 64 + ri];
    double2 acc[MB];
#pragma unroll
    for (int q = 0; q < MB; ++q) acc[q] = make_double2(0.0, 0.0);
    for (int k0 = 0; k0 < width; k0 += U)
    {
      // branch-free: indices clamped into the slice, every load issued before the first wait;
      // entries that are not stored (padding, mask bit clear, k >= width) gather the row's own
      // in-window element and are discarded by a select, never multiplied in (the reference
      // loops over stored entries only: inf * 0 or -0 + 0 must not enter the sum)
      double a[U];
      i64 c[U];
      bool okk[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
      {
        const int k = k0 + u < width ? k0 + u : width - 1;
        a[u] = __builtin_nontemporal_load(val + base + k * 64 + ri);
        if (STENCIL)
        {
          okk[u] = (k0 + u < width) && ((m >> (k0 + u)) & 1u);
          c[u] = okk[u] ? own + r + st_delta[8 * s + k] : own + rs;
        }
        else
        {
          const i32 ci = __builtin_nontemporal_load(col + base + k * 64 + ri);
          okk[u] = (k0 + u < width) && ci >= 0;
          c[u] = okk[u] ? (i64)ci : own + rs;
        }
      }
      double2 xv[U][MB];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < MB; ++q) xv[u][q] = *reinterpret_cast<const double2 *>(Xc + ((i64)q * ld + c[u]) * 8);
      if (EPI == kStore || EPI == kResid)
      {
        // bitwise the reference: separately rounded products and sums over stored entries only
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int q = 0; q < MB; ++q)
          {
            const double tx = acc[q].x + a[u] * xv[u][q].x, ty = acc[q].y + a[u] * xv[u][q].y;
            acc[q].x = okk[u] ? tx : acc[q].x;
            acc[q].y = okk[u] ? ty : acc[q].y;
          }
      }
      else
      {
        // Chebyshev step (tolerance-checked, not bitwise): fused multiply-adds, non-stored
        // entries contribute 0 * (the row's own finite x) = 0
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
          const double au = okk[u] ? a[u] : 0.0;
#pragma unroll
          for (int q = 0; q < MB; ++q)
          {
            acc[q].x = __builtin_fma(au, xv[u][q].x, acc[q].x);
            acc[q].y = __builtin_fma(au, xv[u][q].y, acc[q].y);
          }
        }
      }
    }
    if (r < nrows)
    {
      // read-once / write-once streams are non-temporal so that the XCD's L2 keeps X for the
      // neighbour reuse of the plane-slab schedule
      double di = 0.0;
      if (EPI == kCheb) di = __builtin_nontemporal_load(dinv + r);
#pragma unroll
      for (int q = 0; q < MB; ++q)
      {
        const i64 at = ((i64)(b0 + q) * ld + own + r) * 8 + 2 * cp;
        double *yr = Y + at;
        double o0, o1;
        if (EPI == kStore)
        {
          o0 = acc[q].x;
          o1 = acc[q].y;
        }
        else if (EPI == kResid)
        {
          const dv2 bb = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(Bv + at));
          o0 = bb.x - acc[q].x;
          o1 = bb.y - acc[q].y;
        }
        else
        {
          const double2 xk = *reinterpret_cast<const double2 *>(X + at);
          const dv2 bb = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(Bv + at));
          const dv2 xo = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(yr));
          const double gd = gamma * di;
          o0 = omega * (xk.x + gd * (bb.x - acc[q].x) - xo.x) + xo.x;
          o1 = omega * (xk.y + gd * (bb.y - acc[q].y) - xo.y) + xo.y;
        }
        __builtin_nontemporal_store(dv2{o0, o1}, reinterpret_cast<dv2 *>(yr));
      }
    }
  }
}

// Grouped-quad mapping: a wave owns a whole 64-row slice; lane l owns column pair cp = l & 3 of
// the four rows (l >> 2) + 16 h, h = 0..3, of every column block, so each 16-B gather instruction
// of the wave reads 16 consecutive X rows (1 KiB contiguous for a stencil offset: whole cache
// lines, unlike the lane-per-row mapping whose instructions touch 64 rows at a 64-B stride), and
// the loop overhead, mask byte and stencil offsets are shared by the lane's 4 rows.  Units of 4
// slices (4 waves per workgroup) on the XCD plane-slab schedule of k_sell_mv8q.  Per column, the
// row sum runs over the stored entries in ascending-column order (bitwise the reference for kStore).
template <int MB, int U, bool STENCIL, int EPI>
__global__ __launch_bounds__(256) void k_sell_mv8g(i64 nrows, i64 nslices, const i64 *__restrict__ slice_ptr,
                                                   const double *__restrict__ val, const i32 *__restrict__ col,
                                                   const i32 *__restrict__ st_delta, const uint8_t *__restrict__ st_mask,
                                                   const double *__restrict__ X, double *__restrict__ Y, i64 ld, i64 own,
                                                   int b0, const double *__restrict__ Bv,
                                                   const double *__restrict__ dinv, double omega, double gamma, i64 per)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cp = lane & 3, rq = lane >> 2;
  const i64 nunits = (nslices + 3) / 4;
  const i64 seg = per;
  const int xcd = blockIdx.x & 7;
  const i64 nloc = gridDim.x >> 3;
  const double *Xc = X + (i64)b0 * ld * 8 + 2 * cp;
  for (i64 t = blockIdx.x >> 3;; t += nloc)
  {
    const i64 pl = t / seg;
    const i64 un = pl * 8 * seg + xcd * seg + (t - pl * seg);
    if (pl * 8 * seg >= nunits) break;
    const i64 s = un * 4 + wave;
    if (un >= nunits || s >= nslices) continue;
    const i64 base = slice_ptr[s];
    const int width = (int)((slice_ptr[s + 1] - base) >> 6);
    unsigned m[4] = {0u, 0u, 0u, 0u};
    if (STENCIL)
    {
#pragma unroll
      for (int h = 0; h < 4; ++h) m[h] = st_mask[s * 64 + rq + 16 * h];
    }
    double2 acc[4][MB];
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int q = 0; q < MB; ++q) acc[h][q] = make_double2(0.0, 0.0);
    for (int k0 = 0; k0 < width; k0 += U)
    {
      double a[U][4];
      i64 c[U][4];
      bool okk[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u)
      {
        const int k = k0 + u < width ? k0 + u : width - 1;
        i64 dl = 0;
        if (STENCIL) dl = st_delta[8 * s + k];
#pragma unroll
        for (int h = 0; h < 4; ++h)
        {
          const int ri = rq + 16 * h;
          const i64 r = s * 64 + ri;
          const i64 rs = r < nrows ? r : nrows - 1;  // (padding rows: see k_sell_mv8q)
          a[u][h] = __builtin_nontemporal_load(val + base + k * 64 + ri);
          if (STENCIL)
          {
            okk[u][h] = (k0 + u < width) && ((m[h] >> (k0 + u)) & 1u);
            c[u][h] = okk[u][h] ? own + r + dl : own + rs;
          }
          else
          {
            const i32 ci = __builtin_nontemporal_load(col + base + k * 64 + ri);
            okk[u][h] = (k0 + u < width) && ci >= 0;
            c[u][h] = okk[u][h] ? (i64)ci : own + rs;
          }
        }
      }
      double2 xv[U][4][MB];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int h = 0; h < 4; ++h)
#pragma unroll
          for (int q = 0; q < MB; ++q)
            xv[u][h][q] = *reinterpret_cast<const double2 *>(Xc + ((i64)q * ld + c[u][h]) * 8);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int h = 0; h < 4; ++h)
#pragma unroll
          for (int q = 0; q < MB; ++q)
          {
            if (EPI == kStore || EPI == kResid)
            {
              const double tx = acc[h][q].x + a[u][h] * xv[u][h][q].x, ty = acc[h][q].y + a[u][h] * xv[u][h][q].y;
              acc[h][q].x = okk[u][h] ? tx : acc[h][q].x;
              acc[h][q].y = okk[u][h] ? ty : acc[h][q].y;
            }
            else
            {
              const double au = okk[u][h] ? a[u][h] : 0.0;
              acc[h][q].x = __builtin_fma(au, xv[u][h][q].x, acc[h][q].x);
              acc[h][q].y = __builtin_fma(au, xv[u][h][q].y, acc[h][q].y);
            }
          }
    }
#pragma unroll
    for (int h = 0; h < 4; ++h)
    {
      const i64 r = s * 64 + rq + 16 * h;
      if (r >= nrows) continue;
      double di = 0.0;
      if (EPI == kCheb) di = __builtin_nontemporal_load(dinv + r);
#pragma unroll
      for (int q = 0; q < MB; ++q)
      {
        const i64 at = ((i64)(b0 + q) * ld + own + r) * 8 + 2 * cp;
        double *yr = Y + at;
        double o0 = acc[h][q].x, o1 = acc[h][q].y;
        if (EPI == kResid)
        {
          const dv2 bb = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(Bv + at));
          o0 = bb.x - o0;
          o1 = bb.y - o1;
        }
        if (EPI == kCheb)
        {
          const double2 xk = *reinterpret_cast<const double2 *>(X + at);
          const dv2 bb = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(Bv + at));
          const dv2 xo = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(yr));
          const double gd = gamma * di;
          o0 = omega * (xk.x + gd * (bb.x - o0) - xo.x) + xo.x;
          o1 = omega * (xk.y + gd * (bb.y - o1) - xo.y) + xo.y;
        }
        __builtin_nontemporal_store(dv2{o0, o1}, reinterpret_cast<dv2 *>(yr));
      }
    }
  }
}

namespace {
bool all_stencil(const eig_mat_s &A) { return A.n_stencil_slices == A.nslices && A.n_stencil_slices > 0; }

}  // namespace

namespace {
template <int EPI>
void sell_mv8(const eig_mat_s &A, i64 m, const double *X, double *Y, const double *Bv, const double *dinv,
              double omega, double gamma, hipStream_t s)
{
  EIG_CHECK(A.br == 1 && A.bc == 1, EIG_ERR_BLOCKSIZE,
            "matmul_sparse_tallskinny_blocked: only implemented for FieldMatrix<..,1,1>");
  const int nblk = (int)(m / 8);
  const bool st = all_stencil(A);
  if (nblk == 1)
  {
    // one column block: grouped quad (k_sell_mv8g, MB = 1): 119 vs 131 us for the lane-per-row
    // mapping on the 7-point SpMM at 128^3, 221 vs 241 us on the 15-point P1 mass matrix
    const i64 gcap = (i64)A.ctx->num_cu * 4 / 2;
    const i64 nunits = (A.nslices + 3) / 4;
    const i64 gx = std::max<i64>(8, std::min<i64>(gcap, (nunits + 7) / 8 * 8) / 8 * 8);
    const i64 prow = A.bandwidth > 0 ? A.bandwidth : std::max<i64>(1, A.nb_rows);
    const i64 per = std::max<i64>(1, (prow + 8 * 256 - 1) / (8 * 256));
#define EIGMI_GRP(STV)                                                                                         \
  hipLaunchKernelGGL((k_sell_mv8g<1, 2, STV, EPI>), dim3((unsigned)gx), dim3(256), 0, s, A.nb_rows, A.nslices, \
                     A.slice_ptr, A.val, A.col, A.st_delta, A.st_mask, X, Y, A.window, A.own_offset, 0, Bv, dinv, \
                     omega, gamma, per)
    if (st) EIGMI_GRP(true);
    else EIGMI_GRP(false);
#undef EIGMI_GRP
  }
  else
  {
    // quad: 4 column blocks (32 columns) per matrix pass, 4 entries in flight, 2-wave workgroups;
    // grid from the XCD-aware schedule (k_sell_mv8q)
    constexpr int MBq = 4;
    constexpr int W = 2;
    const i64 nunits = A.nslices * (4 / W);
    const i64 rows_per_unit = 16 * W;
    // resident 2-wave workgroups at the kernel's occupancy (4 waves / SIMD for MB = 4, 8 for MB = 2),
    // a multiple of 8 (one share per XCD)
    const i64 resident = (i64)A.ctx->num_cu * 4 * 4 / W;
    // half the resident capacity: the plane-slab working set (front + the previous and next
    // planes' segments) then fits the XCD's 4 MiB L2 better (tools/spmm_sweep.py: -10 % time on
    // the 7-point SpMM / Chebyshev step at 224^3, equal on the 15-point P1 mass)
    const i64 gcap = resident / 2;
    const i64 gx = std::max<i64>(8, std::min<i64>(gcap, (nunits + 7) / 8 * 8) / 8 * 8);
    // plane segment: bandwidth rows / 8, in units (at least 1); no bandwidth (diagonal): 1/8 of all
    const i64 prow = A.bandwidth > 0 ? A.bandwidth : std::max<i64>(1, A.nb_rows);
    const i64 per = std::max<i64>(1, (prow + 8 * rows_per_unit - 1) / (8 * rows_per_unit));
    for (int b0 = 0; b0 < nblk; b0 += MBq)
    {
      const int nb = nblk - b0 < MBq ? nblk - b0 : MBq;
#define EIGMI_QUAD(MBV, STV)                                                                                        \
  hipLaunchKernelGGL((k_sell_mv8q<MBV, 4, W, STV, EPI>), dim3((unsigned)gx), dim3(64 * W), 0, s, A.nb_rows, A.nslices, \
                     A.slice_ptr, A.val, A.col, A.st_delta, A.st_mask, X, Y, A.window, A.own_offset, b0, Bv, dinv,     \
                     omega, gamma, per)
#define EIGMI_QUAD_NB(STV)            \
  switch (nb)                         \
  {                                   \
    case 1: EIGMI_QUAD(1, STV); break; \
    case 2: EIGMI_QUAD(2, STV); break; \
    case 3: EIGMI_QUAD(3, STV); break; \
    default: EIGMI_QUAD(4, STV); break; \
  }
      if (st)
      {
        EIGMI_QUAD_NB(true)
      }
      else
      {
        EIGMI_QUAD_NB(false)
      }
#undef EIGMI_QUAD_NB
#undef EIGMI_QUAD
    }
  }
  EIG_HIP(hipGetLastError());
}
}  // namespace

int sell_mv8_launches(i64 m)
{
  // (the Chebyshev step the caller counts never takes the march)
  const int nblk = (int)(m / 8);
  if (nblk <= 1) return nblk;
  return (nblk + 3) / 4;
}

void launch_sell_mv8(const eig_mat_s &A, i64 m, const double *X, double *Y, hipStream_t s)
{
  // symmetric band image with a marchable band (3-D / 2-D stencils): k_spmm8_march (k_spmv.hip)
  // 3-D box stencils (7-point, P1 Kuhn), 32 columns per matrix pass: LDS-tiled plane march (k_box.hip)
  if (launch_box_spmm(A, m, X, Y, s)) return;
  if (launch_spmm_march(A, m, X, Y, s)) return;
  sell_mv8<kStore>(A, m, X, Y, nullptr, nullptr, 0.0, 0.0, s);
}

void launch_resid_mv8(const eig_mat_s &A, i64 m, const double *X, const double *B, double *R, hipStream_t s)
{
  // R = B - A X; R may be B (each row reads its own B entry before writing it), never X
  if (launch_box_resid(A, m, X, B, R, s)) return;
  sell_mv8<kResid>(A, m, X, R, B, nullptr, 0.0, 0.0, s);
}

void launch_cheb_step(const eig_mat_s &M, i64 m, const double *Xk, double *Xold, const double *B, const double *dinv,
                      double omega, double gamma, hipStream_t s)
{
  // symmetric band image with a marchable band (the P1 mass matrix of config C5): k_spmm8_marchg
  if (launch_box_cheb(M, m, Xk, Xold, B, dinv, omega, gamma, s)) return;
  if (launch_cheb_march(M, m, Xk, Xold, B, dinv, omega, gamma, s)) return;
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
  double *part = (double *)ctx_buffer(ctx, 8, (size_t)gx * ny * E * sizeof(double));  // slot 8: panel partials
  hipLaunchKernelGGL((k_panel_gram_part<TI, TJ>), dim3(gx, ny), dim3(256), 0, s, n, ld, (int)m1, (int)m2, nbj, Q1, Q2,
                     part);
  EIG_HIP(hipGetLastError());
  hipLaunchKernelGGL((k_panel_gram_reduce<TI, TJ>), dim3((unsigned)(((i64)ny * E + 63) / 64)), dim3(256), 0, s, gx, ny,
                     nbj, (int)m1, (int)m2, part, G);
  EIG_HIP(hipGetLastError());
}
}  // namespace

// The block Lanczos panel products run on the a6 Gram kernel (k_mv8.hip launch_gram_panel: paired
// 16-column tiles, one launch with its deterministic two-level reduction); the two-launch form
// above (k_panel_gram_part + k_panel_gram_reduce) is kept as launch_panel_gram_2stage for A/B.
void launch_panel_gram(eig_ctx_t ctx, i64 n, i64 ld, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G,
                       hipStream_t s)
{
  launch_gram_panel(ctx, n, ld, m1, m2, Q1, Q2, G, s);
}

void launch_panel_gram_2stage(eig_ctx_t ctx, i64 n, i64 ld, i64 m1, i64 m2, const double *Q1, const double *Q2,
                              double *G, hipStream_t s)
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

// ---------------------------------------------------------------------------------------------
// CholQR's small factorisation on the device (block Lanczos, blanczos.cpp mcholqr2): one workgroup
// takes the b x b M-Gram G (b <= 32), symmetrises it, factors G = R^T R (upper R), inverts R and
// folds R into the running product Rtot <- R Rtot (pass 0: Rtot = I).  The same operations in the
// same order as the host chol_upper / tri_upper_inv (dense.cpp) and mcholqr2's product -- each
// entry's sum sequential in one thread, correctly rounded sqrt and division, no contraction -- so
// the factors are the host's bit for bit.  A non-positive pivot sets *flag (the caller reports
// EIG_ERR_BREAKDOWN at its next synchronisation).  Row-major b x b everywhere.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_chol_small(int b, int pass, const double *__restrict__ G, double *R,
                                                    double *Ri, double *Rtot, int *flag)
{
  __shared__ double g[32][32], r[32][32], ri[32][32], rt[32][32];
  const int t = threadIdx.x;
  for (int e = t; e < b * b; e += 256)
  {
    const int i = e / b, j = e % b;
    g[i][j] = G[e];
    r[i][j] = 0.0;
    ri[i][j] = 0.0;
    rt[i][j] = pass == 0 ? (i == j ? 1.0 : 0.0) : Rtot[e];
  }
  __syncthreads();
  for (int e = t; e < b * b; e += 256)
  {
    const int i = e / b, j = e % b;
    if (i < j)  // (each pair read and written by its i < j thread only)
    {
      const double v = 0.5 * (g[i][j] + g[j][i]);
      g[i][j] = v;
      g[j][i] = v;
    }
  }
  __syncthreads();
  for (int j = 0; j < b; ++j)
  {
    if (t == 0)
    {
      double s = g[j][j];
      for (int k = 0; k < j; ++k) s -= r[k][j] * r[k][j];
      if (!(s > 0.0)) *flag = 1;
      r[j][j] = sqrt(s);
    }
    __syncthreads();
    const double rjj = r[j][j];
    for (int i = j + 1 + t; i < b; i += 256)
    {
      double u = g[j][i];
      for (int k = 0; k < j; ++k) u -= r[k][j] * r[k][i];
      r[j][i] = u / rjj;
    }
    __syncthreads();
  }
  if (t < b)  // column c = t of R^-1, back substitution
  {
    const int c = t;
    for (int i = c; i >= 0; --i)
    {
      double s = (i == c) ? 1.0 : 0.0;
      for (int k = i + 1; k <= c; ++k) s -= r[i][k] * ri[k][c];
      ri[i][c] = s / r[i][i];
    }
  }
  __syncthreads();
  for (int e = t; e < b * b; e += 256)
  {
    const int i = e / b, j = e % b;
    double acc = 0.0;
    for (int q = i; q <= j; ++q) acc += r[i][q] * rt[q][j];
    R[e] = r[i][j];
    Ri[e] = ri[i][j];
    Rtot[e] = acc;
  }
}

void launch_chol_small(int b, int pass, const double *G, double *R, double *Ri, double *Rtot, int *flag,
                       hipStream_t s)
{
  EIG_CHECK(b >= 1 && b <= 32, EIG_ERR_ARG, "chol_small: b <= 32");
  hipLaunchKernelGGL(k_chol_small, dim3(1), dim3(256), 0, s, b, pass, G, R, Ri, Rtot, flag);
  EIG_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// CholQR2's middle step fused (blanczos.cpp mcholqr2, b = 32 columns = 4 blocks): with S = R^-1 of
// the first pass (upper triangular, row-major 32 x 32), Z <- Z' = Z S and G = Z'^T (MZ S) in ONE
// pass over Z and MZ -- MZ S (the first pass's update of M Z) is never stored, and Z' is not read
// back for the second Gram.  Both products on v_mfma_f64_16x16x4f64, 16 rows per wave iteration:
//  * transform: lane (k, i) loads row i's columns 2k, 2k + 1 of each 8-column block (a 16-B load;
//    one wave instruction reads 16 whole 64-B rows) and the MFMA h of block kb takes inner index
//    k -> column 8 kb + 2 k + h, with B[k][j] = S[8 kb + 2 k + h][16 t + j] held in registers for
//    the whole launch.  S is upper triangular, so output columns 0..15 need blocks 0 and 1 only;
//  * the transform's output layout (lane (k, i), register q: row k + 4 q, column 16 t + i) is the
//    Gram MFMA's operand layout for the row group q, so Z' and MZ' go from the accumulators into
//    the Gram MFMAs without any exchange; Z' is stored from the same registers (in place: a wave
//    reads its 16 rows completely before it writes them).
// The Gram sums are reduced as k_gram_mv8's: waves in order into one LDS image, then grid_sum2.
// Not bitwise the two-launch form (the MFMA's four-term products round differently from
// k_panel_update's FMA chain); the block Lanczos results are checked against scipy.
// ---------------------------------------------------------------------------------------------
constexpr int kFoldThreads = 256;

__global__ __launch_bounds__(kFoldThreads) void k_cholqr_fold(i64 n, i64 ld, double *Z, const double *__restrict__ MZ,
                                                              const double *__restrict__ S, double *__restrict__ G,
                                                              double *partials, unsigned *tickets)
{
  constexpr int E = 4 * 256;  // the 2 x 2 tiles of 16 x 16
  __shared__ double red[E];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k = lane >> 4, i = lane & 15;
  double sb[4][2][2];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 2; ++t) sb[kb][h][t] = S[(8 * kb + 2 * k + h) * 32 + 16 * t + i];
  d4 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[t][u] = d4{0.0, 0.0, 0.0, 0.0};
  const i64 ntile = (n + 15) / 16;
  const i64 ws = (i64)gridDim.x * (kFoldThreads / 64);
  for (i64 tile = (i64)blockIdx.x * (kFoldThreads / 64) + wave; tile < ntile; tile += ws)
  {
    const i64 r = tile * 16 + i;
    const bool ok = r < n;
    const i64 rr = ok ? r : 0;
    dv2 zv[4], mv[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
    {
      zv[kb] = *reinterpret_cast<const dv2 *>(Z + ((i64)kb * ld + rr) * 8 + 2 * k);
      mv[kb] = *reinterpret_cast<const dv2 *>(MZ + ((i64)kb * ld + rr) * 8 + 2 * k);
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
    {
      zv[kb] = ok ? zv[kb] : dv2{0.0, 0.0};
      mv[kb] = ok ? mv[kb] : dv2{0.0, 0.0};
    }
    d4 zt[2], mt[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) zt[t] = mt[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          if (t == 1 || kb < 2)
          {
            zt[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(zv[kb][h], sb[kb][h][t], zt[t], 0, 0, 0);
            mt[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(mv[kb][h], sb[kb][h][t], mt[t], 0, 0, 0);
          }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q)
      {
        const i64 row = tile * 16 + 4 * q + k;
        if (row < n) Z[((i64)(2 * t + (i >> 3)) * ld + row) * 8 + (i & 7)] = zt[t][q];
      }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(zt[t][q], mt[u][q], acc[t][u], 0, 0, 0);
  }
  for (int w = 0; w < kFoldThreads / 64; ++w)
  {
    if (wave == w)
    {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int q = 0; q < 4; ++q)
          {
            const int e = (t * 2 + u) * 256 + (k + 4 * q) * 16 + i;
            red[e] = w == 0 ? acc[t][u][q] : red[e] + acc[t][u][q];
          }
    }
    __syncthreads();
  }
  if (!grid_sum2<kFoldThreads>(red, E, partials, partials + (size_t)gridDim.x * E, tickets, blockIdx.x, gridDim.x,
                               red))
    return;
  for (int e = threadIdx.x; e < E; e += kFoldThreads)
  {
    const int tu = e / 256, t = tu / 2, u = tu % 2, el = e % 256;
    G[(16 * t + el / 16) * 32 + 16 * u + el % 16] = red[e];
  }
}

void launch_cholqr_fold(eig_ctx_t ctx, i64 n, i64 ld, double *Z, const double *MZ, const double *S, double *G,
                        hipStream_t s)
{
  constexpr int E = 4 * 256;
  const i64 ntile = (n + 15) / 16;
  // two workgroups per CU (122 VGPRs + 48 AGPRs: two waves per SIMD)
  const int gx = (int)std::max<i64>(1, std::min<i64>(512, (ntile + 3) / 4));
  double *part = (double *)ctx_buffer(ctx, 8, (size_t)(gx + 8) * E * sizeof(double));
  hipLaunchKernelGGL(k_cholqr_fold, dim3(gx), dim3(kFoldThreads), 0, s, n, ld, Z, MZ, S, G, part,
                     ctx->red.ticket(0));
  EIG_HIP(hipGetLastError());
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
