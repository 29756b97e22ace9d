// k_trsv.hip -- Qout = A^-1 Qin from exported LU factors (matmul_inverse_tallskinny_blocked,
// kernels_cpp.hh:660-755) on gfx950.
//
//   k_perm_scale   Qout(k, :) = scale[k] Qin(P[k], :)           (row scaling + row permutation)
//   k_lsolve       Qin = L^-1 Qout   (unit lower, rows in ascending column order)
//   k_usolve       Qin = U^-1 Qin    (rows in DESCENDING column order = the reference's push order)
//   k_perm_out     Qout(Q[j], :) = Qin(j, :)
//
// The solves keep the reference's per-row operation sequence (sum = rhs; sum -= l * x_j for the
// stored entries in order; U: x = sum / u_ii), so results are bitwise the reference's.  A triangular
// solve is a dependency chain over the rows, so the mapping buys latency, not bandwidth: one
// workgroup per 8-column block, one wave per column, 64-row blocks in sequence.  Per block:
//   phase 1  lane r subtracts every entry of row bs + r whose column lies BEFORE the block (all
//            already solved; a prefix of the row, its end usplit / lsplit precomputed), loads
//            issued eight at a time, x of the last three solved blocks read from an LDS ring;
//   phase 2  the in-block entries sit in an LDS tile (tile[t][r], bit t of mask[r]); step t
//            broadcasts row bs + t's final value with readlane and every lane r > t subtracts its
//            entry in column bs + t -- a register wavefront, no barrier inside the block.
// U runs the blocks bottom-up with t descending.  x of earlier blocks is re-read by the same
// workgroup after a __syncthreads (workgroup-scope ordering).
// Default where the factor fits the staged image: the block-inverse solve (k_binv_z +
// k_binv_chain below; to rounding, not bitwise); EIGMI_TRSV=staged / csr keep the bitwise kernels.
#include "internal.h"

#include <atomic>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <thread>

namespace eigmi {

namespace {
constexpr int kTB = 64;       // rows per block
constexpr int kTThreads = 512;  // 8 waves = the 8 columns of a column block
constexpr int kRing = 3;        // solved blocks whose x stays in LDS for phase 1
constexpr int kThreadsT = kTThreads;

__global__ __launch_bounds__(256) void k_perm_scale(i64 n, int nblk, const i32 *__restrict__ P,
                                                    const double *__restrict__ scale, const double *__restrict__ Qin,
                                                    double *__restrict__ Qout)
{
  const i64 total = n * nblk;
  for (i64 idx = (i64)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (i64)gridDim.x * 256)
  {
    const i64 b = idx / n, k = idx - b * n;
    const double sc = scale[k];
    const double *src = Qin + (b * n + P[k]) * 8;
    double *dst = Qout + (b * n + k) * 8;
#pragma unroll
    for (int s = 0; s < 8; ++s) dst[s] = sc * src[s];
  }
}

__global__ __launch_bounds__(256) void k_perm_out(i64 n, int nblk, const i32 *__restrict__ Q,
                                                  const double *__restrict__ Xin, double *__restrict__ Qout)
{
  const i64 total = n * nblk;
  for (i64 idx = (i64)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (i64)gridDim.x * 256)
  {
    const i64 b = idx / n, j = idx - b * n;
    const double *src = Xin + (b * n + j) * 8;
    double *dst = Qout + (b * n + Q[j]) * 8;
#pragma unroll
    for (int s = 0; s < 8; ++s) dst[s] = src[s];
  }
}

// Explicit global-address-space access (addrspace 1): a generic (flat) access would also count on
// lgkmcnt, so every LDS wait of the solve loops would wait for it too.
typedef __attribute__((address_space(1))) double gdouble;
__device__ __forceinline__ double gld(const double *p) { return *(const gdouble *)p; }
__device__ __forceinline__ void gst(double *p, double v) { *(gdouble *)p = v; }

// Wave-uniform broadcast of lane t's double (two v_readlane_b32: scalar, no LDS crossbar).
__device__ __forceinline__ double lane_bcast(double v, int t)
{
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffull), t);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), t);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// LOWER = true: L solve (blocks top-down, unit diagonal); false: U solve (bottom-up, divide by d).
// rhs and x are the column block's base pointers (n rows of 8); x may equal rhs (U solve).
template <bool LOWER>
__global__ __launch_bounds__(kTThreads) void k_tsolve(i64 n, const i64 *__restrict__ rp, const i64 *__restrict__ split,
                                                      const i32 *__restrict__ cj, const double *__restrict__ cv,
                                                      const double *__restrict__ diag, const double *rhs, double *x)
{
  __shared__ double tile[kTB][kTB];  // tile[t][r]: entry (row bs + r, column bs + t)
  __shared__ unsigned long long tmask[kTB];
  // x of the kRing most recently solved blocks, per column: ring[slot][row][col]; a phase-1 entry
  // whose column falls in one of them is read from LDS instead of global memory
  __shared__ double ring[kRing][kTB][8];
  const int r = threadIdx.x & 63;
  const int c = threadIdx.x >> 6;  // column inside the block of 8
  const i64 cb = (i64)blockIdx.x * n * 8;
  const double *R = rhs + cb;
  double *X = x + cb;
  const i64 nblocks = (n + kTB - 1) / kTB;
  for (i64 bi = 0; bi < nblocks; ++bi)
  {
    const i64 blk = LOWER ? bi : nblocks - 1 - bi;
    const i64 bs = blk * kTB;
    const i64 i = bs + r;
    const bool valid = i < n;
    double sum = valid ? R[i * 8 + c] : 0.0;
    i64 k = valid ? rp[i] : 0;
    const i64 ks = valid ? split[i] : 0, ke = valid ? rp[i + 1] : 0;
    // blocks [lo_blk, hi_blk] are in the ring (the kRing blocks solved last)
    const i64 nring = bi < kRing ? bi : kRing;
    const i64 lo_blk = LOWER ? blk - nring : blk + 1, hi_blk = LOWER ? blk - 1 : blk + nring;
    // the block's own entries into the LDS tile: all 8 waves, wave c takes entries c, c+8, ... of
    // each row (a band of 64 is one load round); the row masks are OR-ed together in LDS
    if (c == 0) tmask[r] = 0ull;
    __syncthreads();
    {
      unsigned long long mm = 0;
      for (i64 q0 = ks + c; q0 < ke; q0 += 64)
      {
        double a[8];
        i32 cc[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
        {
          const i64 q = q0 + 8 * u;
          const i64 qq = q < ke ? q : ke - 1;
          a[u] = cv[qq];
          cc[u] = cj[qq];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (q0 + 8 * u < ke)
          {
            const int t = (int)(cc[u] - bs);
            tile[t][r] = a[u];
            mm |= 1ull << t;
          }
      }
      if (mm) atomicOr(&tmask[r], mm);
    }
    // phase 1: entries outside the block (columns before it for L, after it for U), in order;
    // the loads of 32 entries are issued before the 32 dependent subtractions, x of the recent
    // blocks comes from the LDS ring
    auto xval = [&](i64 col) -> double {
      const i64 cbk = col / kTB;
      if (nring > 0 && cbk >= lo_blk && cbk <= hi_blk) return ring[cbk % kRing][col - cbk * kTB][c];
      return X[col * 8 + c];
    };
    for (; k < ks; k += 32)
    {
      double a[32];
      i32 cc[32];
#pragma unroll
      for (int u = 0; u < 32; ++u)
      {
        const i64 q = k + u < ks ? k + u : ks - 1;
        a[u] = cv[q];
        cc[u] = cj[q];
      }
#pragma unroll
      for (int u = 0; u < 32; ++u)
        if (k + u < ks) sum -= a[u] * xval(cc[u]);
    }
    __syncthreads();
    const unsigned long long m = tmask[r];
    const int nb = (int)((n - bs) < kTB ? (n - bs) : kTB);
    double mine = 0.0;
    if (LOWER)
    {
      for (int t = 0; t < nb; ++t)
      {
        const double xt = lane_bcast(sum, t);  // row bs + t is final
        if (r == t) mine = xt;
        if (r > t && ((m >> t) & 1ull)) sum -= tile[t][r] * xt;
      }
    }
    else
    {
      for (int t = nb - 1; t >= 0; --t)
      {
        const double xt = lane_bcast(sum, t) / diag[bs + t];  // x = (rhs - sum_j u x_j) / u_tt
        if (r == t) mine = xt;
        if (r < t && ((m >> t) & 1ull)) sum -= tile[t][r] * xt;
      }
    }
    if (valid) X[i * 8 + c] = mine;
    ring[blk % kRing][r][c] = mine;
    __syncthreads();  // ring / x of this block visible to the next; the tile free for reuse
  }
}

// Block-staged triangular solve (default when the factor fits it: at most kSlab outside-the-block
// entries per row and every one within the kRing4 blocks solved last -- envelope factors of
// bandwidth <= 256; other factors take k_tsolve).  Same per-row operation sequence as k_tsolve
// (bitwise equal), but every global load of a block is coalesced and issued one block AHEAD: the
// 512 threads load block b+1's ELL slab of outside-the-block entries ([k][r]: 64 rows per
// instruction) and its dense in-block tile into registers during block b's register wavefront; at
// staging the columns become ring indices, so phase 1 is LDS reads and selected subtractions
// without per-entry branches.
constexpr int kRing4 = 4;   // ring slots of the staged kernel (power of two)
constexpr int kSlab = 128;  // slab entries per row staged at once (LDS: 96 KiB of slab + 32 KiB tile)
// block-inverse image: at most kBinvMaxGD coupled blocks per factor (envelope bandwidth <= 512 rows)
// and kBinvTiles 64 x 64 double tiles for both factors (1 GiB); a diagonal block whose estimated
// condition max|D_b| max|inv(D_b)| 64 exceeds kBinvCond keeps the factors on the substitution
// kernels (products with an inverse of an ill-conditioned block lose what substitution keeps)
constexpr int kBinvMaxGD = 8;
constexpr i64 kBinvTiles = 32768;
constexpr double kBinvCond = 1e6;

struct Staged {
  const i64 *off1;
  const i32 *w1;
  const double *v1;
  const i32 *c1;
  const double *tile;
  const unsigned long long *tmask;
};

template <bool LOWER>
__global__ __launch_bounds__(kTThreads) void k_tsolve_staged(i64 n, Staged F, const double *__restrict__ diag,
                                                             const double *rhs, double *x)
{
  __shared__ double tile[kTB][kTB];  // tile[t][r]
  __shared__ unsigned long long tmask[kTB];
  __shared__ double sv[kSlab][kTB];  // slab chunk: value of entry k of row r
  __shared__ i32 sc[kSlab][kTB];     // its column (-1: padding)
  // x of the kRing4 most recently solved blocks, [slot][column c][row]: a phase-1 read by lane r
  // of a banded row hits consecutive rows, i.e. distinct banks (a [row][c] layout would put the
  // 64 lanes 64 B apart: 16-way bank conflicts)
  __shared__ double ring[kRing4][8][kTB];
  const int tid = threadIdx.x, r = tid & 63, c = tid >> 6;
  const i64 cb = (i64)blockIdx.x * n * 8;
  const double *R = rhs + cb;
  double *X = x + cb;
  const i64 nblocks = (n + kTB - 1) / kTB;
  // prefetch registers: 8 tile doubles, 8 slab entries (value, column) per thread, one mask
  constexpr int kQ = kSlab * kTB / kThreadsT;  // slab entries per thread per chunk
  double pt[8], pv[kQ];
  i32 pc[kQ];
  unsigned long long pm = 0;
  int pw = 0;
  // one block's staging loads: all at fixed, block-indexed addresses (no dependent metadata load,
  // no predicates), so they stay in flight until the next block's staging consumes them
  auto prefetch = [&](i64 blk) {
    const double *tg = F.tile + blk * (kTB * kTB);
    const double *vg = F.v1 + blk * (kSlab * kTB);
    const i32 *cg = F.c1 + blk * (kSlab * kTB);
#pragma unroll
    for (int q = 0; q < 8; ++q) pt[q] = tg[q * kThreadsT + tid];
#pragma unroll
    for (int q = 0; q < kQ; ++q)
    {
      pv[q] = vg[q * kThreadsT + tid];  // entry k = q * 8 + c of row r
      pc[q] = cg[q * kThreadsT + tid];
    }
    pm = F.tmask[blk * kTB + r];
    pw = F.w1[blk];
  };
  prefetch(LOWER ? 0 : nblocks - 1);
  for (i64 bi = 0; bi < nblocks; ++bi)
  {
    const i64 blk = LOWER ? bi : nblocks - 1 - bi;
    const i64 bs = blk * kTB;
    const i64 i = bs + r;
    const bool valid = i < n;
    double sum = valid ? gld(R + i * 8 + c) : 0.0;
    const int w1 = pw;
    // stage the prefetched block into LDS
    const double dr = (!LOWER && valid) ? gld(diag + i) : 1.0;  // U pivot of row i
#pragma unroll
    for (int q = 0; q < 8; ++q)
    {
      const int e = q * kThreadsT + tid;
      tile[e >> 6][e & 63] = pt[q];
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q)
    {
      const int e = q * kThreadsT + tid;
      sv[e >> 6][e & 63] = pv[q];
      // column -> its x in the ring: slot (block mod kRing4) * 512 + row (the column offset c * 64
      // is added by the reading wave)
      sc[e >> 6][e & 63] = pc[q] < 0 ? -1 : ((((pc[q] >> 6) & (kRing4 - 1)) << 9) | (pc[q] & 63));
    }
    if (c == 0) tmask[r] = pm;
    __syncthreads();
    // phase 1: the outside-the-block entries of row r in entry order (at most kSlab, all in the
    // ring: the host admits a factor to this kernel only then), 8 per round: their LDS reads are
    // issued before the 8 dependent subtractions; stored entries are selected, never branched on
    const double *rf = &ring[0][c][0];
    for (int kk = 0; kk < w1; kk += 8)
    {
      i32 ix[8];
      double a[8], xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
      {
        ix[u] = sc[(kk + u) & (kSlab - 1)][r];  // ring index (slot * 512 + row) or -1
        a[u] = sv[(kk + u) & (kSlab - 1)][r];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) xv[u] = rf[ix[u] < 0 ? 0 : ix[u]];
#pragma unroll
      for (int u = 0; u < 8; ++u)
      {
        const double upd = sum - a[u] * xv[u];
        sum = (kk + u < w1 && ix[u] >= 0) ? upd : sum;
      }
    }
    // next block's staging loads fly during the wavefront and the end-of-block barrier
    if (bi + 1 < nblocks) prefetch(LOWER ? blk + 1 : blk - 1);
    // this lane's update mask: stored in-block entries in the columns solved before its row
    const unsigned long long m = tmask[r] & (LOWER ? ((1ull << r) - 1ull) : ~((2ull << r) - 1ull));
    const int nb = (int)((n - bs) < kTB ? (n - bs) : kTB);
    // register wavefront, 8 steps per round: the round's tile entries are read from LDS before its
    // chain of broadcasts, the round's 8 mask bits come from one 32-bit shift.  A lane's own row
    // is final once the wavefront passes it (no later step updates it), so its x is read off its
    // sum after the loop (U: sum / u_rr, the same division the broadcast step performs).
    const int nb8 = (nb + 7) & ~7;
    if (LOWER)
    {
      for (int t0 = 0; t0 < nb; t0 += 8)
      {
        double tv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) tv[u] = tile[(t0 + u) & 63][r];
        const unsigned mr = (unsigned)(m >> t0);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (t0 + u < nb)
          {
            const double xt = lane_bcast(sum, t0 + u);  // row bs + t is final
            const double upd = sum - tv[u] * xt;
            sum = ((mr >> u) & 1u) ? upd : sum;  // stored entries of rows below t only
          }
      }
    }
    else
    {
      for (int t0 = nb8 - 8; t0 >= 0; t0 -= 8)
      {
        double tv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) tv[u] = tile[(t0 + 7 - u) & 63][r];
        const unsigned mr = (unsigned)(m >> t0);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (t0 + 7 - u < nb)
          {
            const int t = t0 + 7 - u;
            const double xt = lane_bcast(sum, t) / lane_bcast(dr, t);  // x = (rhs - sum u x) / u_tt
            const double upd = sum - tv[u] * xt;
            sum = ((mr >> (7 - u)) & 1u) ? upd : sum;  // stored entries of rows above t only
          }
      }
    }
    const double mine = LOWER ? sum : sum / dr;
    if (valid) gst(X + i * 8 + c, mine);
    ring[blk & (kRing4 - 1)][c][r] = mine;
    // ring visible to the next block, LDS staging free for reuse: an LDS-only barrier (x is never
    // re-read from global memory here), so the next block's staging loads stay in flight
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
}

// Block-inverse solve (the default when the factor fits the staged image and the block-inverse
// image is small enough; not bitwise: the products with inv(D_b) round differently from the
// substitution, agreement with the reference arithmetic is to ~1e-15 relative).  With D_b the
// 64 x 64 diagonal block b of the factor, T(b, d) its coupling to the block d away (d <= kRing4),
// z_b = inv(D_b) y_b and G(b, d) = inv(D_b) T(b, d) (both built on the host at upload):
//     x_b = z_b - sum_d G(b, d) x_(b -+ d).
// z for all blocks is one parallel launch (k_binv_z); the chain over the blocks (k_binv_chain)
// has no dependency inside a block, so a block costs a few dense 64 x 64 x 8 products and one
// barrier instead of a 64-step register wavefront.  Independent of the staged image: any factor
// whose off-block entries lie within kBinvMaxGD blocks (the RCM envelope of a 200^2 grid: gd 7).
//
// k_binv_z: one workgroup per (64-row block, 8-column block); PERM: y = scale * Qin(P, :) (the
// row scaling + permutation of the L solve), else y = Y.  Thread (r, s) forms the partial products
// of row r over the columns t of slice s (8 t), the slices are summed in LDS in a fixed order.
template <bool PERM>
__global__ __launch_bounds__(kThreadsT) void k_binv_z(i64 n, const double *__restrict__ dinv, const i32 *__restrict__ P,
                                                      const double *__restrict__ scale, const double *__restrict__ Y,
                                                      double *__restrict__ Z)
{
  __shared__ double ys[kTB][8];
  __shared__ double part[8][kTB][9];  // rows padded to 9 doubles: lane r's stores on distinct banks
  const int tid = threadIdx.x, r = tid & 63, s = tid >> 6;
  const i64 b = blockIdx.x, bs = b * kTB, cb = (i64)blockIdx.y * n * 8;
  {
    const int t = tid >> 3, c = tid & 7;
    const i64 i = bs + t;
    double v = 0.0;
    if (i < n) v = PERM ? scale[i] * Y[cb + (i64)P[i] * 8 + c] : Y[cb + i * 8 + c];
    ys[t][c] = v;
  }
  const double *D = dinv + b * (kTB * kTB);
  double g[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) g[q] = D[(s * 8 + q) * kTB + r];
  __syncthreads();
  double acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = fma(g[q], ys[s * 8 + q][c], acc[c]);
#pragma unroll
  for (int c = 0; c < 8; ++c) part[s][r][c] = acc[c];
  __syncthreads();
  const int t = tid >> 3, c = tid & 7;
  double z = part[0][t][c];
#pragma unroll
  for (int q = 1; q < 8; ++q) z += part[q][t][c];
  if (bs + t < n) Z[cb + (bs + t) * 8 + c] = z;
}

// k_binv_chain: one workgroup per 8-column block, the blocks in sequence (L top-down, U bottom-up).
// Thread (r, s) multiplies the G entries of row r in slice s with the solved x rows of that slice,
// which wave s keeps in a private LDS ring (broadcast reads); the partial sums of the 8 slices meet
// in LDS (double-buffered by block parity, so one barrier per block), and lane (u, c) of wave s
// finishes x(row s*8+u, column c) = z - sum, the rows its wave needs from this block later.
// GD = coupled blocks (G tiles per block, gd <= GD at run time), RING = ring slots (>= GD, power of
// two).  The G tiles and z of the next PF
// blocks are in flight in a register ring (PF buffers, the loop unrolled by PF so every buffer index
// is static).  The partials' rows are padded to 9 doubles: lane r's 8 stores then fall on distinct
// banks (a 64-B row stride put 8 lanes on each bank pair).
template <bool LOWER, int GD, int PF, int RING>
__global__ __launch_bounds__(kThreadsT) void k_binv_chain(i64 n, int gd, const double *__restrict__ G,
                                                          const double *Z, double *X)
{
  static_assert(RING >= GD && (RING & (RING - 1)) == 0, "ring slots");
  __shared__ double part[2][8][kTB][9];
  __shared__ double ring[8][RING][8][8];  // [wave s][slot][row u of slice s][column]
  const int tid = threadIdx.x, r = tid & 63, s = tid >> 6;
  const int u = r >> 3, c = r & 7;  // the reduction role of lane r
  const i64 cb = (i64)blockIdx.x * n * 8;
  const i64 nblocks = (n + kTB - 1) / kTB;
#pragma unroll
  for (int q = 0; q < RING; ++q) ring[s][q][u][c] = 0.0;
  double pg[PF][GD][8], pz[PF];
  // tiles and z of the bi-th block solved.  Every load is unconditional (clamped block, tile and row
  // indices; values past the end are never used or are masked at use), the loop runs a whole number
  // of PF rounds (padded blocks compute but store nothing), and a buffer is refilled only once its
  // old contents are dead (the tiles after the products, z after x): otherwise the compiler merges
  // the loaded register into the loop-carried one with a copy right behind the load
  // (s_waitcnt vmcnt(0)), which serialised the prefetch ring on the load latency.
  auto fetch_g = [&](i64 bi, double (&g)[GD][8]) {
    const i64 bc = bi < nblocks ? bi : nblocks - 1;
    const i64 blk = LOWER ? bc : nblocks - 1 - bc;
    const double *gb = G + blk * gd * (kTB * kTB);
#pragma unroll
    for (int d = 0; d < GD; ++d)
    {
      const int dd = d < gd ? d : 0;  // (gd = 0: the one-tile placeholder buffer)
#pragma unroll
      for (int q = 0; q < 8; ++q) g[d][q] = gb[dd * (kTB * kTB) + (s * 8 + q) * kTB + r];
    }
  };
  auto fetch_z = [&](i64 bi, double &z) {
    const i64 bc = bi < nblocks ? bi : nblocks - 1;
    const i64 i = (LOWER ? bc : nblocks - 1 - bc) * kTB + s * 8 + u;
    z = gld(Z + cb + (i < n ? i : n - 1) * 8 + c);
  };
#pragma unroll
  for (int p = 0; p < PF; ++p)
  {
    fetch_g(p, pg[p]);
    fetch_z(p, pz[p]);
  }
  // the prologue's loads complete before the loop: the loop header then sees only the latch's
  // pending loads, and the first use of a round waits for its own tiles (vmcnt(N)), not vmcnt(0)
  __builtin_amdgcn_s_waitcnt(0);
  const i64 nround = (nblocks + PF - 1) / PF * PF;
  for (i64 b0 = 0; b0 < nround; b0 += PF)
  {
#pragma unroll
    for (int p = 0; p < PF; ++p)
    {
      const i64 bi = b0 + p;
      const bool live = bi < nblocks;  // (uniform)
      const i64 blk = LOWER ? bi : nblocks - 1 - bi;
      double acc[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = 0.0;
#pragma unroll
      for (int d = 0; d < GD; ++d)
        if (d < gd && d < bi)  // block blk -+ (d + 1) exists and is solved
        {
          const i64 src = LOWER ? blk - (d + 1) : blk + (d + 1);
          const double(*xr)[8] = ring[s][src & (RING - 1)];
#pragma unroll
          for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] = fma(pg[p][d][q], xr[q][k], acc[k]);
        }
      fetch_g(bi + PF, pg[p]);  // the tiles of the block PF ahead
      double(*pp)[kTB][9] = part[bi & 1];
#pragma unroll
      for (int k = 0; k < 8; ++k) pp[s][r][k] = acc[k];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS-only barrier, the tile loads stay in flight
      __builtin_amdgcn_s_barrier();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      const int t = s * 8 + u;
      double sum = pp[0][t][c];
#pragma unroll
      for (int q = 1; q < 8; ++q) sum += pp[q][t][c];
      const i64 i = blk * kTB + t;
      const bool own = live && i < n;
      const double x = (own ? pz[p] : 0.0) - sum;  // rows past n: 0 (their G columns are zero)
      ring[s][blk & (RING - 1)][u][c] = x;  // read back by this wave only (LDS is in order per wave)
      if (own) gst(X + cb + i * 8 + c, x);
      fetch_z(bi + PF, pz[p]);
      __builtin_amdgcn_wave_barrier();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
  }
}

// k_binv_chain16 (round 4): the same chain on 16 waves per column block -- wave s multiplies the
// 4 inner indices s*4 .. s*4+3 (half the products per thread, twice the waves per SIMD to hide the
// LDS / FMA latency that bounds the 8-wave chain: PMC 44 % of wave cycles waiting) and finishes
// rows s*4 .. s*4+3 of x.  Partials in LDS transposed ([slice][column][row], rows padded to 66:
// lane r's stores are consecutive, the 8 column reads of a row hit distinct banks), double-buffered
// by block parity; the same x = z - sum with the slices summed in fixed order (0 .. 15).
constexpr int kChain16 = 1024;
constexpr int kC16Pad = 66;
template <bool LOWER, int GD, int PF, int RING>
__global__ __launch_bounds__(kChain16) void k_binv_chain16(i64 n, int gd, const double *__restrict__ G,
                                                           const double *Z, double *X)
{
  static_assert(RING >= GD && (RING & (RING - 1)) == 0, "ring slots");
  __shared__ double part[2][16][8][kC16Pad];
  __shared__ __attribute__((aligned(16))) double ring[16][RING][4][8];  // [wave s][slot][row u of slice s][column]
  const int tid = threadIdx.x, r = tid & 63, s = tid >> 6;
  const int u = (r >> 3) & 3, c = r & 7;  // reduction role of lanes r < 32: row s*4+u, column c
  const bool red = r < 32;
  const i64 cb = (i64)blockIdx.x * n * 8;
  const i64 nblocks = (n + kTB - 1) / kTB;
  if (red)
#pragma unroll
    for (int q = 0; q < RING; ++q) ring[s][q][u][c] = 0.0;
  double pg[PF][GD][4], pz[PF];
  auto fetch_g = [&](i64 bi, double (&g)[GD][4]) {
    const i64 bc = bi < nblocks ? bi : nblocks - 1;
    const i64 blk = LOWER ? bc : nblocks - 1 - bc;
    const double *gb = G + blk * gd * (kTB * kTB);
#pragma unroll
    for (int d = 0; d < GD; ++d)
    {
      const int dd = d < gd ? d : 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) g[d][q] = gb[dd * (kTB * kTB) + (s * 4 + q) * kTB + r];
    }
  };
  auto fetch_z = [&](i64 bi, double &z) {
    const i64 bc = bi < nblocks ? bi : nblocks - 1;
    const i64 i = (LOWER ? bc : nblocks - 1 - bc) * kTB + s * 4 + u;
    z = gld(Z + cb + (i < n ? i : n - 1) * 8 + c);
  };
#pragma unroll
  for (int p = 0; p < PF; ++p)
  {
    fetch_g(p, pg[p]);
    fetch_z(p, pz[p]);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();  // (ring zeroed)
  typedef double d2v __attribute__((ext_vector_type(2)));
  const i64 nround = (nblocks + PF - 1) / PF * PF;
  for (i64 b0 = 0; b0 < nround; b0 += PF)
  {
#pragma unroll
    for (int p = 0; p < PF; ++p)
    {
      const i64 bi = b0 + p;
      const bool live = bi < nblocks;
      const i64 blk = LOWER ? bi : nblocks - 1 - bi;
      double acc[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = 0.0;
#pragma unroll
      for (int d = 0; d < GD; ++d)
        if (d < gd && d < bi)
        {
          const i64 src = LOWER ? blk - (d + 1) : blk + (d + 1);
          const d2v *xr = reinterpret_cast<const d2v *>(&ring[s][src & (RING - 1)][0][0]);
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int k2 = 0; k2 < 4; ++k2)
            {
              const d2v xv = xr[q * 4 + k2];
              acc[2 * k2] = fma(pg[p][d][q], xv.x, acc[2 * k2]);
              acc[2 * k2 + 1] = fma(pg[p][d][q], xv.y, acc[2 * k2 + 1]);
            }
        }
      fetch_g(bi + PF, pg[p]);
      double(*pp)[8][kC16Pad] = part[bi & 1];
#pragma unroll
      for (int k = 0; k < 8; ++k) pp[s][k][r] = acc[k];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS-only barrier, the tile loads stay in flight
      __builtin_amdgcn_s_barrier();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      const int t = s * 4 + u;
      if (red)
      {
        double sum = pp[0][c][t];
#pragma unroll
        for (int q = 1; q < 16; ++q) sum += pp[q][c][t];
        const i64 i = blk * kTB + t;
        const bool own = live && i < n;
        const double x = (own ? pz[p] : 0.0) - sum;
        ring[s][blk & (RING - 1)][u][c] = x;  // read back by this wave only (LDS is in order per wave)
        if (own) gst(X + cb + i * 8 + c, x);
      }
      fetch_z(bi + PF, pz[p]);
      __builtin_amdgcn_wave_barrier();
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
  }
}

// 16-wave chain (k_binv_chain16) unless EIGMI_BINV_CHAIN=8 (the 8-wave k_binv_chain, A/B)
// (ADVICE-style note: an environment switch for measurement only, as EIGMI_TRSV)
static bool binv_chain16()
{
  static const bool on = [] {
    const char *e = std::getenv("EIGMI_BINV_CHAIN");
    return !(e && std::strcmp(e, "8") == 0);
  }();
  return on;
}

template <bool LOWER>
void launch_binv_chain(int gd, int nblk, i64 n, const double *G, const double *Z, double *X, hipStream_t s)
{
  // 16 waves for 3 or 4 coupled blocks (the 8-slot ring of gd > 4 does not fit beside the partials).
  // Measured (profiles/r04ab_*): 200^2 GenEO pencil (gd 4) matmul_inverse 4.05 vs 4.88 ms,
  // GeneralizedInverse 1.39 vs 1.65 s; at 64^2 (gd 1) the 8-wave chain is faster (178 vs 200 us)
  if (binv_chain16() && gd >= 3 && gd <= 4)
  {
    hipLaunchKernelGGL((k_binv_chain16<LOWER, 4, 2, 4>), dim3(nblk), dim3(kChain16), 0, s, n, gd, G, Z, X);
    return;
  }
  // prefetch depth by register budget: PF x GD x 8 doubles per thread (512-thread workgroups: up to
  // 256 VGPRs per lane)
  if (gd <= 1)
    hipLaunchKernelGGL((k_binv_chain<LOWER, 1, 4, 4>), dim3(nblk), dim3(kThreadsT), 0, s, n, gd, G, Z, X);
  else if (gd == 2)
    hipLaunchKernelGGL((k_binv_chain<LOWER, 2, 3, 4>), dim3(nblk), dim3(kThreadsT), 0, s, n, gd, G, Z, X);
  else if (gd <= 4)
    hipLaunchKernelGGL((k_binv_chain<LOWER, 4, 2, 4>), dim3(nblk), dim3(kThreadsT), 0, s, n, gd, G, Z, X);
  else
    hipLaunchKernelGGL((k_binv_chain<LOWER, 8, 1, 8>), dim3(nblk), dim3(kThreadsT), 0, s, n, gd, G, Z, X);
}

int grid256(i64 work)
{
  i64 g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

template <class T>
T *upload(const std::vector<T> &h, hipStream_t stream)
{
  void *p = nullptr;
  EIG_HIP(hipMalloc(&p, std::max<size_t>(h.size(), 1) * sizeof(T)));
  if (!h.empty())
  {
    EIG_HIP(hipMemcpyAsync(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, stream));
    EIG_HIP(hipStreamSynchronize(stream));
  }
  return static_cast<T *>(p);
}
}  // namespace

struct TrsvHostRows {
  std::vector<i64> lrp;
  std::vector<i32> lc;
  std::vector<double> lv;
  std::vector<i64> ls, urp;
  std::vector<i32> uc;
  std::vector<double> uv;
  std::vector<i64> us;
};

namespace {
// Build the block-staged images (k_tsolve_staged) from the host rows kept at upload.
void build_staged(TrsvImage &img)
{
  const i64 n = img.n;
  const TrsvHostRows &H = *img.host;
  // block-staged images (k_tsolve_staged): per 64-row block, the outside-the-block entries of each
  // row as an ELL slab [k][r] in the row's own order, the inside entries as a dense tile [t][r]
  auto stage = [&](int f, const std::vector<i64> &rp, const std::vector<i32> &cj, const std::vector<double> &cv,
                   const std::vector<i64> &split) {
    // slab: the first kSlab entries of every row at a fixed place (block b: b * kSlab * 64), the
    // rest (rows wider than kSlab) in an overflow slab at off[b]
    const i64 nblocks = (n + kTB - 1) / kTB;
    std::vector<i64> off(nblocks + 1, 0);
    std::vector<i32> w(std::max<i64>(nblocks, 1), 0);
    const i64 fixed = nblocks * kSlab * kTB;
    for (i64 b = 0; b < nblocks; ++b)
    {
      i64 mw = 0;
      for (i64 i = b * kTB; i < std::min(n, b * kTB + kTB); ++i) mw = std::max(mw, split[i] - rp[i]);
      w[b] = (i32)mw;
      off[b + 1] = off[b] + std::max<i64>(mw - kSlab, 0) * kTB;
    }
    for (i64 b = 0; b <= nblocks; ++b) off[b] += fixed;
    std::vector<double> v1(std::max<i64>(off[nblocks], 1), 0.0);
    std::vector<i32> c1(std::max<i64>(off[nblocks], 1), -1);
    std::vector<double> tl((size_t)std::max<i64>(nblocks, 1) * kTB * kTB, 0.0);
    std::vector<unsigned long long> tm((size_t)std::max<i64>(nblocks, 1) * kTB, 0ull);
    for (i64 b = 0; b < nblocks; ++b)
      for (i64 i = b * kTB; i < std::min(n, b * kTB + kTB); ++i)
      {
        const i64 r = i - b * kTB;
        for (i64 q = rp[i]; q < split[i]; ++q)
        {
          const i64 k = q - rp[i];
          const i64 at = k < kSlab ? (b * kSlab + k) * kTB + r : off[b] + (k - kSlab) * kTB + r;
          v1[at] = cv[q];
          c1[at] = cj[q];
        }
        for (i64 q = split[i]; q < rp[i + 1]; ++q)
        {
          const i64 t = cj[q] - b * kTB;
          tl[(size_t)b * kTB * kTB + t * kTB + r] = cv[q];
          tm[(size_t)b * kTB + r] |= 1ull << t;
        }
      }
    off.resize(nblocks);
    img.off1[f] = upload(off, img.stream);
    img.w1[f] = upload(w, img.stream);
    img.v1[f] = upload(v1, img.stream);
    img.c1[f] = upload(c1, img.stream);
    img.tile[f] = upload(tl, img.stream);
    img.tmask[f] = upload(tm, img.stream);
  };
  stage(0, H.lrp, H.lc, H.lv, H.ls);
  stage(1, H.urp, H.uc, H.uv, H.us);
  img.staged_built = true;
  img.host.reset();
}
}  // namespace

namespace {
// f(b0, b1) over contiguous block ranges on up to 16 host threads
template <class F>
void parallel_blocks(i64 nb, F &&f)
{
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (nb < 32) nt = 1;
  if (nt == 1) return f(0, nb);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back([&, t] { f(nb * t / nt, nb * (t + 1) / nt); });
  for (auto &t : th) t.join();
}
}  // namespace

namespace {
// split points: L row i -> first entry inside i's 64-row block; U row i (descending columns) ->
// first entry with a column inside the block
void row_splits(i64 n, const std::vector<i64> &lrp, const std::vector<i32> &lc, const std::vector<i64> &urp,
                const std::vector<i32> &uc, std::vector<i64> &ls, std::vector<i64> &us)
{
  ls.resize(n);
  us.resize(n);
  for (i64 i = 0; i < n; ++i)
  {
    const i64 bs = i / kTB * kTB, be = std::min(bs + kTB, n);
    i64 k = lrp[i];
    while (k < lrp[i + 1] && lc[k] < bs) ++k;
    ls[i] = k;
    k = urp[i];
    while (k < urp[i + 1] && uc[k] >= be) ++k;
    us[i] = k;
  }
}

// Host arrays into ONE device allocation with ONE copy (a dozen separate small hipMalloc + hipMemcpy
// calls cost ~1 ms each); returns the allocation and the device address of every part.
void *upload_parts(const std::vector<std::pair<const void *, size_t>> &parts, std::vector<char *> &at,
                   hipStream_t stream)
{
  std::vector<size_t> off(parts.size());
  size_t total = 0;
  for (size_t k = 0; k < parts.size(); ++k)
  {
    off[k] = total;
    total += (std::max<size_t>(parts[k].second, 8) + 255) / 256 * 256;
  }
  std::vector<char> h(total, 0);
  for (size_t k = 0; k < parts.size(); ++k)
    if (parts[k].second) std::memcpy(h.data() + off[k], parts[k].first, parts[k].second);
  void *d = nullptr;
  const bool trace = std::getenv("EIGMI_TRACE_SETUP") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  EIG_HIP(hipMalloc(&d, total));
  auto t1 = std::chrono::steady_clock::now();
  EIG_HIP(hipMemcpyAsync(d, h.data(), total, hipMemcpyHostToDevice, stream));
  EIG_HIP(hipStreamSynchronize(stream));
  auto t2 = std::chrono::steady_clock::now();
  if (trace)
    fprintf(stderr, "upload_parts %zu B: malloc %.2f ms, memcpy %.2f ms\n", total,
            std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(t2 - t1).count());
  at.resize(parts.size());
  for (size_t k = 0; k < parts.size(); ++k) at[k] = static_cast<char *>(d) + off[k];
  return d;
}
}  // namespace

// The row-CSR factors the substitution kernels read (k_tsolve, and the U diagonal of the staged one).
void trsv_upload_rows(TrsvImage &img, const std::vector<i64> &lrp, const std::vector<i32> &lc,
                      const std::vector<double> &lv, const std::vector<i64> &urp, const std::vector<i32> &uc,
                      const std::vector<double> &uv, const std::vector<double> &ud)
{
  if (img.rows) return;
  std::vector<i64> ls, us;
  row_splits(img.n, lrp, lc, urp, uc, ls, us);
  std::vector<char *> at;
  img.arena_rows = upload_parts({{lrp.data(), lrp.size() * 8}, {ls.data(), ls.size() * 8}, {lc.data(), lc.size() * 4},
                                 {lv.data(), lv.size() * 8}, {urp.data(), urp.size() * 8}, {us.data(), us.size() * 8},
                                 {uc.data(), uc.size() * 4}, {uv.data(), uv.size() * 8}, {ud.data(), ud.size() * 8}},
                                at, img.stream);
  img.lrp = (i64 *)at[0];
  img.lsplit = (i64 *)at[1];
  img.lc = (i32 *)at[2];
  img.lv = (double *)at[3];
  img.urp = (i64 *)at[4];
  img.usplit = (i64 *)at[5];
  img.uc = (i32 *)at[6];
  img.uv = (double *)at[7];
  img.ud = (double *)at[8];
  img.rows = true;
}

void trsv_upload(eig_ctx_t ctx, i64 n, const std::vector<i64> &lrp, const std::vector<i32> &lc,
                 const std::vector<double> &lv, const std::vector<i64> &urp, const std::vector<i32> &uc,
                 const std::vector<double> &uv, const std::vector<double> &ud, const std::vector<i64> &P,
                 const std::vector<i64> &Q, const std::vector<double> &scale, TrsvImage &img)
{
  img.n = n;
  img.stream = ctx ? ctx->stream : nullptr;
  // EIGMI_TRACE_SETUP=1: phase times of the upload on stderr
  const bool trace = std::getenv("EIGMI_TRACE_SETUP") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto phase = [&](const char *what) {
    if (!trace) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "trsv_upload %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - t_last).count());
    t_last = now;
  };
  std::vector<i64> ls, us;
  row_splits(n, lrp, lc, urp, uc, ls, us);
  std::vector<i32> p32(n), q32(n);
  for (i64 k = 0; k < n; ++k)
  {
    p32[k] = (i32)P[k];
    q32[k] = (i32)Q[k];
  }
  // admission to the staged kernel: <= kSlab outside entries per row, all within kRing4 blocks
  auto fits = [&](const std::vector<i64> &rp, const std::vector<i32> &cj, const std::vector<i64> &split, bool lower) {
    for (i64 i = 0; i < n; ++i)
    {
      if (split[i] - rp[i] > kSlab) return false;
      const i64 blk = i / kTB;
      for (i64 q = rp[i]; q < split[i]; ++q)
      {
        const i64 cb = cj[q] / kTB;
        if (lower ? (cb < blk - kRing4) : (cb > blk + kRing4)) return false;
      }
    }
    return true;
  };
  phase("split");
  img.staged = fits(lrp, lc, ls, true) && fits(urp, uc, us, false);
  phase("staged");
  // block-inverse images (k_binv_z / k_binv_chain) for factors whose every coupling lies within
  // kBinvMaxGD blocks, when the tiles stay within kBinvTiles (a 64 x 64 tile per diagonal block and
  // per coupled block) and every diagonal block is well conditioned
  const i64 nblocks = (n + kTB - 1) / kTB;
  auto coupled = [&](const std::vector<i64> &rp, const std::vector<i32> &cj, const std::vector<i64> &split,
                     bool lower) {
    int dm = 0;
    for (i64 i = 0; i < n; ++i)
      for (i64 q = rp[i]; q < split[i]; ++q)
        dm = std::max<int>(dm, (int)(lower ? i / kTB - cj[q] / kTB : cj[q] / kTB - i / kTB));
    return dm;
  };
  // returns false (nothing uploaded) when a diagonal block fails the conditioning test
  auto binv_image = [&](int f, const std::vector<i64> &rp, const std::vector<i32> &cj, const std::vector<double> &cv,
                        const std::vector<i64> &split, const double *diag) -> bool {
    const bool lower = diag == nullptr;
    const int gd = img.gd[f];
    const size_t T2 = (size_t)kTB * kTB;
    std::vector<double> dinv((size_t)nblocks * T2, 0.0), gt((size_t)std::max<i64>(nblocks * gd, 1) * T2, 0.0);
    std::atomic<bool> ok{true};
    // blocks are independent: threads over contiguous block ranges
    parallel_blocks(nblocks, [&](i64 b0, i64 b1) {
    // Di holds inv(D_b) by columns (Di[j * 64 + i] = inv(D)[i][j]): each column is one triangular
    // solve with contiguous operands, and it is already the device layout of dinv ([t][r])
    std::vector<double> Db(T2), Di(T2), Tb(T2);
    for (i64 b = b0; b < b1 && ok.load(std::memory_order_relaxed); ++b)
    {
      const i64 bs = b * kTB, nbr = std::min<i64>(kTB, n - bs);
      // the diagonal block D[r][t] (rows past n: identity)
      std::fill(Db.begin(), Db.end(), 0.0);
      for (int r = 0; r < kTB; ++r) Db[r * kTB + r] = (r < nbr && !lower) ? diag[bs + r] : 1.0;
      for (i64 r = 0; r < nbr; ++r)
        for (i64 q = split[bs + r]; q < rp[bs + r + 1]; ++q) Db[r * kTB + (cj[q] - bs)] = cv[q];
      // its inverse, column j = the solution of D x = e_j (lower: top-down, upper: bottom-up)
      std::fill(Di.begin(), Di.end(), 0.0);
      for (int j = 0; j < kTB; ++j)
      {
        double *x = &Di[(size_t)j * kTB];
        if (lower)
          for (int i = j; i < kTB; ++i)
          {
            const double *Dr = &Db[(size_t)i * kTB];
            double v = i == j ? 1.0 : 0.0;
            for (int k = j; k < i; ++k) v -= Dr[k] * x[k];
            x[i] = v / Dr[i];
          }
        else
          for (int i = j; i >= 0; --i)
          {
            const double *Dr = &Db[(size_t)i * kTB];
            double v = i == j ? 1.0 : 0.0;
            for (int k = i + 1; k <= j; ++k) v -= Dr[k] * x[k];
            x[i] = v / Dr[i];
          }
      }
      {
        double dm = 0.0, im = 0.0;
        for (size_t q = 0; q < T2; ++q)
        {
          dm = std::max(dm, std::fabs(Db[q]));
          im = std::max(im, std::fabs(Di[q]));
        }
        if (!(dm * im * kTB <= kBinvCond)) ok = false;  // (NaN included)
      }
      std::copy(Di.begin(), Di.end(), dinv.begin() + (size_t)b * T2);
      // G(b, d) = inv(D_b) T(b, d), T(b, d)[r'][t] = the entry of row bs + r' in column t of block b -+ d
      for (int d = 1; d <= gd; ++d)
      {
        const i64 src = lower ? b - d : b + d;
        if (src < 0 || src >= nblocks) continue;
        std::fill(Tb.begin(), Tb.end(), 0.0);
        bool any = false;
        for (i64 r = 0; r < nbr; ++r)
          for (i64 q = rp[bs + r]; q < split[bs + r]; ++q)
            if (cj[q] / kTB == src)
            {
              Tb[r * kTB + (cj[q] - src * kTB)] += cv[q];
              any = true;
            }
        if (!any) continue;
        double *gb = &gt[((size_t)b * gd + (d - 1)) * T2];
        for (int rr = 0; rr < kTB; ++rr)  // G[:, t] += inv(D)[:, rr] T[rr][t] (column rr of inv(D):
        {                                 // rows rr.. (lower) / ..rr (upper) are its nonzeros)
          const double *dcol = &Di[(size_t)rr * kTB];
          const int r0 = lower ? rr : 0, r1 = lower ? kTB : rr + 1;
          for (int t = 0; t < kTB; ++t)
          {
            const double tv = Tb[rr * kTB + t];
            if (tv == 0.0) continue;
            double *gcol = gb + (size_t)t * kTB;
            for (int r = r0; r < r1; ++r) gcol[r] += dcol[r] * tv;
          }
        }
      }
    }
    });
    if (!ok) return false;
    img.dinv[f] = upload(dinv, img.stream);
    img.g[f] = upload(gt, img.stream);
    return true;
  };
  {
    img.gd[0] = coupled(lrp, lc, ls, true);
    img.gd[1] = coupled(urp, uc, us, false);
    const i64 tiles = nblocks * (2 + img.gd[0] + img.gd[1]);
    bool pivots = true;  // a zero U pivot leaves the reference's division to produce inf / nan
    for (i64 i = 0; i < n; ++i) pivots = pivots && ud[i] != 0.0;
    img.binv = pivots && tiles <= kBinvTiles && img.gd[0] <= kBinvMaxGD && img.gd[1] <= kBinvMaxGD;
    if (img.binv)
    {
      img.binv = binv_image(0, lrp, lc, lv, ls, nullptr) && binv_image(1, urp, uc, uv, us, ud.data());
      if (!img.binv)
        for (int f = 0; f < 2; ++f)
        {
          if (img.dinv[f]) (void)hipFree(img.dinv[f]);
          if (img.g[f]) (void)hipFree(img.g[f]);
          img.dinv[f] = img.g[f] = nullptr;
        }
    }
  }
  // host rows for a later build of the staged image: only when the staged kernel is the default
  // (no block-inverse image); with one, EIG_TRSV_STAGED takes the row-CSR kernel (bitwise too)
  if (img.staged && !img.binv)
    img.host = std::make_shared<TrsvHostRows>(TrsvHostRows{lrp, lc, lv, ls, urp, uc, uv, us});
  phase("binv");
  // permutations and scaling (every solve); the row-CSR factors only where a substitution kernel
  // is the default -- with the block-inverse image they are uploaded when eig_lu_set_solver asks
  // for EIG_TRSV_STAGED / _CSR (lu.cpp rebuilds them from the factors it keeps)
  {
    std::vector<char *> at;
    img.arena = upload_parts({{p32.data(), p32.size() * 4}, {q32.data(), q32.size() * 4},
                              {scale.data(), scale.size() * 8}}, at, img.stream);
    img.P = (i32 *)at[0];
    img.Q = (i32 *)at[1];
    img.scale = (double *)at[2];
  }
  if (!img.binv) trsv_upload_rows(img, lrp, lc, lv, urp, uc, uv, ud);
  phase("csr");
}

// The permutations and scaling every solve applies, for an image whose block-inverse tiles were
// built on the device (band_lu_device, k_band.hip).
void trsv_attach_perm(eig_ctx_t ctx, i64 n, const std::vector<i64> &P, const std::vector<i64> &Q,
                      const std::vector<double> &scale, TrsvImage &img)
{
  img.n = n;
  img.stream = ctx->stream;
  std::vector<i32> p32(n), q32(n);
  for (i64 k = 0; k < n; ++k)
  {
    p32[k] = (i32)P[k];
    q32[k] = (i32)Q[k];
  }
  std::vector<char *> at;
  img.arena = upload_parts({{p32.data(), p32.size() * 4}, {q32.data(), q32.size() * 4}, {scale.data(), scale.size() * 8}},
                           at, img.stream);
  img.P = (i32 *)at[0];
  img.Q = (i32 *)at[1];
  img.scale = (double *)at[2];
}

void trsv_free(TrsvImage &img)
{
  for (int f = 0; f < 2; ++f)
    for (void *p : {(void *)img.off1[f], (void *)img.w1[f], (void *)img.v1[f], (void *)img.c1[f], (void *)img.tile[f],
                    (void *)img.tmask[f], (void *)img.dinv[f], (void *)img.g[f]})
      if (p) (void)hipFree(p);
  if (img.arena) (void)hipFree(img.arena);
  if (img.arena_rows) (void)hipFree(img.arena_rows);  // (the row-CSR arrays live inside it)
  img = TrsvImage();
}

void launch_inverse_mv8(TrsvImage &img, i64 m, double *Qin, double *Qout, hipStream_t s)
{
  const i64 n = img.n;
  const int nblk = (int)(m / 8);
  // 1. Qout = P (R Qin)   2. Qin = L^-1 Qout   3. Qin = U^-1 Qin   4. Qout = Q Qin
  // (block-inverse: Qout = inv(D) P R Qin, Qin = L^-1 chain, Qout = inv(D_U) Qin, Qin = U^-1 chain)
  // img.solver (eig_lu_set_solver): EIG_TRSV_CSR = the row-CSR kernel, EIG_TRSV_STAGED = the
  // block-staged kernel (both bitwise the reference arithmetic); AUTO / BLOCKINV: the block-inverse
  // solve when the factor has its image
  const bool csr = img.solver == EIG_TRSV_CSR, staged = img.solver == EIG_TRSV_STAGED;
  if (img.binv && !csr && !staged)
  {
    const i64 nblocks = (n + kTB - 1) / kTB;
    hipLaunchKernelGGL(k_binv_z<true>, dim3((unsigned)nblocks, nblk), dim3(kThreadsT), 0, s, n, (const double *)img.dinv[0],
                       (const i32 *)img.P, (const double *)img.scale, (const double *)Qin, Qout);
    launch_binv_chain<true>(img.gd[0], nblk, n, img.g[0], Qout, Qin, s);
    hipLaunchKernelGGL(k_binv_z<false>, dim3((unsigned)nblocks, nblk), dim3(kThreadsT), 0, s, n,
                       (const double *)img.dinv[1], (const i32 *)nullptr, (const double *)nullptr, (const double *)Qin,
                       Qout);
    launch_binv_chain<false>(img.gd[1], nblk, n, img.g[1], Qout, Qin, s);
    hipLaunchKernelGGL(k_perm_out, dim3(grid256(n * nblk)), dim3(256), 0, s, n, nblk, img.Q, Qin, Qout);
    EIG_HIP(hipGetLastError());
    return;
  }
  EIG_CHECK(img.rows, EIG_ERR_ARG, "triangular solve: row factors not on the device (eig_lu_set_solver uploads them)");
  if (img.staged && !img.staged_built && !csr && img.host) build_staged(img);
  hipLaunchKernelGGL(k_perm_scale, dim3(grid256(n * nblk)), dim3(256), 0, s, n, nblk, img.P, img.scale, Qin, Qout);
  if (!img.staged_built || csr)
  {
    hipLaunchKernelGGL(k_tsolve<true>, dim3(nblk), dim3(kTThreads), 0, s, n, img.lrp, img.lsplit, img.lc, img.lv,
                       (const double *)nullptr, (const double *)Qout, Qin);
    hipLaunchKernelGGL(k_tsolve<false>, dim3(nblk), dim3(kTThreads), 0, s, n, img.urp, img.usplit, img.uc, img.uv,
                       (const double *)img.ud, (const double *)Qin, Qin);
  }
  else
  {
    const Staged L{img.off1[0], img.w1[0], img.v1[0], img.c1[0], img.tile[0], img.tmask[0]};
    const Staged U{img.off1[1], img.w1[1], img.v1[1], img.c1[1], img.tile[1], img.tmask[1]};
    hipLaunchKernelGGL(k_tsolve_staged<true>, dim3(nblk), dim3(kTThreads), 0, s, n, L, (const double *)nullptr,
                       (const double *)Qout, Qin);
    hipLaunchKernelGGL(k_tsolve_staged<false>, dim3(nblk), dim3(kTThreads), 0, s, n, U, (const double *)img.ud,
                       (const double *)Qin, Qin);
  }
  hipLaunchKernelGGL(k_perm_out, dim3(grid256(n * nblk)), dim3(256), 0, s, n, nblk, img.Q, Qin, Qout);
  EIG_HIP(hipGetLastError());
}

}  // namespace eigmi
