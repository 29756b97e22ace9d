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
#include "internal.h"

namespace eigmi {

namespace {
constexpr int kTB = 64;       // rows per block
constexpr int kTThreads = 512;  // 8 waves = the 8 columns of a column block
constexpr int kRing = 3;        // solved blocks whose x stays in LDS for phase 1

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

int grid256(i64 work)
{
  i64 g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

template <class T>
T *upload(const std::vector<T> &h)
{
  void *p = nullptr;
  EIG_HIP(hipMalloc(&p, std::max<size_t>(h.size(), 1) * sizeof(T)));
  if (!h.empty()) EIG_HIP(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return static_cast<T *>(p);
}
}  // namespace

void trsv_upload(eig_ctx_t ctx, i64 n, const std::vector<i64> &lrp, const std::vector<i32> &lc,
                 const std::vector<double> &lv, const std::vector<i64> &urp, const std::vector<i32> &uc,
                 const std::vector<double> &uv, const std::vector<double> &ud, const std::vector<i64> &P,
                 const std::vector<i64> &Q, const std::vector<double> &scale, TrsvImage &img)
{
  (void)ctx;
  img.n = n;
  // split points: L row i -> first entry inside i's 64-row block; U row i (descending columns) ->
  // first entry with a column inside the block
  std::vector<i64> ls(n), us(n);
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
  std::vector<i32> p32(n), q32(n);
  for (i64 k = 0; k < n; ++k)
  {
    p32[k] = (i32)P[k];
    q32[k] = (i32)Q[k];
  }
  img.lrp = upload(lrp);
  img.lsplit = upload(ls);
  img.lc = upload(lc);
  img.lv = upload(lv);
  img.urp = upload(urp);
  img.usplit = upload(us);
  img.uc = upload(uc);
  img.uv = upload(uv);
  img.ud = upload(ud);
  img.P = upload(p32);
  img.Q = upload(q32);
  img.scale = upload(scale);
}

void trsv_free(TrsvImage &img)
{
  for (void *p : {(void *)img.lrp, (void *)img.lsplit, (void *)img.lc, (void *)img.lv, (void *)img.urp,
                  (void *)img.usplit, (void *)img.uc, (void *)img.uv, (void *)img.ud, (void *)img.P, (void *)img.Q,
                  (void *)img.scale})
    if (p) (void)hipFree(p);
  img = TrsvImage();
}

void launch_inverse_mv8(const TrsvImage &img, i64 m, double *Qin, double *Qout, hipStream_t s)
{
  const i64 n = img.n;
  const int nblk = (int)(m / 8);
  // 1. Qout = P (R Qin)   2. Qin = L^-1 Qout   3. Qin = U^-1 Qin   4. Qout = Q Qin
  hipLaunchKernelGGL(k_perm_scale, dim3(grid256(n * nblk)), dim3(256), 0, s, n, nblk, img.P, img.scale, Qin, Qout);
  hipLaunchKernelGGL(k_tsolve<true>, dim3(nblk), dim3(kTThreads), 0, s, n, img.lrp, img.lsplit, img.lc, img.lv,
                     (const double *)nullptr, (const double *)Qout, Qin);
  hipLaunchKernelGGL(k_tsolve<false>, dim3(nblk), dim3(kTThreads), 0, s, n, img.urp, img.usplit, img.uc, img.uv,
                     (const double *)img.ud, (const double *)Qin, Qin);
  hipLaunchKernelGGL(k_perm_out, dim3(grid256(n * nblk)), dim3(256), 0, s, n, nblk, img.Q, Qin, Qout);
  EIG_HIP(hipGetLastError());
}

}  // namespace eigmi
