// k_band.hip -- the factorisation of eig_lu_create_bcsr on the device (the
// factors matmul_inverse_tallskinny_blocked applies, kernels_cpp.hh:660-755).
//
// The matrix B = (R^-1 A)[perm, perm] (row-sum scaling, reverse Cuthill-McKee order: lu.cpp) is
// factored B = L U without pivoting -- the host envelope LU's arithmetic contract -- as a BAND of
// 64 x 64 tiles: block row b keeps the tiles of block columns b - gd .. b + gd, gd = the envelope's
// reach in blocks.  Fill of an LU without pivoting stays inside the envelope, so the band's entries
// outside it stay exact zeros and the factors downloaded for export have the host factor's pattern.
// Block step b (right-looking):
//   k_band_panel   2 gd workgroups, each eliminates the diagonal tile together with ONE coupled tile:
//                  "tall" [D; A(b+i, b)] -> L_bb, U_bb and L(b+i, b) = A(b+i, b) U_bb^-1, or "wide"
//                  [D, A(b, b+j)] -> U(b, b+j) = L_bb^-1 A(b, b+j).  Every workgroup repeats the same
//                  operations on D in the same order (identical results), so none waits for another.
//   k_band_update  gd^2 workgroups: A(b+i, b+j) -= L(b+i, b) U(b, b+j).
// Then the block-inverse image of k_binv_z / k_binv_chain (k_trsv.hip) straight from the tiles:
//   k_band_tinv    inv(L_bb) (unit lower) and inv(U_bb) per block, with the conditioning estimate
//                  max|D_b| max|inv(D_b)| 64 the host image builder applies (kBinvCond);
//   k_band_g       G(b, d) = inv(D_b) T(b, d), T = the coupled tiles L(b, b-d) / U(b, b+d).
// Tiles are column-major ([c][r], element (r, c) at c * 64 + r), the layout of the image's dinv
// and G tiles.  The host envelope LU plus the host image builder were ~70 % of a 200^2 setup
// (n bw^2 multiply-adds each, on host cores); here they are ~2 nb + 2 short launches.
#include "internal.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace eigmi {

namespace {
constexpr int kB = 64;
constexpr int kB2 = kB * kB;
constexpr int kPanelThreads = 128;

__device__ __forceinline__ i64 tile_at(i64 b, int d, int gd) { return (b * (2 * gd + 1) + d + gd) * kB2; }

// band (zeroed) <- the entries of B; row i of A is row inv[i] of B
__global__ __launch_bounds__(256) void k_band_scatter(i64 n, const i64 *__restrict__ rp, const i32 *__restrict__ cj,
                                                      const double *__restrict__ cv, const i32 *__restrict__ inv,
                                                      const double *__restrict__ rs, int gd, double *__restrict__ band)
{
  const i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const i64 k = inv[i];
  const double r = rs[i];
  for (i64 q = rp[i]; q < rp[i + 1]; ++q)
  {
    const i64 j = inv[cj[q]];
    band[tile_at(k >> 6, (int)((j >> 6) - (k >> 6)), gd) + (j & 63) * kB + (k & 63)] = cv[q] / r;
  }
}

// rows past n in the last block: a unit diagonal (the host image builder's identity padding)
__global__ __launch_bounds__(64) void k_band_pad(i64 n, int gd, double *band)
{
  const i64 k = (n & ~(i64)63) + threadIdx.x;
  if (k >= n && (n & 63)) band[tile_at(k >> 6, 0, gd) + (k & 63) * kB + (k & 63)] = 1.0;
}

// One block step's panels.  Workgroup w < G (G = max(gd, 1)): tall panel [D; A(b+1+w, b)];
// w >= G: wide panel [D, A(b, b+1+w-G)].  Threads 0..63 hold row t of D in registers, threads
// 64..127 row t-64 of the tall tile or column t-64 of the wide tile.  Elimination step k (unrolled:
// every register index is static): the rows below k take the multiplier l = v[k] (1 / p(k)) against
// the pivot row p published in LDS, store it in v[k] and subtract l p from their columns > k; the
// wide tile's columns apply the previous step's multipliers (x_i -= l_i x_(k-1), i >= k: the
// forward substitution with L_bb, one step behind); the row that becomes the next pivot publishes
// itself.  One barrier per step (pivot rows and multipliers double-buffered by step parity).  D
// itself is only read (other workgroups of the launch may still be loading it): workgroup 0 stores
// the factored diagonal tile to dfac (copied into the band after the last step) and reports a zero
// or non-finite pivot in *bad.
__global__ __launch_bounds__(kPanelThreads) void k_band_panel(i64 b, i64 nb, int gd, double *band, double *dfac,
                                                              int *bad)
{
  __shared__ double prow[2][kB];
  __shared__ double lcol[2][kB];
  __shared__ double prcp[2];  // 1 / pivot
  const int G = gd > 0 ? gd : 1;
  const int w = blockIdx.x, t = threadIdx.x;
  const bool tall = w < G;
  const int off = tall ? w + 1 : w - G + 1;  // coupled block distance
  const bool has = off <= gd && b + off < nb;
  if (!has && w != 0) return;
  const double *D = band + tile_at(b, 0, gd);
  double *X = has ? band + (tall ? tile_at(b + off, -off, gd) : tile_at(b, off, gd)) : nullptr;
  const int q = t & 63;
  const bool drow = t < kB, active = drow || has, xcol = active && !tall && !drow, xrow = active && !drow && tall;
  double v[kB];
#pragma unroll
  for (int c = 0; c < kB; ++c) v[c] = 0.0;
  if (drow)
  {
#pragma unroll
    for (int c = 0; c < kB; ++c) v[c] = D[c * kB + q];
  }
  else if (xrow)
  {
#pragma unroll
    for (int c = 0; c < kB; ++c) v[c] = X[c * kB + q];
  }
  else if (xcol)
  {
#pragma unroll
    for (int i = 0; i < kB; ++i) v[i] = X[q * kB + i];
  }
  if (t == 0)
  {
#pragma unroll
    for (int c = 0; c < kB; ++c) prow[0][c] = v[c];
    prcp[0] = 1.0 / v[0];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kB; ++k)
  {
    const double *pr = prow[k & 1];
    if ((drow && q > k) || xrow)
    {
      const double l = v[k] * prcp[k & 1];
      v[k] = l;
#pragma unroll
      for (int c = k + 1; c < kB; ++c) v[c] = fma(-l, pr[c], v[c]);
      if (drow)
      {
        lcol[k & 1][q] = l;
        if (q == k + 1)
        {
#pragma unroll
          for (int c = k + 1; c < kB; ++c) prow[(k + 1) & 1][c] = v[c];
          prcp[(k + 1) & 1] = 1.0 / v[k + 1];
        }
      }
    }
    if (xcol && k > 0)
    {
      const double *lc = lcol[(k - 1) & 1];
      const double xk = v[k - 1];
#pragma unroll
      for (int i = k; i < kB; ++i) v[i] = fma(-lc[i], xk, v[i]);
    }
    if (w == 0 && t == 0)
    {
      const double p = fabs(pr[k]);
      if (!(p > 0.0 && p <= 1.7976931348623157e308)) bad[0] = 1;
    }
    __syncthreads();
  }
  if (w == 0 && drow)
  {
    double *Dw = dfac + b * kB2;
#pragma unroll
    for (int c = 0; c < kB; ++c) Dw[c * kB + q] = v[c];
  }
  if (xrow)
  {
#pragma unroll
    for (int c = 0; c < kB; ++c) X[c * kB + q] = v[c];
  }
  if (xcol)
  {
#pragma unroll
    for (int i = 0; i < kB; ++i) X[q * kB + i] = v[i];
  }
}

// the factored diagonal tiles into the band
__global__ __launch_bounds__(256) void k_band_diag_copy(int gd, const double *__restrict__ dfac, double *band)
{
  const i64 b = blockIdx.x;
  for (int e = threadIdx.x; e < kB2; e += 256) band[tile_at(b, 0, gd) + e] = dfac[b * kB2 + e];
}

// C (+)= sign * A B for 64 x 64 column-major tiles, 256 threads, thread t: rows 4 (t & 15) .., columns
// 4 (t >> 4) ..; A staged as [k][r], B transposed into [k][c] so both operands are contiguous reads.
__device__ __forceinline__ void tile_mm(const double *__restrict__ A, const double *__restrict__ Bm, double *C,
                                        double sign, bool accumulate, double *As, double *Bs)
{
  const int t = threadIdx.x;
  for (int e = t; e < kB2; e += 256)
  {
    As[e] = A[e];                                        // (r, k) -> As[k * 64 + r]
    const int c = e >> 6, k = e & 63;                    // Bm element (k, c) at c * 64 + k
    Bs[k * 65 + c] = Bm[e];
  }
  __syncthreads();
  const int r0 = (t & 15) * 4, c0 = (t >> 4) * 4;
  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
  for (int k = 0; k < kB; ++k)
  {
    double a[4], bb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = As[k * kB + r0 + i];
#pragma unroll
    for (int j = 0; j < 4; ++j) bb[j] = Bs[k * 65 + c0 + j];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = fma(a[i], bb[j], acc[i][j]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
    {
      const i64 at = (i64)(c0 + j) * kB + r0 + i;
      C[at] = accumulate ? C[at] + sign * acc[i][j] : sign * acc[i][j];
    }
}

// trailing update of block step b: A(b+i, b+j) -= L(b+i, b) U(b, b+j), i, j = 1 .. gd
__global__ __launch_bounds__(256) void k_band_update(i64 b, i64 nb, int gd, double *band)
{
  __shared__ double As[kB2];
  __shared__ double Bs[kB * 65];
  const int i = blockIdx.x / gd + 1, j = blockIdx.x % gd + 1;
  if (b + i >= nb || b + j >= nb) return;
  tile_mm(band + tile_at(b + i, -i, gd), band + tile_at(b, j, gd), band + tile_at(b + i, j - i, gd), -1.0, true, As,
          Bs);
}

// inv(L_bb) (blockIdx.y 0, unit lower) / inv(U_bb) (1) column by column: lane j owns column j of X
// (LDS), X = I, then L: X(i, j) -= L(i, k) X(k, j) for k ascending, i > k; U: X(k, j) /= U(k, k),
// X(i, j) -= U(i, k) X(k, j) for k descending, i < k.  flag[2 b + f] = 1 when max|D| max|X| 64 >
// kCond (or NaN): that factor keeps the substitution kernels (lu.cpp).
__global__ __launch_bounds__(64) void k_band_tinv(int gd, const double *__restrict__ band, double *dinv_l,
                                                  double *dinv_u, int *flag, double cond)
{
  __shared__ double Dt[kB * 65];  // D(i, k) at k * 65 + i
  __shared__ double X[kB * 65];   // X(i, j) at i * 65 + j
  const int j = threadIdx.x, f = blockIdx.y;
  const i64 b = blockIdx.x;
  const double *D = band + tile_at(b, 0, gd);
  double dm = 0.0;
  for (int k = 0; k < kB; ++k)
  {
    double v = D[k * kB + j];  // D(j, k)
    if (f == 0) v = (j > k) ? v : (j == k ? 1.0 : 0.0);
    else v = (j <= k) ? v : 0.0;
    Dt[k * 65 + j] = v;
    dm = fmax(dm, fabs(v));
  }
  for (int i = 0; i < kB; ++i) X[i * 65 + j] = (i == j) ? 1.0 : 0.0;
  __syncthreads();
  if (f == 0)
    for (int k = 0; k < kB; ++k)
    {
      const double xk = X[k * 65 + j];
      for (int i = k + 1; i < kB; ++i) X[i * 65 + j] -= Dt[k * 65 + i] * xk;
    }
  else
    for (int k = kB - 1; k >= 0; --k)
    {
      const double xk = X[k * 65 + j] / Dt[k * 65 + k];
      X[k * 65 + j] = xk;
      for (int i = 0; i < k; ++i) X[i * 65 + j] -= Dt[k * 65 + i] * xk;
    }
  double im = 0.0;
  for (int i = 0; i < kB; ++i) im = fmax(im, fabs(X[i * 65 + j]));
  __syncthreads();
  double *out = (f == 0 ? dinv_l : dinv_u) + b * kB2;
  for (int c = 0; c < kB; ++c) out[c * kB + j] = X[j * 65 + c];  // (row j, column c): coalesced in j
  // wave maxima (one wave)
  for (int o = 32; o > 0; o >>= 1)
  {
    dm = fmax(dm, __shfl_xor(dm, o));
    im = fmax(im, __shfl_xor(im, o));
  }
  if (j == 0) flag[2 * b + f] = (dm * im * kB <= cond) ? 0 : 1;
}

// G(b, d) = inv(D_b) T(b, d): blockIdx = (b, d - 1, f), T = tile (b, -d) of L (f 0) / (b, +d) of U
__global__ __launch_bounds__(256) void k_band_g(int gd, const double *__restrict__ band, const double *dinv_l,
                                                const double *dinv_u, double *g_l, double *g_u)
{
  __shared__ double As[kB2];
  __shared__ double Bs[kB * 65];
  const i64 b = blockIdx.x;
  const int d = blockIdx.y + 1, f = blockIdx.z;
  const double *Di = (f == 0 ? dinv_l : dinv_u) + b * kB2;
  const double *T = band + tile_at(b, f == 0 ? -d : d, gd);
  double *G = (f == 0 ? g_l : g_u) + (b * gd + d - 1) * kB2;
  tile_mm(Di, T, G, 1.0, false, As, Bs);
}

}  // namespace

// Factor B on the device and build the block-inverse image into img (dinv / g / gd / binv); the
// band stays allocated in *band_out (the exported factors are read from it on demand).  Returns
// false when a diagonal tile fails the conditioning test (the caller then takes the host image
// path); throws EIG_ERR_BREAKDOWN on a zero pivot like the host LU.
bool band_lu_device(eig_ctx_t ctx, i64 n, int gd, const std::vector<i64> &rp, const std::vector<i32> &cj,
                    const std::vector<double> &cv, const std::vector<i32> &inv, const std::vector<double> &rs,
                    TrsvImage &img, double **band_out)
{
  hipStream_t s = ctx->stream;
  const bool trace = std::getenv("EIGMI_TRACE_SETUP") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto phase = [&](const char *what) {
    if (!trace) return;
    EIG_HIP(hipStreamSynchronize(s));
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "band_lu    %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - t_last).count());
    t_last = now;
  };
  const i64 nb = (n + kB - 1) / kB;
  const i64 band_tiles = nb * (2 * gd + 1);
  // inputs: one allocation, one copy
  const size_t o_rp = 0, o_cj = o_rp + (size_t)(n + 1) * 8, o_cv = o_cj + (cj.size() * 4 + 7) / 8 * 8,
               o_inv = o_cv + cv.size() * 8, o_rs = o_inv + ((size_t)n * 4 + 7) / 8 * 8, o_end = o_rs + (size_t)n * 8;
  std::vector<char> h(o_end);
  std::memcpy(h.data() + o_rp, rp.data(), (size_t)(n + 1) * 8);
  std::memcpy(h.data() + o_cj, cj.data(), cj.size() * 4);
  std::memcpy(h.data() + o_cv, cv.data(), cv.size() * 8);
  std::memcpy(h.data() + o_inv, inv.data(), (size_t)n * 4);
  std::memcpy(h.data() + o_rs, rs.data(), (size_t)n * 8);
  DevBuf in(o_end);
  EIG_HIP(hipMemcpyAsync(in.d(), h.data(), o_end, hipMemcpyHostToDevice, s));
  char *ib = reinterpret_cast<char *>(in.d());
  double *band = nullptr, *dl = nullptr, *du = nullptr, *gl = nullptr, *gu = nullptr;
  int *flags = nullptr;
  EIG_HIP(hipMalloc(&band, (size_t)band_tiles * kB2 * 8));
  EIG_HIP(hipMemsetAsync(band, 0, (size_t)band_tiles * kB2 * 8, s));
  const int gdi = gd > 0 ? gd : 1;  // (the image keeps one placeholder G tile per block at gd = 0)
  EIG_HIP(hipMalloc(&dl, (size_t)nb * kB2 * 8));
  EIG_HIP(hipMalloc(&du, (size_t)nb * kB2 * 8));
  EIG_HIP(hipMalloc(&gl, (size_t)nb * gdi * kB2 * 8));
  EIG_HIP(hipMalloc(&gu, (size_t)nb * gdi * kB2 * 8));
  EIG_HIP(hipMalloc(&flags, (size_t)(2 * nb + 1) * sizeof(int)));
  EIG_HIP(hipMemsetAsync(gl, 0, (size_t)nb * gdi * kB2 * 8, s));
  EIG_HIP(hipMemsetAsync(gu, 0, (size_t)nb * gdi * kB2 * 8, s));
  EIG_HIP(hipMemsetAsync(flags, 0, (size_t)(2 * nb + 1) * sizeof(int), s));
  auto release = [&] {
    for (void *p : {(void *)band, (void *)dl, (void *)du, (void *)gl, (void *)gu, (void *)flags})
      if (p) (void)hipFree(p);
  };
  try
  {
    hipLaunchKernelGGL(k_band_scatter, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n,
                       (const i64 *)(ib + o_rp), (const i32 *)(ib + o_cj), (const double *)(ib + o_cv),
                       (const i32 *)(ib + o_inv), (const double *)(ib + o_rs), gd, band);
    hipLaunchKernelGGL(k_band_pad, dim3(1), dim3(64), 0, s, n, gd, band);
    EIG_HIP(hipGetLastError());
    phase("scatter");
    int *bad = flags + 2 * nb;
    {
      DevBuf dfac((size_t)nb * kB2 * 8);
      for (i64 b = 0; b < nb; ++b)
      {
        hipLaunchKernelGGL(k_band_panel, dim3(2 * gdi), dim3(kPanelThreads), 0, s, b, nb, gd, band, dfac.d(), bad);
        if (gd > 0 && b + 1 < nb) hipLaunchKernelGGL(k_band_update, dim3(gd * gd), dim3(256), 0, s, b, nb, gd, band);
      }
      hipLaunchKernelGGL(k_band_diag_copy, dim3((unsigned)nb), dim3(256), 0, s, gd, (const double *)dfac.d(), band);
      EIG_HIP(hipGetLastError());
      EIG_HIP(hipStreamSynchronize(s));  // (dfac)
    }
    phase("factor");
    hipLaunchKernelGGL(k_band_tinv, dim3((unsigned)nb, 2), dim3(64), 0, s, gd, (const double *)band, dl, du, flags,
                       1e6);
    if (gd > 0)
      hipLaunchKernelGGL(k_band_g, dim3((unsigned)nb, gd, 2), dim3(256), 0, s, gd, (const double *)band,
                         (const double *)dl, (const double *)du, gl, gu);
    EIG_HIP(hipGetLastError());
    std::vector<int> fl(2 * nb + 1);
    EIG_HIP(hipMemcpyAsync(fl.data(), flags, fl.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    EIG_HIP(hipStreamSynchronize(s));
    phase("image");
    EIG_CHECK(fl[2 * nb] == 0, EIG_ERR_BREAKDOWN, "LU: zero pivot (matrix needs pivoting)");
    bool ok = true;
    for (i64 q = 0; q < 2 * nb; ++q) ok = ok && fl[q] == 0;
    (void)hipFree(flags);
    flags = nullptr;
    *band_out = band;
    band = nullptr;
    if (!ok)
    {
      release();
      return false;
    }
    img.dinv[0] = dl;
    img.dinv[1] = du;
    img.g[0] = gl;
    img.g[1] = gu;
    img.gd[0] = img.gd[1] = gd;
    img.binv = true;
    return true;
  }
  catch (...)
  {
    release();
    throw;
  }
}

}  // namespace eigmi
