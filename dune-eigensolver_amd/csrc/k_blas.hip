// k_blas.hip -- BlockVector-level kernels (dot / axpy / norm), the fused Lanczos update and
// the column-major GEMV pair used by the Lanczos re-orthogonalisation (gfx950).
//
// All streaming kernels read 16 B per lane (double2) where alignment allows and grid-stride
// over 2048 workgroups; every reduction is the deterministic grid_sum of reduce_dev.h.
#include "internal.h"
#include "reduce_dev.h"

namespace eigmi {

static inline int stream_grid(i64 n, int per_thread = 2)
{
  const i64 need = (n + (i64)kStreamThreads * per_thread - 1) / ((i64)kStreamThreads * per_thread);
  if (need < 1) return 1;
  return (int)(need < kStreamBlocks ? need : kStreamBlocks);
}

// ---------------------------------------------------------------------------------------------
// Lanczos step, kernel 2 (DESIGN.md "Lanczos step"):
//   alpha_j = sig_j * dsum[j];  u_{j+1} = t - (alpha_j sig_j) u_j;  nsum[j+1] = ||u_{j+1}||^2
// t is updated in place (it becomes u_{j+1}).  Same rounding sequence as orc_lanczos.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kStreamThreads) void k_lanczos_update(i64 n, const double *__restrict__ u,
                                                                   double *__restrict__ t, int j,
                                                                   const double *__restrict__ dsum,
                                                                   const double *__restrict__ nsum,
                                                                   double *__restrict__ alpha_out,
                                                                   double *__restrict__ nsum_out, double *partials,
                                                                   unsigned *ticket)
{
  __shared__ double tot[1];
  const double sig = 1.0 / sqrt(nsum[j]);
  const double alpha = sig * dsum[j];
  const double as = alpha * sig;
  double acc = 0.0;
  const i64 n2 = n >> 1;
  const double2 *u2 = reinterpret_cast<const double2 *>(u);
  double2 *t2 = reinterpret_cast<double2 *>(t);
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n2; i += (i64)gridDim.x * kStreamThreads)
  {
    double2 tv = t2[i], uv = u2[i];
    double2 r;
    r.x = tv.x - as * uv.x;
    r.y = tv.y - as * uv.y;
    t2[i] = r;
    acc += r.x * r.x;
    acc += r.y * r.y;
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0)
  {
    double r = t[n - 1] - as * u[n - 1];
    t[n - 1] = r;
    acc += r * r;
  }
  double v[1] = {acc};
  if (grid_sum<1, kStreamThreads>(v, partials, ticket, tot))
  {
    if (threadIdx.x == 0)
    {
      nsum_out[0] = tot[0];
      if (alpha_out) alpha_out[0] = alpha;
    }
  }
}

void launch_lanczos_update(i64 n, const double *u, double *t, int j, const LanczosState &st, int ticket,
                           hipStream_t s, ReduceWS red)
{
  EIG_CHECK((((uintptr_t)u | (uintptr_t)t) & 15) == 0, EIG_ERR_ARG, "lanczos update: vectors must be 16-B aligned");
  hipLaunchKernelGGL(k_lanczos_update, dim3(stream_grid(n)), dim3(kStreamThreads), 0, s, n, u, t, j, st.dsum,
                     st.nsum, st.alpha + j, st.nsum + j + 1, red.partials, red.ticket(ticket));
}

// beta[j] = sqrt(nsum[j]) (records the final beta of a run).
__global__ void k_beta_tail(const double *nsum, double *beta, int j)
{
  if (threadIdx.x == 0 && blockIdx.x == 0) beta[j] = sqrt(nsum[j]);
}
void launch_beta_tail(const LanczosState &st, int j, hipStream_t s)
{
  hipLaunchKernelGGL(k_beta_tail, dim3(1), dim3(64), 0, s, st.nsum, st.beta, j);
}

// ---------------------------------------------------------------------------------------------
// BlockVector ops.  Dots sum per lane in index order, then the fixed grid tree.
// ---------------------------------------------------------------------------------------------
template <bool SQ>
__global__ __launch_bounds__(kStreamThreads) void k_dot(i64 n, const double *__restrict__ x,
                                                        const double *__restrict__ y, double *out, double *partials,
                                                        unsigned *ticket)
{
  __shared__ double tot[1];
  double acc = 0.0;
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
  {
    const double a = x[i];
    acc += a * (SQ ? a : y[i]);
  }
  double v[1] = {acc};
  if (grid_sum<1, kStreamThreads>(v, partials, ticket, tot))
    if (threadIdx.x == 0) out[0] = tot[0];
}

void launch_dot(i64 n, const double *x, const double *y, double *out, int ticket, hipStream_t s, ReduceWS red)
{
  hipLaunchKernelGGL(k_dot<false>, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, x, y, out, red.partials,
                     red.ticket(ticket));
}
void launch_nrm2sq(i64 n, const double *x, double *out, int ticket, hipStream_t s, ReduceWS red)
{
  hipLaunchKernelGGL(k_dot<true>, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, x, x, out, red.partials,
                     red.ticket(ticket));
}

// The external driver's Lanczos update in one pass (eig_lanczos_update; what ARPACK's dsaitr does
// with the vector multMv returned, arpack_geneo_wrapper.hh:257-279):
//   w_i <- (w_i - alpha v_i) - beta p_i;   out[0] = sum w_i^2,  out[1] = sum v_i w_i  (new w)
// alpha / beta from device memory (beta / p absent: no third term).  Per lane in index order, then
// the fixed grid tree of reduce_dev.h: deterministic.
__global__ __launch_bounds__(kStreamThreads) void k_lanczos_update_ext(i64 n, const double *__restrict__ alpha,
                                                                       const double *__restrict__ beta,
                                                                       const double *__restrict__ v,
                                                                       const double *__restrict__ p,
                                                                       double *__restrict__ w, double *out,
                                                                       double *partials, unsigned *ticket)
{
  __shared__ double tot[2];
  const double a = alpha[0], b = p ? beta[0] : 0.0;
  double s0 = 0.0, s1 = 0.0;
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
  {
    const double vi = v[i];
    double r = w[i] - a * vi;
    if (p) r -= b * p[i];
    w[i] = r;
    s0 += r * r;
    s1 += vi * r;
  }
  double t[2] = {s0, s1};
  if (grid_sum<2, kStreamThreads>(t, partials, ticket, tot))
    if (threadIdx.x < 2) out[threadIdx.x] = tot[threadIdx.x];
}

void launch_lanczos_update_ext(i64 n, const double *alpha, const double *beta, const double *v, const double *p,
                               double *w, double *out, int ticket, hipStream_t s, ReduceWS red)
{
  hipLaunchKernelGGL(k_lanczos_update_ext, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, alpha, beta, v, p,
                     w, out, red.partials, red.ticket(ticket));
}

// y += a x   (a from the host, or a = scale * (*a_dev) from device memory)
__global__ __launch_bounds__(kStreamThreads) void k_axpy(i64 n, double a, const double *a_dev, double scale,
                                                         const double *__restrict__ x, double *__restrict__ y)
{
  if (a_dev) a = scale * a_dev[0];
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
    y[i] += a * x[i];
}
void launch_axpy(i64 n, double a, const double *x, double *y, hipStream_t s)
{
  hipLaunchKernelGGL(k_axpy, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, a, (const double *)nullptr, 1.0,
                     x, y);
}
void launch_axpy_dev(i64 n, const double *a, double scale, const double *x, double *y, hipStream_t s)
{
  hipLaunchKernelGGL(k_axpy, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, 0.0, a, scale, x, y);
}

// x[i] = standard normal numbers from a counter-based generator (splitmix64 of (seed, i), Box-Muller):
// start blocks of the block Krylov drivers, generated where they are used
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z)
{
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(kStreamThreads) void k_fill_normal(i64 n, unsigned long long seed, double *__restrict__ x)
{
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
  {
    const unsigned long long a = splitmix64(seed ^ splitmix64(2 * (unsigned long long)i));
    const unsigned long long b = splitmix64(seed ^ splitmix64(2 * (unsigned long long)i + 1));
    const double u1 = ((double)(a >> 11) + 0.5) * 0x1.0p-53, u2 = (double)(b >> 11) * 0x1.0p-53;
    x[i] = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  }
}
void launch_fill_normal(i64 n, unsigned seed, double *x, hipStream_t s)
{
  hipLaunchKernelGGL(k_fill_normal, dim3(stream_grid(n, 1)), dim3(kStreamThreads), 0, s, n,
                     0x5eedull * 0x100000001ull + (unsigned long long)seed, x);
}

// x *= a ; or x *= 1/sqrt(*a_dev) (normalise by a device-resident squared norm)
__global__ __launch_bounds__(kStreamThreads) void k_scal(i64 n, double a, const double *a_dev, int rsqrt_mode,
                                                         double *__restrict__ x)
{
  if (a_dev) a = rsqrt_mode ? 1.0 / sqrt(a_dev[0]) : a_dev[0];
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
    x[i] *= a;
}
void launch_scal(i64 n, double a, double *x, hipStream_t s)
{
  hipLaunchKernelGGL(k_scal, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, a, (const double *)nullptr, 0,
                     x);
}
void launch_scal_dev(i64 n, const double *a, bool reciprocal_sqrt, double *x, hipStream_t s)
{
  hipLaunchKernelGGL(k_scal, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, 0.0, a, reciprocal_sqrt ? 1 : 0,
                     x);
}

__global__ void k_sqrt_inplace(double *v, int count)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) v[i] = sqrt(v[i]);
}
void launch_sqrt_inplace(double *v, int count, hipStream_t s)
{
  hipLaunchKernelGGL(k_sqrt_inplace, dim3((count + 63) / 64), dim3(64), 0, s, v, count);
}

// ---------------------------------------------------------------------------------------------
// a13: A += shift * I on the SELL image (eigensolver.hh:59-66).  The diagonal block of block
// row r has window-local block column r + own_offset / bc.
// ---------------------------------------------------------------------------------------------
__global__ void k_shift_diag(i64 nbrows, i64 own_blk, const i64 *__restrict__ slice_ptr, const i32 *__restrict__ col,
                             double *__restrict__ val, int br, int bc, int C, double shift)
{
  const i64 r = (i64)blockIdx.x * blockDim.x + threadIdx.x;  // block row
  if (r >= nbrows) return;
  const i64 s = r / C, l = r % C;
  const i64 base = slice_ptr[s];
  const int width = (int)((slice_ptr[s + 1] - base) / C);
  const int bb = br * bc, nd = br < bc ? br : bc;
  for (int k = 0; k < width; ++k)
  {
    const i32 c = col[base + (i64)k * C + l];
    if (c == (i32)(r + own_blk))
      for (int d = 0; d < nd; ++d) val[(base + (i64)k * C) * bb + (i64)(d * bc + d) * C + l] += shift;
  }
}
// The symmetric band image's diagonal array (offset 0 = sym_off[k0]): rows whose mask has bit k0.
template <class MT>
__global__ void k_shift_sym(i64 nrows, i64 own, const MT *__restrict__ mask, int k0, double *__restrict__ diag,
                            double shift)
{
  const i64 r = (i64)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  if ((mask[r] >> k0) & 1u) diag[own + r] += shift;
}
static void launch_shift_values(eig_mat_s &A, double shift, i64 G, hipStream_t s);
void launch_shift_diag(eig_mat_s &A, double shift, hipStream_t s)
{
  box_invalidate(A);  // (the box image copies the band values; rebuilt at its next use)
  A.diag_sum += shift * (double)A.diag_count;
  const i64 G = (A.nb_rows + 255) / 256;
  if (G == 0) return;
  launch_shift_values(A, shift, G, s);
  // the packed value image of the value march copies the band values too: refilled in place after the
  // shift (same buffer, so a hipGraph captured over the march stays valid)
  if (A.sym_pack) sym_pack_fill(A, s);
}
static void launch_shift_values(eig_mat_s &A, double shift, i64 G, hipStream_t s)
{
  hipLaunchKernelGGL(k_shift_diag, dim3((unsigned)G), dim3(256), 0, s, A.nb_rows, A.own_offset / A.bc, A.slice_ptr,
                     A.col, A.val, A.br, A.bc, 64 * A.R, shift);
  if (A.sym_val)
  {
    int k0 = -1;
    for (int k = 0; k < A.sym_nd; ++k)
      if (A.sym_off[k] == 0) k0 = k;
    if (k0 < 0) return;  // no row stores a diagonal entry
    double *diag = A.sym_val + (i64)A.sym_dj[k0] * A.sym_ld;
    A.sym_uc[A.sym_dj[k0]] += shift;  // (k_shift_sym's addition: a uniform diagonal stays uniform)
    if (A.sym_mask_bytes == 1)
      hipLaunchKernelGGL(k_shift_sym<uint8_t>, dim3((unsigned)G), dim3(256), 0, s, A.nb_rows, A.own_offset,
                         static_cast<const uint8_t *>(A.sym_mask), k0, diag, shift);
    else
      hipLaunchKernelGGL(k_shift_sym<uint32_t>, dim3((unsigned)G), dim3(256), 0, s, A.nb_rows, A.own_offset,
                         static_cast<const uint32_t *>(A.sym_mask), k0, diag, shift);
  }
}

// ---------------------------------------------------------------------------------------------
// Re-orthogonalisation GEMVs on a column-major basis V (k columns, leading dimension ldv):
//   c = V^T w  (column tiles of 8 on grid.y, one grid reduction per tile)
//   w -= V c
// ---------------------------------------------------------------------------------------------
constexpr int kGemvBlocks = 512;

constexpr double kDgks2 = 0.717 * 0.717;  // ARPACK dsaitr's DGKS threshold, squared

__device__ __forceinline__ bool gated_off(const double *gate)
{
  return gate && !(gate[0] <= kDgks2 * gate[1]);
}

__global__ __launch_bounds__(kStreamThreads) void k_gemv_t(i64 n, int k, const double *__restrict__ V, i64 ldv,
                                                           const double *__restrict__ w, double *__restrict__ c,
                                                           double *partials, unsigned *tickets, const double *gate)
{
  if (gated_off(gate)) return;  // (every block: the ticket is never touched)
  __shared__ double tot[8];
  const int c0 = blockIdx.y * 8;
  double acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.0;
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
  {
    const double wi = w[i];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (c0 + q < k) acc[q] += V[(i64)(c0 + q) * ldv + i] * wi;
  }
  if (grid_sum_n<8, kStreamThreads>(acc, partials + (size_t)blockIdx.y * gridDim.x * 8, tickets + (size_t)blockIdx.y * kTicketStride, tot,
                                    blockIdx.x, gridDim.x))
  {
    if (threadIdx.x < 8 && c0 + (int)threadIdx.x < k) c[c0 + threadIdx.x] = tot[threadIdx.x];
  }
}

void launch_gemv_t(i64 n, int k, const double *V, i64 ldv, const double *w, double *c, int ticket, hipStream_t s,
                   ReduceWS red, const double *gate)
{
  const int tiles = (k + 7) / 8;
  EIG_CHECK(ticket + tiles <= kNumTickets, EIG_ERR_ARG, "gemv_t: too many column tiles for the ticket pool");
  int G = stream_grid(n, 4);
  if (G > kGemvBlocks) G = kGemvBlocks;
  EIG_CHECK((i64)G * tiles * 8 <= (i64)kMaxRedBlocks * kMaxRedVals, EIG_ERR_ARG, "gemv_t: partials overflow");
  hipLaunchKernelGGL(k_gemv_t, dim3(G, tiles), dim3(kStreamThreads), 0, s, n, k, V, ldv, w, c, red.partials,
                     red.ticket(ticket), gate);
}

__global__ __launch_bounds__(kStreamThreads) void k_gemv_n(i64 n, int k, const double *__restrict__ V, i64 ldv,
                                                           const double *__restrict__ c, const double *__restrict__ sc,
                                                           int mode, double *__restrict__ w, const double *gate)
{
  if (gated_off(gate)) return;
  // mode 0: w -= sum V_q c_q / sc_q (sc may be null)  ; mode 1: w = sum V_q c_q / sqrt(sc_q)
  __shared__ double coef[512];
  for (int q = threadIdx.x; q < k && q < 512; q += blockDim.x)
  {
    double cq = c[q];
    if (sc) cq = (mode == 0) ? cq / sc[q] : cq * (1.0 / sqrt(sc[q]));
    coef[q] = cq;
  }
  __syncthreads();
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
  {
    double s = 0.0;
    for (int q = 0; q < k; ++q) s += V[(i64)q * ldv + i] * coef[q];
    if (mode == 0) w[i] -= s;
    else w[i] = s;
  }
}
void launch_gemv_n_sub(i64 n, int k, const double *V, i64 ldv, const double *c, const double *scale2, double *w,
                       hipStream_t s, const double *gate)
{
  EIG_CHECK(k <= 512, EIG_ERR_ARG, "gemv_n: at most 512 basis vectors");
  if (k <= 0) return;
  hipLaunchKernelGGL(k_gemv_n, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, k, V, ldv, c, scale2, 0, w,
                     gate);
}
// t = 0 when the gate is on (DGKS gave up: dsaitr's r = 0, rnorm = 0); returns at once otherwise
__global__ __launch_bounds__(kStreamThreads) void k_zero_gated(i64 n, double *__restrict__ w, const double *gate)
{
  if (gated_off(gate)) return;
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads) w[i] = 0.0;
}
void launch_zero_gated(i64 n, double *w, const double *gate, hipStream_t s)
{
  hipLaunchKernelGGL(k_zero_gated, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, w, gate);
}
void launch_gemv_n_set(i64 n, int k, const double *V, i64 ldv, const double *c, const double *nsum, double *y,
                       hipStream_t s)
{
  EIG_CHECK(k <= 512, EIG_ERR_ARG, "gemv_n: at most 512 basis vectors");
  hipLaunchKernelGGL(k_gemv_n, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, k, V, ldv, c, nsum, 1, y,
                     (const double *)nullptr);
}

// out = ||x - theta*y||^2
__global__ __launch_bounds__(kStreamThreads) void k_resid_sq(i64 n, const double *__restrict__ x,
                                                             const double *__restrict__ y, double theta, double *out,
                                                             double *partials, unsigned *ticket)
{
  __shared__ double tot[1];
  double acc = 0.0;
  for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += (i64)gridDim.x * kStreamThreads)
  {
    const double r = x[i] - theta * y[i];
    acc += r * r;
  }
  double v[1] = {acc};
  if (grid_sum<1, kStreamThreads>(v, partials, ticket, tot))
    if (threadIdx.x == 0) out[0] = tot[0];
}
void launch_resid_sq(i64 n, const double *x, const double *y, double theta, double *out, int ticket, hipStream_t s,
                     ReduceWS red)
{
  hipLaunchKernelGGL(k_resid_sq, dim3(stream_grid(n, 4)), dim3(kStreamThreads), 0, s, n, x, y, theta, out,
                     red.partials, red.ticket(ticket));
}

}  // namespace eigmi

namespace eigmi {
// ---------------------------------------------------------------------------------------------
// Stream copy y = x (the measured HBM peak the roofline fractions are also quoted against, SURVEY
// 8(d)): 16 B per lane.  MODE (A/B, tools/copy_sweep.py): bit 0 = nontemporal loads / stores, bit 1
// = one element per thread over a full grid (else a resident grid striding 4 elements per pass).
// ---------------------------------------------------------------------------------------------
typedef double dv2s __attribute__((ext_vector_type(2)));
template <int MODE>
__global__ __launch_bounds__(kStreamThreads) void k_stream_copy(i64 n2, const dv2s *__restrict__ x,
                                                                dv2s *__restrict__ y)
{
  auto ld = [&](i64 i) { return (MODE & 1) ? __builtin_nontemporal_load(x + i) : x[i]; };
  auto st = [&](i64 i, dv2s v) {
    if (MODE & 1) __builtin_nontemporal_store(v, y + i);
    else y[i] = v;
  };
  i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x;
  if (MODE & 2)
  {
    if (i < n2) st(i, ld(i));
    return;
  }
  const i64 stride = (i64)gridDim.x * kStreamThreads;
  for (; i + 3 * stride < n2; i += 4 * stride)
  {
    dv2s a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = ld(i + k * stride);
#pragma unroll
    for (int k = 0; k < 4; ++k) st(i + k * stride, a[k]);
  }
  for (; i < n2; i += stride) st(i, ld(i));
}

void launch_stream_copy(i64 n, const double *x, double *y, int num_cu, hipStream_t s, int mode)
{
  const i64 n2 = n / 2;
  const i64 full = (n2 + kStreamThreads - 1) / kStreamThreads;
  const int G = (int)std::max<i64>(1, (mode & 2) ? full : std::min<i64>(full, (i64)num_cu * 8));
  const dv2s *xv = reinterpret_cast<const dv2s *>(x);
  dv2s *yv = reinterpret_cast<dv2s *>(y);
  if (n2 > 0) switch (mode & 3)
    {
      case 0: hipLaunchKernelGGL(k_stream_copy<0>, dim3(G), dim3(kStreamThreads), 0, s, n2, xv, yv); break;
      case 1: hipLaunchKernelGGL(k_stream_copy<1>, dim3(G), dim3(kStreamThreads), 0, s, n2, xv, yv); break;
      case 2: hipLaunchKernelGGL(k_stream_copy<2>, dim3(G), dim3(kStreamThreads), 0, s, n2, xv, yv); break;
      default: hipLaunchKernelGGL(k_stream_copy<3>, dim3(G), dim3(kStreamThreads), 0, s, n2, xv, yv); break;
    }
  if (n & 1) EIG_HIP(hipMemcpyAsync(y + n - 1, x + n - 1, sizeof(double), hipMemcpyDeviceToDevice, s));
  EIG_HIP(hipGetLastError());
}
}  // namespace eigmi
