// k_box.hip -- 32-column SpMM and fused Chebyshev step for 3-D box stencils (gfx950), config C5.
//
// A square 1x1 matrix whose band image (internal.h eig_mat_s::sym_*) has offsets d = a P + b Nx + c,
// a, b, c in {-1, 0, 1}, on an Nx x Ny x Nz grid (rows x + Nx (y + Ny z), no entry crossing a grid
// face: the generators' 7-point Poisson and P1 Kuhn K / M), multiplied into m = 32 columns
// (4 column blocks of a MultiVector<double,8>) at once.
//
// Why a separate kernel: the register plane march (k_spmm8_marchg) gathers each X row ~11 times
// from L2 (every non-carried offset), and at 32 columns the streams of a plane (X, B, x_{k-1},
// x_{k+1}, band) fill an XCD's 4 MiB L2, so the neighbour rows are evicted before their reuse:
// rocprof measured 32.6 GB fetched per Chebyshev launch against ~18 GB of data
// (profiles/r02_c5_pmc_summary.json).  Here a workgroup owns a TX x TY tile of every plane and
// marches z, keeping X of planes z-1, z, z+1 with a one-row halo in LDS (3 x 10 x 18 rows x 32
// columns): every X row is fetched ~1.4 times (the halo) and every matrix value once for all 32
// columns.  The values come from a "box image": one array per stored offset in ascending order
// (lower entries mirrored from the band image), built on the device at first use.
//
// Per row and column the stored entries are summed in ascending-column order; EPI = kBoxStore
// rounds products and sums separately (bitwise the reference SpMM, kernels_cpp.hh:644-655),
// kBoxCheb uses fused multiply-adds and the Chebyshev-Jacobi update of k_spmm8_marchg.
#include "internal.h"

namespace eigmi {

namespace {

constexpr int kBoxTX = 16, kBoxTY = 8;                         // tile rows (x, y)
constexpr int kBoxHX = kBoxTX + 2, kBoxHY = kBoxTY + 2;        // with the one-row halo
constexpr int kBoxThreads = 1024;  // 16 waves: wave = (tile y, x half), lane = (x, 4-column quad)
constexpr int kBoxChunks = kBoxHY * kBoxHX * 4 * 4;            // 16-B chunks of one plane (rows x blocks x 4)
constexpr int kBoxRounds = (kBoxChunks + kBoxThreads - 1) / kBoxThreads;
enum { kBoxStore = 0, kBoxCheb = 1 };
constexpr int kBoxMaxNd = 15;  // offsets the kernel holds in registers (P1 Kuhn: 15, 7-point: 7)

typedef double dv2b __attribute__((ext_vector_type(2)));

struct BoxGeom {
  int nx, ny, nz;  // grid
  int P;           // nx * ny
  int ntx, nty;    // tiles per plane
  int nseg;        // z runs per tile column
  int nd;          // stored offsets
  // per offset k: plane step dz (-1 / 0 / +1), LDS row shift (dy * kBoxHX + dx)
  int dz[27], dxy[27];
};

// Box image of the band: val[k * n + r] = a(r, r + off[k]) (0 where row r does not store it).
__global__ void k_box_image(i64 n, i64 ld, int nd, const i32 *__restrict__ off, const i32 *__restrict__ dj,
                            const double *__restrict__ sym, const void *__restrict__ mask, int mask_bytes,
                            double *__restrict__ val)
{
  for (i64 r = (i64)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (i64)gridDim.x * blockDim.x)
  {
    const unsigned m = mask_bytes == 1 ? static_cast<const uint8_t *>(mask)[r] : static_cast<const uint32_t *>(mask)[r];
    for (int k = 0; k < nd; ++k)
    {
      double v = 0.0;
      if ((m >> k) & 1u)
      {
        const i64 w = off[k] < 0 ? r + off[k] : r;
        v = sym[(i64)dj[k] * ld + w];
      }
      val[(i64)k * n + r] = v;
    }
  }
}

// Geometry check: every stored entry of row r stays inside the grid (no x / y / z wrap-around).
__global__ void k_box_check(i64 n, int nx, int ny, int nz, int nd, const i32 *__restrict__ dx,
                            const i32 *__restrict__ dy, const i32 *__restrict__ dzz, const void *__restrict__ mask,
                            int mask_bytes, unsigned *__restrict__ bad)
{
  for (i64 r = (i64)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (i64)gridDim.x * blockDim.x)
  {
    const unsigned m = mask_bytes == 1 ? static_cast<const uint8_t *>(mask)[r] : static_cast<const uint32_t *>(mask)[r];
    const int x = (int)(r % nx), y = (int)((r / nx) % ny), z = (int)(r / ((i64)nx * ny));
    for (int k = 0; k < nd; ++k)
      if ((m >> k) & 1u)
      {
        const int X = x + dx[k], Y = y + dy[k], Z = z + dzz[k];
        if (X < 0 || X >= nx || Y < 0 || Y >= ny || Z < 0 || Z >= nz) atomicOr(bad, 1u);
      }
  }
}

template <int EPI>
__global__ __launch_bounds__(kBoxThreads) void k_box_mv32(BoxGeom g, i64 ld, const double *__restrict__ val,
                                                          const uint32_t *__restrict__ mask32,
                                                          const uint8_t *__restrict__ mask8,
                                                          const double *__restrict__ X, double *__restrict__ Y,
                                                          const double *__restrict__ Xold,
                                                          const double *__restrict__ Bv,
                                                          const double *__restrict__ dinv, double omega,
                                                          double gamma)
{
  // X of planes z-1, z, z+1 (tile + halo, 32 columns per row, 256-B rows; column c of an odd row
  // at c ^ 2: the 16-B reads of lanes on adjacent rows then fall on distinct banks), and the
  // plane's matrix values and row masks (staged once per plane, read by the 8 threads of a row)
  __shared__ __attribute__((aligned(16))) double ring[3][kBoxHY * kBoxHX][32];
  __shared__ double atile[kBoxMaxNd][kBoxTX * kBoxTY];
  __shared__ unsigned mtile[kBoxTX * kBoxTY];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // 8 threads per row (4 columns each): 16 waves = 4 per SIMD with one workgroup per CU
  const int yi = wave >> 1, xi = (wave & 1) * 8 + (lane >> 3), cq = lane & 7, blk = cq >> 1, c4 = (cq & 1) * 4;
  // item = (tile, z run) in dispatch order (an XCD-contiguous item map -- workgroup b on XCD b % 8
  // taking one run of adjacent tiles -- measured no faster)
  const int item = (int)blockIdx.x;
  const int tile = item % (g.ntx * g.nty), seg = item / (g.ntx * g.nty);
  const int x0 = (tile % g.ntx) * kBoxTX, y0 = (tile / g.ntx) * kBoxTY;
  const int z0 = seg * g.nz / g.nseg, z1 = (seg + 1) * g.nz / g.nseg;
  const i64 n = (i64)g.P * g.nz;
  auto swz = [](int row, int col) { return col ^ ((row & 1) << 1); };
  // X plane zz of the tile + halo into ring slot zz mod 3: 16-B chunks, consecutive threads on
  // consecutive chunks of one (line, block) segment of 18 rows x 64 B
  dv2b pre[kBoxRounds];
  auto fetch = [&](int zz) {
#pragma unroll
    for (int i = 0; i < kBoxRounds; ++i)
    {
      const int c = tid + i * kBoxThreads;
      const int q = c & 3, hx = (c >> 2) % kBoxHX, rest = (c >> 2) / kBoxHX, b = rest & 3, hy = rest >> 2;
      const int x = x0 + hx - 1, y = y0 + hy - 1;
      const bool ok = c < kBoxChunks && zz >= 0 && zz < g.nz && x >= 0 && x < g.nx && y >= 0 && y < g.ny;
      const i64 row = ok ? (i64)x + (i64)g.nx * y + (i64)g.P * zz : 0;
      // plain loads: a plane's rows are also the halo of the neighbouring tiles (nontemporal X
      // loads measured the same, 4.21 vs 4.23 ms, in one interleaved run)
      const dv2b *src = reinterpret_cast<const dv2b *>(X + (i64)b * ld * 8 + row * 8) + q;
      pre[i] = ok ? *src : dv2b{0.0, 0.0};
    }
  };
  auto store = [&](int zz) {
    const int sl = ((zz % 3) + 3) % 3;
#pragma unroll
    for (int i = 0; i < kBoxRounds; ++i)
    {
      const int c = tid + i * kBoxThreads;
      if (c < kBoxChunks)
      {
        const int q = c & 3, hx = (c >> 2) % kBoxHX, rest = (c >> 2) / kBoxHX, b = rest & 3, hy = rest >> 2;
        const int hr = hy * kBoxHX + hx;
        *reinterpret_cast<dv2b *>(&ring[sl][hr][swz(hr, b * 8 + q * 2)]) = pre[i];
      }
    }
  };
  // the plane's matrix values / masks: thread t stages (row t % 128, offsets t / 128 + 8 j)
  constexpr int kRows = kBoxTX * kBoxTY, kVal = (kBoxMaxNd * kRows + kBoxThreads - 1) / kBoxThreads;
  const int srow = tid % kRows, sk0 = tid / kRows;
  const int sx = x0 + (srow % kBoxTX), sy = y0 + (srow / kBoxTX);
  const bool sown = sx < g.nx && sy < g.ny;
  double vpre[kVal];
  unsigned mpre = 0u;
  auto fetch_vals = [&](int zz) {
    const i64 r = sown && zz < z1 ? (i64)sx + (i64)g.nx * sy + (i64)g.P * zz : -1;
#pragma unroll
    for (int j = 0; j < kVal; ++j)
    {
      const int k = sk0 + j * (kBoxThreads / kRows);
      vpre[j] = (r >= 0 && k < g.nd) ? __builtin_nontemporal_load(val + (i64)k * n + r) : 0.0;
    }
    if (sk0 == 0) mpre = r >= 0 ? (mask32 ? mask32[r] : (unsigned)mask8[r]) : 0u;
  };
  auto store_vals = [&]() {
#pragma unroll
    for (int j = 0; j < kVal; ++j)
    {
      const int k = sk0 + j * (kBoxThreads / kRows);
      if (k < kBoxMaxNd) atile[k][srow] = vpre[j];
    }
    if (sk0 == 0) mtile[srow] = mpre;
  };
  const int x = x0 + xi, y = y0 + yi;
  const bool own = x < g.nx && y < g.ny;
  const int trow = yi * kBoxTX + xi;            // this thread's row in the tile
  const int hrow = (yi + 1) * kBoxHX + xi + 1;  // ... and in the halo tile
  // this thread's Chebyshev operands of plane zz (B, x_{k-1}, gamma / a_rr), one plane ahead
  dv2b bb[2] = {}, xo[2] = {}, bn[2] = {}, xn[2] = {};
  double gd = 0.0, gn = 0.0;
  auto fetch_cheb = [&](int zz, dv2b (&b2)[2], dv2b (&x2)[2], double &gg) {
    if (EPI != kBoxCheb || !own || zz >= z1) return;
    const i64 r = (i64)x + (i64)g.nx * y + (i64)g.P * zz;
    const double *br = Bv + (i64)blk * ld * 8 + r * 8 + c4, *yr = Xold + (i64)blk * ld * 8 + r * 8 + c4;
    gg = gamma * __builtin_nontemporal_load(dinv + r);
#pragma unroll
    for (int j = 0; j < 2; ++j)
    {
      b2[j] = __builtin_nontemporal_load(reinterpret_cast<const dv2b *>(br) + j);
      x2[j] = __builtin_nontemporal_load(reinterpret_cast<const dv2b *>(yr) + j);
    }
  };
  // prologue: X planes z0 - 1 .. z0 + 1, the values of plane z0, the Chebyshev operands of z0
  fetch(z0 - 1);
  store(z0 - 1);
  fetch(z0);
  store(z0);
  fetch(z0 + 1);
  store(z0 + 1);
  fetch_vals(z0);
  store_vals();
  fetch_cheb(z0, bb, xo, gd);
  for (int z = z0; z < z1; ++z)
  {
    __syncthreads();  // ring holds planes z - 1, z, z + 1; atile / mtile plane z
    // in flight during the products: the next plane's values and operands, X of plane z + 2
    fetch_vals(z + 1);
    fetch_cheb(z + 1, bn, xn, gn);
    fetch(z + 2);
    const unsigned m = own ? mtile[trow] : 0u;
    double acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = 0.0;
    // (partially unrolled: a full unroll hoists all 15 offsets' LDS reads and spills)
#pragma unroll 4
    for (int k = 0; k < g.nd; ++k)
    {
      if (!((m >> k) & 1u)) continue;
      const double a = atile[k][trow];
      const int sl = (((z + g.dz[k]) % 3) + 3) % 3, hr = hrow + g.dxy[k];
      // two 16-B LDS reads (ds_read_b128)
      const dv2b p0 = *reinterpret_cast<const dv2b *>(&ring[sl][hr][swz(hr, blk * 8 + c4)]);
      const dv2b p1 = *reinterpret_cast<const dv2b *>(&ring[sl][hr][swz(hr, blk * 8 + c4 + 2)]);
      const double xr[4] = {p0.x, p0.y, p1.x, p1.y};
#pragma unroll
      for (int j = 0; j < 4; ++j)
      {
        if (EPI == kBoxStore) acc[j] = acc[j] + a * xr[j];
        else acc[j] = __builtin_fma(a, xr[j], acc[j]);
      }
    }
    if (own)
    {
      const i64 r = (i64)x + (i64)g.nx * y + (i64)g.P * z;
      double *yr = Y + (i64)blk * ld * 8 + r * 8 + c4;
      if (EPI == kBoxStore)
      {
#pragma unroll
        for (int j = 0; j < 4; j += 2) __builtin_nontemporal_store(dv2b{acc[j], acc[j + 1]}, reinterpret_cast<dv2b *>(yr + j));
      }
      else
      {
        const int sl = ((z % 3) + 3) % 3;
        const dv2b c0 = *reinterpret_cast<const dv2b *>(&ring[sl][hrow][swz(hrow, blk * 8 + c4)]);
        const dv2b c1 = *reinterpret_cast<const dv2b *>(&ring[sl][hrow][swz(hrow, blk * 8 + c4 + 2)]);
        const double xc[4] = {c0.x, c0.y, c1.x, c1.y};
#pragma unroll
        for (int j = 0; j < 2; ++j)
        {
          const double o0 = omega * (xc[2 * j] + gd * (bb[j].x - acc[2 * j]) - xo[j].x) + xo[j].x;
          const double o1 = omega * (xc[2 * j + 1] + gd * (bb[j].y - acc[2 * j + 1]) - xo[j].y) + xo[j].y;
          __builtin_nontemporal_store(dv2b{o0, o1}, reinterpret_cast<dv2b *>(yr) + j);
        }
      }
    }
    __syncthreads();  // everyone is done with slot (z - 1) mod 3 and with atile
    store(z + 2);
    store_vals();
#pragma unroll
    for (int j = 0; j < 2; ++j)
    {
      bb[j] = bn[j];
      xo[j] = xn[j];
    }
    gd = gn;
  }
}

}  // namespace

void box_invalidate(eig_mat_s &A)
{
  if (A.box_val)
  {
    (void)hipStreamSynchronize(A.ctx->stream);
    (void)hipFree(A.box_val);
    A.device_bytes -= (i64)A.sym_nd * A.nb_rows * (i64)sizeof(double);
  }
  A.box_val = nullptr;
  A.box_state = 0;
}

// Box-stencil geometry of a band image and its device box image (built on first use and cached on
// the matrix); false when the matrix does not qualify.
bool box_prepare(const eig_mat_s &Ac)
{
  eig_mat_s &A = const_cast<eig_mat_s &>(Ac);
  if (A.box_state != 0) return A.box_state > 0;
  A.box_state = -1;
  if (!A.sym_val || A.br != 1 || A.bc != 1 || A.ctx->distributed() || (A.kflags & EIG_MAT_NO_MARCH)) return false;
  if (A.sym_nd > kBoxMaxNd || A.nb_rows != A.nb_rows_global || A.window != A.nb_rows) return false;
  // Nx = the smallest offset > 1, P = the smallest offset > Nx + 1
  i64 nx = 0, P = 0;
  for (int k = 0; k < A.sym_nd; ++k)
    if (A.sym_off[k] > 1 && (nx == 0 || A.sym_off[k] < nx)) nx = A.sym_off[k];
  for (int k = 0; k < A.sym_nd; ++k)
    if (nx > 0 && A.sym_off[k] > nx + 1 && (P == 0 || A.sym_off[k] < P)) P = A.sym_off[k];
  if (nx < kBoxTX || P == 0 || P % nx != 0 || A.nb_rows % P != 0) return false;
  const i64 ny = P / nx, nz = A.nb_rows / P;
  if (ny < kBoxTY || nz < 3 || nz > (1 << 24)) return false;
  std::vector<i32> dx(A.sym_nd), dy(A.sym_nd), dz(A.sym_nd);
  for (int k = 0; k < A.sym_nd; ++k)
  {
    const i64 d = A.sym_off[k];
    bool found = false;
    for (int a = -1; a <= 1 && !found; ++a)
      for (int b = -1; b <= 1 && !found; ++b)
        for (int c = -1; c <= 1 && !found; ++c)
          if (a * P + b * nx + c == d)
          {
            dz[k] = a, dy[k] = b, dx[k] = c;
            found = true;
          }
    if (!found) return false;
  }
  hipStream_t s = A.ctx->stream;
  const i64 n = A.nb_rows;
  // wrap-around check on the device (rows on a face storing an entry across it)
  {
    DevBuf meta((size_t)(4 * A.sym_nd + 2) * sizeof(i32));
    i32 *dm = static_cast<i32 *>(meta.p);
    std::vector<i32> h(4 * A.sym_nd + 2, 0);
    for (int k = 0; k < A.sym_nd; ++k) h[k] = dx[k], h[A.sym_nd + k] = dy[k], h[2 * A.sym_nd + k] = dz[k];
    EIG_HIP(hipMemcpyAsync(dm, h.data(), h.size() * sizeof(i32), hipMemcpyHostToDevice, s));
    unsigned *bad = reinterpret_cast<unsigned *>(dm + 3 * A.sym_nd);
    EIG_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned), s));
    hipLaunchKernelGGL(k_box_check, dim3(2048), dim3(256), 0, s, n, (int)nx, (int)ny, (int)nz, A.sym_nd, dm,
                       dm + A.sym_nd, dm + 2 * A.sym_nd, (const void *)A.sym_mask, A.sym_mask_bytes, bad);
    unsigned hb = 0;
    EIG_HIP(hipMemcpyAsync(&hb, bad, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    EIG_HIP(hipStreamSynchronize(s));
    if (hb) return false;
  }
  // the box image: one array per offset
  {
    DevBuf od((size_t)2 * A.sym_nd * sizeof(i32));
    std::vector<i32> h(2 * A.sym_nd);
    for (int k = 0; k < A.sym_nd; ++k) h[k] = A.sym_off[k], h[A.sym_nd + k] = A.sym_dj[k];
    EIG_HIP(hipMemcpyAsync(od.p, h.data(), h.size() * sizeof(i32), hipMemcpyHostToDevice, s));
    double *val = nullptr;
    EIG_HIP(hipMalloc(&val, (size_t)A.sym_nd * n * sizeof(double)));
    const i32 *o = static_cast<const i32 *>(od.p);
    hipLaunchKernelGGL(k_box_image, dim3(2048), dim3(256), 0, s, n, A.sym_ld, A.sym_nd, o, o + A.sym_nd,
                       (const double *)A.sym_val, (const void *)A.sym_mask, A.sym_mask_bytes, val);
    EIG_HIP(hipStreamSynchronize(s));
    A.box_val = val;
  }
  A.box_nx = (int)nx;
  A.box_ny = (int)ny;
  A.box_nz = (int)nz;
  for (int k = 0; k < A.sym_nd; ++k)
  {
    A.box_dz[k] = dz[k];
    A.box_dxy[k] = dy[k] * kBoxHX + dx[k];
  }
  A.device_bytes += (i64)A.sym_nd * n * (i64)sizeof(double);
  A.box_state = 1;
  return true;
}

// Y = A X (EPI store) or the Chebyshev step into Xold (EPI cheb) for m % 32 == 0 columns on the box
// kernel; false when the matrix has no box geometry (the caller takes the band march).
static bool launch_box(const eig_mat_s &A, i64 m, const double *X, double *Y, const double *Xold, const double *Bv,
                       const double *dinv, double omega, double gamma, bool cheb, hipStream_t s)
{
  if (m <= 0 || m % 32 != 0 || !box_prepare(A)) return false;
  BoxGeom g;
  g.nx = A.box_nx;
  g.ny = A.box_ny;
  g.nz = A.box_nz;
  g.P = g.nx * g.ny;
  g.ntx = (g.nx + kBoxTX - 1) / kBoxTX;
  g.nty = (g.ny + kBoxTY - 1) / kBoxTY;
  // z runs: enough tiles x runs for two rounds of the 256 CUs (one 147 KB workgroup per CU)
  const int tiles = g.ntx * g.nty;
  g.nseg = std::max(1, std::min(g.nz / 8, (2 * A.ctx->num_cu + tiles - 1) / tiles));
  g.nd = A.sym_nd;
  for (int k = 0; k < 27; ++k)
  {
    g.dz[k] = k < A.sym_nd ? A.box_dz[k] : 0;
    g.dxy[k] = k < A.sym_nd ? A.box_dxy[k] : 0;
  }
  const uint32_t *m32 = A.sym_mask_bytes == 4 ? static_cast<const uint32_t *>(A.sym_mask) : nullptr;
  const uint8_t *m8 = A.sym_mask_bytes == 1 ? static_cast<const uint8_t *>(A.sym_mask) : nullptr;
  const i64 ld = A.window;
  for (i64 c0 = 0; c0 < m; c0 += 32)
  {
    const i64 off = c0 * ld;  // 4 column blocks of ld rows x 8
    if (cheb)
      hipLaunchKernelGGL(k_box_mv32<kBoxCheb>, dim3((unsigned)(tiles * g.nseg)), dim3(kBoxThreads), 0, s, g, ld,
                         (const double *)A.box_val, m32, m8, X + off, Y + off, Xold + off, Bv + off, dinv, omega,
                         gamma);
    else
      hipLaunchKernelGGL(k_box_mv32<kBoxStore>, dim3((unsigned)(tiles * g.nseg)), dim3(kBoxThreads), 0, s, g, ld,
                         (const double *)A.box_val, m32, m8, X + off, Y + off, (const double *)nullptr,
                         (const double *)nullptr, (const double *)nullptr, 0.0, 0.0);
  }
  EIG_HIP(hipGetLastError());
  return true;
}

bool launch_box_spmm(const eig_mat_s &A, i64 m, const double *X, double *Y, hipStream_t s)
{
  return launch_box(A, m, X, Y, nullptr, nullptr, nullptr, 0.0, 0.0, false, s);
}

bool launch_box_cheb(const eig_mat_s &M, i64 m, const double *Xk, double *Xold, const double *B, const double *dinv,
                     double omega, double gamma, hipStream_t s, double *Xnew)
{
  return launch_box(M, m, Xk, Xnew ? Xnew : Xold, Xold, B, dinv, omega, gamma, true, s);
}

}  // namespace eigmi
