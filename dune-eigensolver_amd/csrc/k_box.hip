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
#include "reduce_dev.h"

namespace eigmi {

namespace {

constexpr int kBoxTX = 16, kBoxTY = 8;                         // tile rows (x, y)
constexpr int kBoxHX = kBoxTX + 2, kBoxHY = kBoxTY + 2;        // with the one-row halo
constexpr int kBoxThreads = 1024;  // 16 waves: wave = (tile y, x half), lane = (x, 4-column quad)
constexpr int kBoxChunks = kBoxHY * kBoxHX * 4 * 4;            // 16-B chunks of one plane (rows x blocks x 4)
constexpr int kBoxRounds = (kBoxChunks + kBoxThreads - 1) / kBoxThreads;
// kBoxResid: Y = B - A X (multigrid residual).  Row-class kernel only: kBoxChebFirst, the first
// Chebyshev step from x_0 = 0 with x_1 = gamma D^-1 b formed while b's planes enter the ring, and
// kBoxChebSecond, the second step with x_{k-1} = x_1 = gamma D^-1 b formed from the row's b (x_1 is
// never stored: two vector passes less per solve)
// kBoxChebFirstAdd: kBoxChebFirst added into Y (Y += x_2: a degree-2 smoother's correction applied
// in place, the multigrid post-smoother)
// kBoxResidCopy / kBoxResidAcc: kBoxResid that also sets / adds the input block into a second
// output (Xold's slot): the multigrid outer iteration's X = E or X += E beside r = b - A E
enum {
  kBoxStore = 0,
  kBoxCheb = 1,
  kBoxResid = 2,
  kBoxChebFirst = 3,
  kBoxChebSecond = 4,
  kBoxChebFirstAdd = 5,
  kBoxResidCopy = 6,
  kBoxResidAcc = 7,
  kBoxStoreDot = 8,  // kBoxStore + the diagonal dots x_j . y_j of each column (row-class kernel only)
  kBoxStoreDotGram = 9  // kBoxStoreDot + the window Gram y_w . y_c of the 8 columns (m = 8; reduce_dev.h)
};
// kBoxStoreDot's reduction: dp[8 b + j] = sum_r X(r, 8b + j) Y(r, 8b + j), one deterministic grid sum
// (workgroup partials in part, a ticket per column block) -- dot_products_diagonal_blocked fused into
// the product that feeds it (StandardLargest, eigensolver.hh:84-85)
struct BoxDot {
  double *dp = nullptr;
  double *part = nullptr;
  unsigned *tick = nullptr;
  double *gram = nullptr;  // kBoxStoreDotGram: the 8 x 8 window Gram of Y (row-major, upper triangle)
  unsigned *zero_word = nullptr;  // kBoxStoreDotGram: zeroed by the last workgroup (the next MGS's barrier)
};
constexpr int kBoxMaxNd = 15;  // offsets of the box-image kernel's LDS value tile (P1 Kuhn: 15, 7-point: 7)
constexpr int kBoxClassMaxNd = 27;  // offsets of the row-class kernels (27: Galerkin coarse operators)

typedef double dv2b __attribute__((ext_vector_type(2)));

struct BoxGeom {
  int nx, ny, nz;  // grid
  int P;           // nx * ny
  int ntx, nty;    // tiles per plane
  int nseg;        // z runs per tile column
  int nd;          // stored offsets
  int xmap;        // k_box_mv32: 1 = XCD-contiguous item map (eig_mat_tune EIG_TUNE_BOX_MAP)
  int zlo = 0, zhi = 0;  // a rank's slab (k_box_mv32, k_boxc_mv8): ghost planes -1 / nz present in the window
  int gz0 = 0, gnz = 0;  // k_boxc_mv8: the slab's first global plane and the grid's planes (row classes)
  // per offset k: plane step dz (-1 / 0 / +1), LDS row shift (dy * kBoxHX + dx)
  int dz[27], dxy[27];
};

// Compile-time box stencils: SHAPE has bit (dz + 1) 9 + (dy + 1) 3 + (dx + 1) for every stored offset;
// the k-th set bit in that (lexicographic = ascending offset) order is the image's offset k.
constexpr unsigned kShape7 = (1u << 4) | (1u << 10) | (1u << 12) | (1u << 13) | (1u << 14) | (1u << 16) | (1u << 22);
constexpr unsigned kShape27 = (1u << 27) - 1u;  // full box (Galerkin coarse operators)
// P1 on the Kuhn split: all offsets whose nonzero components share one sign
constexpr unsigned kShapeKuhn = (1u << 0) | (1u << 1) | (1u << 3) | (1u << 4) | (1u << 9) | (1u << 10) | (1u << 12) |
                                (1u << 13) | (1u << 14) | (1u << 16) | (1u << 17) | (1u << 22) | (1u << 23) |
                                (1u << 25) | (1u << 26);
struct BoxShapeTab {
  int nd;
  int dz[27], dy[27], dx[27];
};
constexpr BoxShapeTab box_shape_tab(unsigned shape)
{
  BoxShapeTab t{};
  for (int b = 0; b < 27; ++b)
    if ((shape >> b) & 1u)
    {
      t.dz[t.nd] = b / 9 - 1;
      t.dy[t.nd] = (b / 3) % 3 - 1;
      t.dx[t.nd] = b % 3 - 1;
      ++t.nd;
    }
  return t;
}

// Box image of the band: val[k * n + r] = a(r, r + off[k]) (0 where row r does not store it).
// (band arrays window-indexed: owned row r is window row own + r; a slab's mirrored lower entries
// of its first plane sit at ghost window rows)
__global__ void k_box_image(i64 n, i64 ld, i64 own, int nd, const i32 *__restrict__ off, const i32 *__restrict__ dj,
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
        const i64 w = own + (off[k] < 0 ? r + off[k] : r);
        v = sym[(i64)dj[k] * ld + w];
      }
      val[(i64)k * n + r] = v;
    }
  }
}

// Geometry check: every stored entry of row r stays inside the grid (no x / y / z wrap-around),
// else bad |= 1; a row that does not store an offset staying inside the grid sets bad |= 2 (the
// masks are then not the geometric ones: box_geomask stays false).  z is the global plane: a rank's
// slab starts at plane z0 of a grid of nz planes.
__global__ void k_box_check(i64 n, int nx, int ny, int nz, int z0, int nd, const i32 *__restrict__ dx,
                            const i32 *__restrict__ dy, const i32 *__restrict__ dzz, const void *__restrict__ mask,
                            int mask_bytes, unsigned *__restrict__ bad)
{
  unsigned b = 0u;
  for (i64 r = (i64)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (i64)gridDim.x * blockDim.x)
  {
    const unsigned m = mask_bytes == 1 ? static_cast<const uint8_t *>(mask)[r] : static_cast<const uint32_t *>(mask)[r];
    const int x = (int)(r % nx), y = (int)((r / nx) % ny), z = z0 + (int)(r / ((i64)nx * ny));
    for (int k = 0; k < nd; ++k)
    {
      const int X = x + dx[k], Y = y + dy[k], Z = z + dzz[k];
      const bool inside = X >= 0 && X < nx && Y >= 0 && Y < ny && Z >= 0 && Z < nz;
      if ((m >> k) & 1u)
        b |= inside ? 0u : 1u;
      else
        b |= inside ? 2u : 0u;
    }
  }
  if (b) atomicOr(bad, b);
}

template <int EPI, unsigned SHAPE>
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
  // item = (tile, z run) in dispatch order, or (xmap) XCD-contiguous: workgroup b (on XCD b % 8)
  // takes item (b % 8) gridDim / 8 + b / 8, so the workgroups resident on one XCD hold two whole
  // rows of adjacent tiles and read each other's halo rows from that XCD's L2 (measured: the same
  // fetch per row, 8-11 % slower -- profiles/r04j_boxk_map.jsonl; a measurement variant)
  const int item = g.xmap ? (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
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
      // (planes -1 and nz: a slab's ghost planes where the window holds them, else zero rows)
      const bool ok = c < kBoxChunks && zz >= -g.zlo && zz < g.nz + g.zhi && x >= 0 && x < g.nx && y >= 0 && y < g.ny;
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
    if (SHAPE == 0 && sk0 == 0) mpre = r >= 0 ? (mask32 ? mask32[r] : (unsigned)mask8[r]) : 0u;
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
    if (EPI == kBoxStore || !own || zz >= z1) return;
    const i64 r = (i64)x + (i64)g.nx * y + (i64)g.P * zz;
    const double *br = Bv + (i64)blk * ld * 8 + r * 8 + c4;
#pragma unroll
    for (int j = 0; j < 2; ++j) b2[j] = __builtin_nontemporal_load(reinterpret_cast<const dv2b *>(br) + j);
    if (EPI != kBoxCheb) return;
    gg = gamma * __builtin_nontemporal_load(dinv + r);
    if (!Xold) return;  // x_{k-1} = 0 (the first step from a zero start): not read
    const double *yr = Xold + (i64)blk * ld * 8 + r * 8 + c4;
#pragma unroll
    for (int j = 0; j < 2; ++j) x2[j] = __builtin_nontemporal_load(reinterpret_cast<const dv2b *>(yr) + j);
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
    double acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = 0.0;
    auto add = [&](double a, dv2b p0, dv2b p1) {
      const double xr[4] = {p0.x, p0.y, p1.x, p1.y};
#pragma unroll
      for (int j = 0; j < 4; ++j)
      {
        if (EPI == kBoxStore) acc[j] = acc[j] + a * xr[j];
        else acc[j] = __builtin_fma(a, xr[j], acc[j]);
      }
    };
    const int s0 = z % 3, sm = s0 == 0 ? 2 : s0 - 1, sp = s0 == 2 ? 0 : s0 + 1;
    if constexpr (SHAPE != 0)
    {
      // compile-time stencil on geometric masks (box_geomask; as k_boxc_mv8): all offsets summed, an
      // unstored one with its zero image entry against a zero halo row -- the masked sums bitwise.
      // The swizzle of a row depends on its parity only, i.e. on the offset's dx, dy (compile time).
      constexpr BoxShapeTab T = box_shape_tab(SHAPE);
      constexpr int kGroup = 2;
      const int hb0 = hrow - kBoxHX - 1;  // (-1, -1) neighbour in the halo tile
      const double *rg = &ring[0][0][0];
      int pz[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) pz[q] = (q == 0 ? sm : q == 1 ? s0 : sp) * (kBoxHY * kBoxHX * 32) + hb0 * 32;
      const int par = hb0 & 1;  // parity of the (-1, -1) neighbour's halo row
      const int cA = blk * 8 + c4;
      // column offsets of the two 16-B reads for a row of the (-1, -1) neighbour's parity and the other
      const int e0 = swz(par, cA), e1 = swz(par, cA + 2), o0 = swz(par ^ 1, cA), o1 = swz(par ^ 1, cA + 2);
      asm volatile("" : "+v"(pz[0]), "+v"(pz[1]), "+v"(pz[2]));
#pragma unroll
      for (int k = 0; k < T.nd; ++k)
      {
        const int dr = (T.dy[k] + 1) * kBoxHX + T.dx[k] + 1;  // halo-row shift from (-1, -1)
        const int base = pz[T.dz[k] + 1] + dr * 32;
        const bool odd = dr & 1;
        const dv2b p0 = *reinterpret_cast<const dv2b *>(rg + base + (odd ? o0 : e0));
        const dv2b p1 = *reinterpret_cast<const dv2b *>(rg + base + (odd ? o1 : e1));
        add(atile[k][trow], p0, p1);
        // (the next group's reads wait for these sums: a bounded number of LDS reads in flight)
        if ((k + 1) % kGroup == 0 && k + 1 < T.nd)
          asm volatile("" : "+v"(pz[0]), "+v"(pz[1]), "+v"(pz[2]) : "v"(acc[0]), "v"(acc[1]), "v"(acc[2]), "v"(acc[3]));
      }
    }
    else
    {
      const unsigned m = own ? mtile[trow] : 0u;
      // (partially unrolled: a full unroll hoists all 15 offsets' LDS reads and spills)
#pragma unroll 4
      for (int k = 0; k < g.nd; ++k)
      {
        if (!((m >> k) & 1u)) continue;
        const double a = atile[k][trow];
        const int sl = g.dz[k] < 0 ? sm : (g.dz[k] > 0 ? sp : s0), hr = hrow + g.dxy[k];
        // two 16-B LDS reads (ds_read_b128)
        add(a, *reinterpret_cast<const dv2b *>(&ring[sl][hr][swz(hr, blk * 8 + c4)]),
            *reinterpret_cast<const dv2b *>(&ring[sl][hr][swz(hr, blk * 8 + c4 + 2)]));
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
      else if (EPI == kBoxResid)
      {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          __builtin_nontemporal_store(dv2b{bb[j].x - acc[2 * j], bb[j].y - acc[2 * j + 1]}, reinterpret_cast<dv2b *>(yr) + j);
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

// Push-order box kernel (round 4): 16 columns per workgroup and ONE X plane in LDS.  Iteration p
// holds X of plane p (tile + halo) and adds its products into three rows' sums at once: the dz = +1
// terms of the row on plane p - 1 (whose sum is then complete: epilogue), the dz = 0 terms of the row
// on plane p and the dz = -1 terms of the row on plane p + 1.  A row still sums its entries in
// ascending-column order (the dz = -1, 0, +1 groups in turn, ascending inside each), so kBoxStore
// stays bitwise the reference SpMM and every EPI equals k_box_mv32's.  38 KB of LDS and 512
// threads: two workgroups per CU, so one workgroup's load burst overlaps the other's barriers
// (k_box_mv32 keeps three planes, 147 KB, and one workgroup per CU waits for each burst).  The two
// 16-column halves of a tile are workgroups b and b + 8 -- the same XCD, in flight together -- so
// the matrix values and D^-1 they both read can come from L2.  Measured (profiles/r04h_boxk_push.jsonl,
// variable-coefficient P1 256^3, m = 32): SpMM 2561 vs 2252 us, Chebyshev step 4743 vs 3921 us for
// k_box_mv32 -- slower, so it stays a measurement variant (EIG_TUNE_BOX_COLS = 16); k_box_mv32's
// PMC (profiles/r04i_boxk_pmc_summary.json) puts its loss in the X halo re-read, not in the pipeline.
constexpr int kPCols = 16, kPThreads = 512;
constexpr int kPChunks = kBoxHY * kBoxHX * (kPCols / 8) * 4;  // 16-B chunks of one plane (rows x 2 blocks x 4)
constexpr int kPRounds = (kPChunks + kPThreads - 1) / kPThreads;

template <int EPI, unsigned SHAPE>
__global__ __launch_bounds__(kPThreads, 4) void k_box_mv16p(BoxGeom g, i64 ld, int items,
                                                            const double *__restrict__ val,
                                                            const uint32_t *__restrict__ mask32,
                                                            const uint8_t *__restrict__ mask8,
                                                            const double *__restrict__ X, double *__restrict__ Y,
                                                            const double *__restrict__ Xold,
                                                            const double *__restrict__ Bv,
                                                            const double *__restrict__ dinv, double omega,
                                                            double gamma)
{
  __shared__ __attribute__((aligned(16))) double slot[kBoxHY * kBoxHX][kPCols];
  __shared__ double atile[kBoxMaxNd][kBoxTX * kBoxTY];
  __shared__ unsigned mtile[kBoxTX * kBoxTY];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // 4 threads per row (4 columns each): a wave is one x line of the tile
  const int yi = wave, xi = lane >> 2, cq = lane & 3, blk = cq >> 1, c4 = (cq & 1) * 4;
  const int item = (int)(blockIdx.x >> 4) * 8 + (int)(blockIdx.x & 7), half = (int)(blockIdx.x >> 3) & 1;
  if (item >= items) return;  // (whole workgroup: the grid is rounded up to 16 items)
  const i64 cofs = (i64)half * 2 * ld * 8;  // this half's two column blocks
  X += cofs;
  Y += cofs;
  if (Xold) Xold += cofs;
  if (Bv) Bv += cofs;
  const int tile = item % (g.ntx * g.nty), seg = item / (g.ntx * g.nty);
  const int x0 = (tile % g.ntx) * kBoxTX, y0 = (tile / g.ntx) * kBoxTY;
  const int z0 = seg * g.nz / g.nseg, z1 = (seg + 1) * g.nz / g.nseg;
  const i64 n = (i64)g.P * g.nz;
  auto swz = [](int row, int col) { return col ^ ((row & 1) << 1); };
  dv2b pre[kPRounds];
  auto fetch = [&](int zz) {
#pragma unroll
    for (int i = 0; i < kPRounds; ++i)
    {
      const int c = tid + i * kPThreads;
      const int q = c & 3, hx = (c >> 2) % kBoxHX, rest = (c >> 2) / kBoxHX, b = rest & 1, hy = rest >> 1;
      const int x = x0 + hx - 1, y = y0 + hy - 1;
      const bool ok = c < kPChunks && zz >= 0 && zz < g.nz && x >= 0 && x < g.nx && y >= 0 && y < g.ny;
      const i64 row = ok ? (i64)x + (i64)g.nx * y + (i64)g.P * zz : 0;
      const dv2b *src = reinterpret_cast<const dv2b *>(X + (i64)b * ld * 8 + row * 8) + q;
      pre[i] = ok ? *src : dv2b{0.0, 0.0};
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < kPRounds; ++i)
    {
      const int c = tid + i * kPThreads;
      if (c < kPChunks)
      {
        const int q = c & 3, hx = (c >> 2) % kBoxHX, rest = (c >> 2) / kBoxHX, b = rest & 1, hy = rest >> 1;
        const int hr = hy * kBoxHX + hx;
        *reinterpret_cast<dv2b *>(&slot[hr][swz(hr, b * 8 + q * 2)]) = pre[i];
      }
    }
  };
  // values of iteration p: offset k of the row on plane p - dz_k (staged by thread (row t % 128,
  // offsets t / 128 + 4 j); plain loads, the other half's workgroup reads them from L2)
  constexpr int kRows = kBoxTX * kBoxTY, kVal = (kBoxMaxNd * kRows + kPThreads - 1) / kPThreads;
  const int srow = tid % kRows, sk0 = __builtin_amdgcn_readfirstlane(tid / kRows);
  const int sx = x0 + (srow % kBoxTX), sy = y0 + (srow / kBoxTX);
  const bool sown = sx < g.nx && sy < g.ny;
  // the offsets' dz groups as bit sets (the generic path's row masks)
  unsigned bneg = 0u, bzero = 0u, bpos = 0u;
  if constexpr (SHAPE == 0)
    for (int k = 0; k < g.nd; ++k)
      (g.dz[k] < 0 ? bneg : g.dz[k] > 0 ? bpos : bzero) |= 1u << k;
  double vpre[kVal];
  unsigned mpre = 0u;
  auto plane_row = [&](int zz) { return sown && zz >= z0 && zz < z1 ? (i64)sx + (i64)g.nx * sy + (i64)g.P * zz : (i64)-1; };
  auto fetch_vals = [&](int pp) {
#pragma unroll
    for (int j = 0; j < kVal; ++j)
    {
      const int k = sk0 + j * (kPThreads / kRows);
      double v = 0.0;
      if (k < g.nd)
      {
        const i64 r = plane_row(pp - g.dz[k]);
        if (r >= 0) v = val[(i64)k * n + r];
      }
      vpre[j] = v;
    }
    if (SHAPE == 0 && sk0 == 0)
    {
      auto mrow = [&](int zz) {
        const i64 r = plane_row(zz);
        return r >= 0 ? (mask32 ? mask32[r] : (unsigned)mask8[r]) : 0u;
      };
      mpre = (mrow(pp + 1) & bneg) | (mrow(pp) & bzero) | (mrow(pp - 1) & bpos);
    }
  };
  auto store_vals = [&]() {
#pragma unroll
    for (int j = 0; j < kVal; ++j)
    {
      const int k = sk0 + j * (kPThreads / kRows);
      if (k < kBoxMaxNd) atile[k][srow] = vpre[j];
    }
    if (sk0 == 0) mtile[srow] = mpre;
  };
  const int x = x0 + xi, y = y0 + yi;
  const bool own = x < g.nx && y < g.ny;
  const int trow = yi * kBoxTX + xi;
  const int hrow = (yi + 1) * kBoxHX + xi + 1;
  // Chebyshev operands of plane zz (loaded in iteration zz after the epilogue of plane zz - 1, used in
  // iteration zz + 1)
  dv2b bb[2] = {}, xo[2] = {};
  double gd = 0.0;
  auto fetch_cheb = [&](int zz, dv2b (&b2)[2], dv2b (&x2)[2], double &gg) {
    if (EPI == kBoxStore || !own || zz < z0 || zz >= z1) return;
    const i64 r = (i64)x + (i64)g.nx * y + (i64)g.P * zz;
    const double *br = Bv + (i64)blk * ld * 8 + r * 8 + c4;
#pragma unroll
    for (int j = 0; j < 2; ++j) b2[j] = __builtin_nontemporal_load(reinterpret_cast<const dv2b *>(br) + j);
    if (EPI != kBoxCheb) return;
    gg = gamma * dinv[r];
    if (!Xold) return;
    const double *yr = Xold + (i64)blk * ld * 8 + r * 8 + c4;
#pragma unroll
    for (int j = 0; j < 2; ++j) x2[j] = __builtin_nontemporal_load(reinterpret_cast<const dv2b *>(yr) + j);
  };
  // sums of the rows on planes p - 1 (am: completed first, then reused for plane p + 1) and p (a0);
  // X of the own row on plane p - 1
  double am[4] = {}, a0[4] = {};
  dv2b xc[2] = {};
  fetch(z0 - 1);
  fetch_vals(z0 - 1);
  store();
  store_vals();
  for (int p = z0 - 1; p <= z1; ++p)
  {
    __syncthreads();  // slot holds X of plane p, atile / mtile the values of iteration p
    if (p + 1 <= z1)
    {
      fetch_vals(p + 1);
      fetch(p + 1);
    }
    auto add = [&](double (&acc)[4], double a, dv2b p0, dv2b p1) {
      const double xr[4] = {p0.x, p0.y, p1.x, p1.y};
#pragma unroll
      for (int j = 0; j < 4; ++j)
      {
        if (EPI == kBoxStore) acc[j] = acc[j] + a * xr[j];
        else acc[j] = __builtin_fma(a, xr[j], acc[j]);
      }
    };
    // the products of the offsets with dz == D into acc (ascending offsets)
    auto products = [&](auto dtag, double (&acc)[4]) {
      constexpr int D = decltype(dtag)::value;
      if constexpr (SHAPE != 0)
      {
        constexpr BoxShapeTab T = box_shape_tab(SHAPE);
        constexpr int kGroup = 2;
        const int hb0 = hrow - kBoxHX - 1;
        const double *rg = &slot[0][0];
        int pz = hb0 * kPCols;
        const int par = hb0 & 1;
        const int cA = blk * 8 + c4;
        const int e0 = swz(par, cA), e1 = swz(par, cA + 2), o0 = swz(par ^ 1, cA), o1 = swz(par ^ 1, cA + 2);
        asm volatile("" : "+v"(pz));
        int cnt = 0;
#pragma unroll
        for (int k = 0; k < T.nd; ++k)
        {
          if (T.dz[k] != D) continue;
          const int dr = (T.dy[k] + 1) * kBoxHX + T.dx[k] + 1;
          const int base = pz + dr * kPCols;
          const bool odd = dr & 1;
          const dv2b p0 = *reinterpret_cast<const dv2b *>(rg + base + (odd ? o0 : e0));
          const dv2b p1 = *reinterpret_cast<const dv2b *>(rg + base + (odd ? o1 : e1));
          add(acc, atile[k][trow], p0, p1);
          // (the next group's reads wait for these sums: a bounded number of LDS reads in flight)
          if (++cnt % kGroup == 0)
            asm volatile("" : "+v"(pz) : "v"(acc[0]), "v"(acc[1]), "v"(acc[2]), "v"(acc[3]));
        }
      }
      else
      {
        const unsigned m = own ? mtile[trow] : 0u;
#pragma unroll 2
        for (int k = 0; k < g.nd; ++k)
        {
          if (g.dz[k] != D || !((m >> k) & 1u)) continue;
          const double a = atile[k][trow];
          const int hr = hrow + g.dxy[k];
          add(acc, a, *reinterpret_cast<const dv2b *>(&slot[hr][swz(hr, blk * 8 + c4)]),
              *reinterpret_cast<const dv2b *>(&slot[hr][swz(hr, blk * 8 + c4 + 2)]));
        }
      }
    };
    // dz = +1: the row on plane p - 1 is complete -> its epilogue (with the operands loaded in
    // iteration p - 1), then this plane's operands into the same registers
    products(std::integral_constant<int, 1>{}, am);
    if (own && p - 1 >= z0)
    {
      const i64 r = (i64)x + (i64)g.nx * y + (i64)g.P * (p - 1);
      double *yr = Y + (i64)blk * ld * 8 + r * 8 + c4;
      if (EPI == kBoxStore)
      {
#pragma unroll
        for (int j = 0; j < 4; j += 2) __builtin_nontemporal_store(dv2b{am[j], am[j + 1]}, reinterpret_cast<dv2b *>(yr + j));
      }
      else if (EPI == kBoxResid)
      {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          __builtin_nontemporal_store(dv2b{bb[j].x - am[2 * j], bb[j].y - am[2 * j + 1]}, reinterpret_cast<dv2b *>(yr) + j);
      }
      else
      {
        const double xr[4] = {xc[0].x, xc[0].y, xc[1].x, xc[1].y};
#pragma unroll
        for (int j = 0; j < 2; ++j)
        {
          const double o0 = omega * (xr[2 * j] + gd * (bb[j].x - am[2 * j]) - xo[j].x) + xo[j].x;
          const double o1 = omega * (xr[2 * j + 1] + gd * (bb[j].y - am[2 * j + 1]) - xo[j].y) + xo[j].y;
          __builtin_nontemporal_store(dv2b{o0, o1}, reinterpret_cast<dv2b *>(yr) + j);
        }
      }
    }
    fetch_cheb(p, bb, xo, gd);
    if (EPI == kBoxCheb)  // the own row's X on plane p, for its epilogue in iteration p + 1
    {
      xc[0] = *reinterpret_cast<const dv2b *>(&slot[hrow][swz(hrow, blk * 8 + c4)]);
      xc[1] = *reinterpret_cast<const dv2b *>(&slot[hrow][swz(hrow, blk * 8 + c4 + 2)]);
    }
    products(std::integral_constant<int, 0>{}, a0);
#pragma unroll
    for (int j = 0; j < 4; ++j) am[j] = 0.0;
    products(std::integral_constant<int, -1>{}, am);  // (am now holds the row on plane p + 1)
    __syncthreads();  // everyone is done with the slot and atile
    if (p + 1 <= z1)
    {
      store();
      store_vals();
    }
    // rotate: plane p's sum becomes the one completed next iteration
#pragma unroll
    for (int j = 0; j < 4; ++j)
    {
      const double t = a0[j];
      a0[j] = am[j];
      am[j] = t;
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Row-class box kernels.  On a box grid whose matrix has constant entries per geometric class
// (first / interior / last position along x, y and z: 27 classes -- the generators' 7-point Poisson
// and P1 Kuhn K / M, any constant-coefficient stencil with its boundary rows), a row's stored
// entries are those of its class representative.  The class table (27 x (nd values + 1 / a_rr),
// 27 masks) sits in LDS, so the SpMM and the Chebyshev step stream only the vectors: no box image,
// no band values, no row masks, no D^-1.  8 columns (one MultiVector block, 64-B rows) per
// workgroup (blockIdx.y = column block): 4 lanes per row, 16 consecutive x rows per wave, every
// vector access a 1-KiB contiguous run; a 32 x 8 tile with a one-row halo, 3 planes in LDS
// (3 x 340 rows x 64 B = 65 KiB: two workgroups per CU).  Entries summed in ascending-column order
// per row and column: kBoxStore bitwise the reference SpMM, kBoxCheb with FMA (as k_box_mv32).
// ---------------------------------------------------------------------------------------------
constexpr int kCTX = 32, kCTY = 8, kCHX = kCTX + 2, kCHY = kCTY + 2;
constexpr int kCThreads = 1024;
constexpr int kCChunks = kCHY * kCHX * 4;  // 16-B chunks of one plane (tile + halo, 8 columns)
constexpr int kCRounds = (kCChunks + kCThreads - 1) / kCThreads;
constexpr int kBoxClasses = 27;
constexpr int kCStride = 28;  // doubles per class: nd <= 27 values, then 1 / a_rr

__device__ __forceinline__ int box_cls1(int v, int nv) { return v == 0 ? 0 : (v == nv - 1 ? 2 : 1); }

// bad |= 1 when a row's mask or a stored entry differs from its class's (bitwise).
// (z: the global plane -- a rank's slab starts at plane z0 of a grid of nz planes)
__global__ void k_boxc_check(i64 n, int nx, int ny, int z0, int nz, int nd, const double *__restrict__ val,
                             const void *__restrict__ mask, int mask_bytes, const double *__restrict__ ctab,
                             const unsigned *__restrict__ cmask, unsigned *__restrict__ bad)
{
  for (i64 r = (i64)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (i64)gridDim.x * blockDim.x)
  {
    const int x = (int)(r % nx), y = (int)((r / nx) % ny);
    const i64 z = z0 + r / ((i64)nx * ny);
    const int c = (z == 0 ? 0 : (z == nz - 1 ? 2 : 1)) * 9 + box_cls1(y, ny) * 3 + box_cls1(x, nx);
    const unsigned m = mask_bytes == 1 ? static_cast<const uint8_t *>(mask)[r] : static_cast<const uint32_t *>(mask)[r];
    bool ok = m == cmask[c];
    for (int k = 0; k < nd && ok; ++k)
      if ((m >> k) & 1u)
        ok = __double_as_longlong(val[(i64)k * n + r]) == __double_as_longlong(ctab[c * kCStride + k]);
    if (!ok) atomicOr(bad, 1u);
  }
}

// out[c * (kCStride + 1) + k] = val[k n + rep[c]] (k < nd), out[c * (kCStride + 1) + kCStride] = mask
__global__ void k_boxc_gather(i64 n, int nd, const double *__restrict__ val, const void *__restrict__ mask,
                              int mask_bytes, const i64 *__restrict__ rep, double *__restrict__ out)
{
  const int c = blockIdx.x, k = threadIdx.x;
  const i64 r = rep[c];
  if (k < nd) out[c * (kCStride + 1) + k] = val[(i64)k * n + r];
  if (k == kCStride)
    out[c * (kCStride + 1) + k] = (double)(mask_bytes == 1 ? static_cast<const uint8_t *>(mask)[r]
                                                           : static_cast<const uint32_t *>(mask)[r]);
}


template <int EPI, unsigned SHAPE>
__global__ __launch_bounds__(kCThreads, EPI == kBoxStoreDotGram ? 4 : 8) void k_boxc_mv8(BoxGeom g, i64 ld, const double *__restrict__ ctab,
                                                        const unsigned *__restrict__ cmask,
                                                        const double *__restrict__ X, double *__restrict__ Y,
                                                        const double *__restrict__ Xold,
                                                        const double *__restrict__ Bv, double omega, double gamma,
                                                        BoxDot bd)
{
  __shared__ __attribute__((aligned(16))) dv2b ring[3][kCHY * kCHX][4];
  __shared__ double ct[kBoxClasses][kCStride];
  __shared__ unsigned cm[kBoxClasses];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < kBoxClasses * kCStride; i += kCThreads) ct[i / kCStride][i % kCStride] = ctab[i];
  if (tid < kBoxClasses) cm[tid] = cmask[tid];
  if constexpr (EPI == kBoxChebFirst || EPI == kBoxChebFirstAdd)
    __syncthreads();  // the prologue's ring stores read the class table
  const i64 boff = (i64)blockIdx.y * ld * 8;  // column block
  const dv2b *Xb = reinterpret_cast<const dv2b *>(X + boff);
  dv2b *Yb = reinterpret_cast<dv2b *>(Y + boff);
  const dv2b *Ob = reinterpret_cast<const dv2b *>(Xold ? Xold + boff : nullptr);
  const dv2b *Bb = reinterpret_cast<const dv2b *>(Bv ? Bv + boff : nullptr);
  const int item = (int)blockIdx.x;
  const int tile = item % (g.ntx * g.nty), seg = item / (g.ntx * g.nty);
  const int x0 = (tile % g.ntx) * kCTX, y0 = (tile / g.ntx) * kCTY;
  const int z0 = seg * g.nz / g.nseg, z1 = (seg + 1) * g.nz / g.nseg;
  constexpr bool first = EPI == kBoxChebFirst || EPI == kBoxChebFirstAdd;
  constexpr bool cheb = EPI == kBoxCheb || first || EPI == kBoxChebSecond;
  constexpr bool plain = EPI == kBoxStore || EPI == kBoxStoreDot || EPI == kBoxStoreDotGram;  // Y = A X
  constexpr bool dot = EPI == kBoxStoreDot || EPI == kBoxStoreDotGram;
  dv2b dsum = {0.0, 0.0};  // kBoxStoreDot: this thread's x . y over its rows, columns 2 cp, 2 cp + 1
  double gacc[2][8] = {};  // kBoxStoreDotGram: this lane's share of the window Gram (reduce_dev.h)
  // X plane zz of the tile + halo (8 columns, 64-B rows) into ring slot zz mod 3 (kBoxChebFirst: X is
  // b, and the ring takes x_1 = (gamma / a_rr) b with the row's class diagonal, as k_cheb_init)
  dv2b pre[kCRounds];
  auto fetch = [&](int zz) {
#pragma unroll
    for (int i = 0; i < kCRounds; ++i)
    {
      const int c = tid + i * kCThreads, q = c & 3, hr = c >> 2, hx = hr % kCHX, hy = hr / kCHX;
      const int x = x0 + hx - 1, y = y0 + hy - 1;
      const bool ok = c < kCChunks && zz >= -g.zlo && zz < g.nz + g.zhi && x >= 0 && x < g.nx && y >= 0 && y < g.ny;
      const i64 row = ok ? (i64)x + (i64)g.nx * y + (i64)g.P * zz : 0;
      pre[i] = ok ? Xb[row * 4 + q] : dv2b{0.0, 0.0};
    }
  };
  auto store = [&](int zz) {
    const int sl = ((zz % 3) + 3) % 3;
#pragma unroll
    for (int i = 0; i < kCRounds; ++i)
    {
      const int c = tid + i * kCThreads;
      if (c < kCChunks)
      {
        dv2b v = pre[i];
        if constexpr (first)
        {
          const int hr = c >> 2, xx = x0 + hr % kCHX - 1, yy = y0 + hr / kCHX - 1;
          const int zc = zz <= 0 ? 0 : (zz >= g.nz - 1 ? 2 : 1);
          const double gr = gamma * ct[zc * 9 + box_cls1(yy, g.ny) * 3 + box_cls1(xx, g.nx)][kCStride - 1];
          v = dv2b{gr * v.x, gr * v.y};  // (outside rows: 0 either way)
        }
        ring[sl][c >> 2][c & 3] = v;
      }
    }
  };
  // this thread: row (x0 + xi, y0 + yi), column pair cp; a wave = 16 consecutive x rows
  const int xi = (wave & 1) * 16 + (lane >> 2), yi = wave >> 1, cp = lane & 3;
  const int x = x0 + xi, y = y0 + yi;
  const bool own = x < g.nx && y < g.ny;
  const int hrow = (yi + 1) * kCHX + xi + 1;
  const int cxy = (own ? box_cls1(y, g.ny) * 3 + box_cls1(x, g.nx) : 0);
  dv2b bb = {}, xo = {}, bn = {}, xn = {};
  auto fetch_cheb = [&](int zz, dv2b &b2, dv2b &x2) {
    if (plain || !own || zz >= z1) return;
    const i64 r = (i64)x + (i64)g.nx * y + (i64)g.P * zz;
    if constexpr (first)
      b2 = Bb[r * 4 + cp];  // (the plane just went through the ring: an L2 hit)
    else
      b2 = __builtin_nontemporal_load(Bb + r * 4 + cp);
    if (EPI == kBoxCheb && Ob) x2 = __builtin_nontemporal_load(Ob + r * 4 + cp);  // (null: x_{k-1} = 0)
  };
  fetch(z0 - 1);
  store(z0 - 1);
  fetch(z0);
  store(z0);
  fetch(z0 + 1);
  store(z0 + 1);
  fetch_cheb(z0, bb, xo);
  for (int z = z0; z < z1; ++z)
  {
    __syncthreads();  // ring holds planes z - 1, z, z + 1 (and the class table)
    fetch_cheb(z + 1, bn, xn);
    fetch(z + 2);
    const int gz = g.gz0 + z;  // (the global plane: a slab's rows take their grid classes)
    const int cls = (gz == 0 ? 0 : (gz == g.gnz - 1 ? 2 : 1)) * 9 + cxy;
    const unsigned m = own ? cm[cls] : 0u;
    // ring slots of planes z - 1, z, z + 1 (scalar)
    const int s0 = z % 3, sm = s0 == 0 ? 2 : s0 - 1, sp = s0 == 2 ? 0 : s0 + 1;
    dv2b acc = {0.0, 0.0};
    // stored entry k: a * x, summed in ascending offset order; an offset the row does not store is
    // dropped by a select (the class entry is 0 there, but 0 * inf would not be)
    auto add = [&](bool on, double a, dv2b xv) {
      if (plain)
      {
        const double s0v = acc.x + a * xv.x, s1v = acc.y + a * xv.y;
        acc.x = on ? s0v : acc.x;
        acc.y = on ? s1v : acc.y;
      }
      else
      {
        const double f0 = __builtin_fma(a, xv.x, acc.x), f1 = __builtin_fma(a, xv.y, acc.y);
        acc.x = on ? f0 : acc.x;
        acc.y = on ? f1 : acc.y;
      }
    };
    if constexpr (SHAPE != 0)
    {
      // compile-time stencil on a geometric mask (box_geomask): every offset of the shape is summed,
      // in ascending order; one the row does not store has a zero class entry and points at a zero
      // halo row, and +0 added to a sum that starts at +0 changes nothing -- the same sums as with
      // the mask.  LDS offsets are immediates off three per-plane slot bases.
      constexpr BoxShapeTab T = box_shape_tab(SHAPE);
      constexpr int kGroup = cheb ? 2 : 4;  // (the Chebyshev step holds 4 more vectors)
      // ring index (dv2b units) of the (-1, -1) neighbour in the three slots, made opaque to the
      // compiler: otherwise it hoists base + offset for every offset out of the plane loop (one
      // live VGPR per offset and slot, ~110 VGPRs: one workgroup per CU instead of two)
      constexpr int kSlot = kCHY * kCHX * 4;
      const dv2b *r0 = &ring[0][0][0];
      int pz[3];
      pz[0] = sm * kSlot + (hrow - kCHX - 1) * 4 + cp;
      pz[1] = s0 * kSlot + (hrow - kCHX - 1) * 4 + cp;
      pz[2] = sp * kSlot + (hrow - kCHX - 1) * 4 + cp;
      asm volatile("" : "+v"(pz[0]), "+v"(pz[1]), "+v"(pz[2]));
      const double *crow = &ct[cls][0];
#pragma unroll
      for (int k = 0; k < T.nd; ++k)
      {
        add(true, crow[k], r0[pz[T.dz[k] + 1] + ((T.dy[k] + 1) * kCHX + T.dx[k] + 1) * 4]);
        // the next group's LDS reads wait for this group's sums (kGroup reads in flight; without it
        // the scheduler issues all of them at once and needs ~77 VGPRs: one workgroup per CU)
        if ((k + 1) % kGroup == 0 && k + 1 < T.nd)
          asm volatile("" : "+v"(pz[0]), "+v"(pz[1]), "+v"(pz[2]) : "v"(acc.x), "v"(acc.y));
      }
    }
    else
    {
#pragma unroll 4
      for (int k = 0; k < g.nd; ++k)
      {
        if (!((m >> k) & 1u)) continue;
        const int sl = g.dz[k] < 0 ? sm : (g.dz[k] > 0 ? sp : s0);
        add(true, ct[cls][k], ring[sl][hrow + g.dxy[k]][cp]);
      }
    }
    if (own)
    {
      const i64 r = (i64)x + (i64)g.nx * y + (i64)g.P * z;
      if (plain)
      {
        __builtin_nontemporal_store(acc, Yb + r * 4 + cp);
        if constexpr (dot)
        {
          const dv2b xc = ring[s0][hrow][cp];  // the row's own X (plane z)
          dsum.x += xc.x * acc.x;
          dsum.y += xc.y * acc.y;
        }
      }
      else if (EPI == kBoxResid || EPI == kBoxResidCopy || EPI == kBoxResidAcc)
      {
        __builtin_nontemporal_store(dv2b{bb.x - acc.x, bb.y - acc.y}, Yb + r * 4 + cp);
        if constexpr (EPI != kBoxResid)
        {
          dv2b *Xs = const_cast<dv2b *>(Ob);  // (the row's own: read-modify-write by this thread only)
          dv2b v = ring[s0][hrow][cp];
          if constexpr (EPI == kBoxResidAcc)
          {
            const dv2b xa = Xs[r * 4 + cp];
            v = dv2b{xa.x + v.x, xa.y + v.y};
          }
          Xs[r * 4 + cp] = v;
        }
      }
      else
      {
        const dv2b xc = ring[s0][hrow][cp];
        const double gd = gamma * ct[cls][kCStride - 1];
        if constexpr (EPI == kBoxChebSecond) xo = dv2b{gd * bb.x, gd * bb.y};  // x_1 (k_cheb_init's product)
        double o0 = omega * (xc.x + gd * (bb.x - acc.x) - xo.x) + xo.x;
        double o1 = omega * (xc.y + gd * (bb.y - acc.y) - xo.y) + xo.y;
        if constexpr (EPI == kBoxChebFirstAdd)
        {
          const dv2b yv = Yb[r * 4 + cp];  // (the row's own: read-modify-write by this thread only)
          o0 = yv.x + o0;
          o1 = yv.y + o1;
        }
        __builtin_nontemporal_store(dv2b{o0, o1}, Yb + r * 4 + cp);
      }
    }
    if constexpr (EPI == kBoxStoreDotGram) quad_gram_add(gacc, own ? acc.x : 0.0, own ? acc.y : 0.0);  // (a quad = a row)
    __syncthreads();  // everyone is done with slot (z - 1) mod 3
    store(z + 2);
    bb = bn;
    xo = xn;
  }
  if constexpr (EPI == kBoxStoreDotGram)
  {
    // the 8 dots and the 64 Gram slots: workgroup sums (fixed order) into LDS, then the two-level
    // deterministic grid sum (grid.y = 1: one column block)
    __shared__ double gv[72], gt[72];
    quad_gram_block<kCThreads>(gacc, dsum.x, dsum.y, reinterpret_cast<double *>(&ring[0][0][0]), gv);
    if (grid_sum2<kCThreads>(gv, 72, bd.part, bd.part + (size_t)gridDim.x * 72, bd.tick, blockIdx.x, gridDim.x, gt))
    {
      if (tid < 64) bd.gram[tid] = gt[tid];
      if (tid < 8) bd.dp[tid] = gt[64 + tid];
      if (tid == 0 && bd.zero_word) *bd.zero_word = 0u;
    }
  }
  if constexpr (EPI == kBoxStoreDot)
  {
    // every thread of every workgroup arrives here (no early exit above); the 8 column sums of this
    // column block in workgroup order (grid_sum_n: fixed order, independent of dispatch)
    __shared__ double tot[8];
    double v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
      v[2 * q] = q == cp ? dsum.x : 0.0;
      v[2 * q + 1] = q == cp ? dsum.y : 0.0;
    }
    if (grid_sum_n<8, kCThreads>(v, bd.part + (size_t)blockIdx.y * gridDim.x * 8, bd.tick + (size_t)blockIdx.y * kTicketStride,
                                 tot, blockIdx.x, gridDim.x))
    {
      if (tid < 8) bd.dp[blockIdx.y * 8 + tid] = tot[tid];
    }
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
  if (A.box_ctab)
  {
    (void)hipStreamSynchronize(A.ctx->stream);
    (void)hipFree(A.box_ctab);
    (void)hipFree(A.box_cmask);
  }
  A.box_ctab = nullptr;
  A.box_cmask = nullptr;
  A.box_geomask = false;
  A.box_state = 0;
}

// Row classes of a box image (k_boxc_mv8): the 27 representatives' entries and masks to the host,
// 1 / a_rr per class, then every row checked bitwise against its class on the device; on success
// A.box_ctab / box_cmask are set.  Needs a stored diagonal in every class.
// A rank's slab (planes z0 .. z0 + nz - 1 of nzg): classes by global plane; a z class the slab does not
// hold (first / last plane of the grid) takes the interior representative (never read).
static void box_classes(eig_mat_s &A, i64 nx, i64 ny, i64 nz, i64 z0, i64 nzg)
{
  if (nx < 3 || ny < 3 || nz < 3 || A.sym_nd >= kCStride || (A.kflags & EIG_MAT_NO_CLASS)) return;
  int k0 = -1;
  for (int k = 0; k < A.sym_nd; ++k)
    if (A.sym_off[k] == 0) k0 = k;
  if (k0 < 0) return;
  hipStream_t s = A.ctx->stream;
  const i64 n = A.nb_rows;
  std::vector<i64> rep(kBoxClasses);
  auto pos = [](int c, i64 nv) { return c == 0 ? (i64)0 : (c == 1 ? (i64)1 : nv - 1); };
  // local plane of z class c (1: local plane 1, global interior since nz >= 3 and the slab's planes
  // are whole): 0 / nz - 1 only where the slab holds the grid's first / last plane
  auto zpos = [&](int c) { return c == 0 ? (z0 == 0 ? (i64)0 : (i64)1) : (c == 2 ? (z0 + nz == nzg ? nz - 1 : (i64)1) : (i64)1); };
  for (int c = 0; c < kBoxClasses; ++c)
    rep[c] = pos(c % 3, nx) + nx * pos((c / 3) % 3, ny) + nx * ny * zpos(c / 9);
  DevBuf drep(kBoxClasses * sizeof(i64)), dout((size_t)kBoxClasses * (kCStride + 1) * sizeof(double));
  EIG_HIP(hipMemcpyAsync(drep.p, rep.data(), kBoxClasses * sizeof(i64), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_boxc_gather, dim3(kBoxClasses), dim3(64), 0, s, n, A.sym_nd, (const double *)A.box_val,
                     (const void *)A.sym_mask, A.sym_mask_bytes, (const i64 *)drep.p, dout.d());
  std::vector<double> h((size_t)kBoxClasses * (kCStride + 1));
  EIG_HIP(hipMemcpyAsync(h.data(), dout.p, h.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  EIG_HIP(hipStreamSynchronize(s));
  std::vector<double> ctab((size_t)kBoxClasses * kCStride, 0.0);
  std::vector<unsigned> cmask(kBoxClasses);
  for (int c = 0; c < kBoxClasses; ++c)
  {
    const unsigned m = (unsigned)h[(size_t)c * (kCStride + 1) + kCStride];
    cmask[c] = m;
    if (!((m >> k0) & 1u)) return;
    for (int k = 0; k < A.sym_nd; ++k)
      if ((m >> k) & 1u) ctab[(size_t)c * kCStride + k] = h[(size_t)c * (kCStride + 1) + k];
    // the same IEEE division k_diag_inv performs on the row's diagonal
    ctab[(size_t)c * kCStride + kCStride - 1] = 1.0 / ctab[(size_t)c * kCStride + k0];
  }
  double *dct = nullptr;
  unsigned *dcm = nullptr;
  EIG_HIP(hipMalloc(&dct, ctab.size() * sizeof(double)));
  EIG_HIP(hipMalloc(&dcm, (kBoxClasses + 1) * sizeof(unsigned)));
  EIG_HIP(hipMemcpyAsync(dct, ctab.data(), ctab.size() * sizeof(double), hipMemcpyHostToDevice, s));
  EIG_HIP(hipMemcpyAsync(dcm, cmask.data(), kBoxClasses * sizeof(unsigned), hipMemcpyHostToDevice, s));
  unsigned *bad = dcm + kBoxClasses;
  EIG_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned), s));
  hipLaunchKernelGGL(k_boxc_check, dim3(2048), dim3(256), 0, s, n, (int)nx, (int)ny, (int)z0, (int)nzg, A.sym_nd,
                     (const double *)A.box_val, (const void *)A.sym_mask, A.sym_mask_bytes, dct, dcm, bad);
  unsigned hb = 1;
  EIG_HIP(hipMemcpyAsync(&hb, bad, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  EIG_HIP(hipStreamSynchronize(s));
  if (hb)
  {
    (void)hipFree(dct);
    (void)hipFree(dcm);
    return;
  }
  A.box_ctab = dct;
  A.box_cmask = dcm;
}

// Box-stencil geometry of a band image and its device box image (built on first use and cached on
// the matrix); false when the matrix does not qualify.
bool box_prepare(const eig_mat_s &Ac)
{
  eig_mat_s &A = const_cast<eig_mat_s &>(Ac);
  if (A.box_state != 0) return A.box_state > 0;
  A.box_state = -1;
  if (!A.sym_val || A.br != 1 || A.bc != 1 || (A.kflags & EIG_MAT_NO_MARCH)) return false;
  // a rank of a distributed context: its slab of whole planes (checked below, once the plane size is
  // known); one rank: the whole grid in its own window
  const bool slab = A.ctx->distributed();
  if (A.sym_nd > kBoxClassMaxNd || (!slab && (A.nb_rows != A.nb_rows_global || A.window != A.nb_rows))) return false;
  // Grid from the offsets: Nx is the smallest offset > 1 (+1 when the stencil has the (0, +1, -1)
  // neighbour, d = Nx - 1), P = Nx Ny the smallest offset past Nx + 1 (+ 0, 1, Nx - 1, Nx or Nx + 1
  // for the neighbours with dz = 1 and dy, dx < 0 .. dy = 1); every offset must be a P + b Nx + c
  // with a, b, c in {-1, 0, 1}
  i64 s1 = 0;
  for (int k = 0; k < A.sym_nd; ++k)
    if (A.sym_off[k] > 1 && (s1 == 0 || A.sym_off[k] < s1)) s1 = A.sym_off[k];
  std::vector<i32> dx(A.sym_nd), dy(A.sym_nd), dz(A.sym_nd);
  auto decompose = [&](i64 nxc, i64 Pc) {
    for (int k = 0; k < A.sym_nd; ++k)
    {
      const i64 d = A.sym_off[k];
      bool found = false;
      for (int a = -1; a <= 1 && !found; ++a)
        for (int b = -1; b <= 1 && !found; ++b)
          for (int c = -1; c <= 1 && !found; ++c)
            if (a * Pc + b * nxc + c == d)
            {
              dz[k] = a, dy[k] = b, dx[k] = c;
              found = true;
            }
      if (!found) return false;
    }
    return true;
  };
  i64 nx = 0, P = 0;
  for (i64 nxc : {s1, s1 + 1})
  {
    if (nxc < kBoxTX || P) continue;
    i64 t = 0;
    for (int k = 0; k < A.sym_nd; ++k)
      if (A.sym_off[k] > nxc + 1 && (t == 0 || A.sym_off[k] < t)) t = A.sym_off[k];
    if (t == 0) continue;
    for (i64 Pc : {t, t + 1, t + nxc - 1, t + nxc, t + nxc + 1})
      if (!P && Pc % nxc == 0 && A.nb_rows % Pc == 0 && Pc / nxc >= kBoxTY && decompose(nxc, Pc))
      {
        nx = nxc;
        P = Pc;
      }
  }
  if (!P) return false;
  const i64 ny = P / nx, nz = A.nb_rows / P;
  if (nz < 3 || nz > (1 << 24)) return false;
  // slab: whole planes, the window = at most one ghost plane below and above the owned ones in global
  // order (the box kernel reads planes -1 and nz from there; the band arrays are window-indexed)
  int glo = 0, ghi = 0;
  if (slab)
  {
    const i64 tail = A.window - A.own_offset - A.nb_rows;
    if (A.row_begin % P != 0 || A.nb_rows_global % P != 0 || A.own_offset % P != 0 || tail < 0 || tail % P != 0)
      return false;
    glo = (int)(A.own_offset / P);
    ghi = (int)(tail / P);
    if (glo > 1 || ghi > 1 || A.nb_rows_global / P > (1 << 24)) return false;
  }
  const int z0 = slab ? (int)(A.row_begin / P) : 0, nzg = slab ? (int)(A.nb_rows_global / P) : (int)nz;
  decompose(nx, P);
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
    hipLaunchKernelGGL(k_box_check, dim3(2048), dim3(256), 0, s, n, (int)nx, (int)ny, nzg, z0, A.sym_nd, dm,
                       dm + A.sym_nd, dm + 2 * A.sym_nd, (const void *)A.sym_mask, A.sym_mask_bytes, bad);
    unsigned hb = 0;
    EIG_HIP(hipMemcpyAsync(&hb, bad, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    EIG_HIP(hipStreamSynchronize(s));
    if (hb & 1u) return false;
    A.box_geomask = !(hb & 2u);
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
    hipLaunchKernelGGL(k_box_image, dim3(2048), dim3(256), 0, s, n, A.sym_ld, (i64)A.own_offset, A.sym_nd, o, o + A.sym_nd,
                       (const double *)A.sym_val, (const void *)A.sym_mask, A.sym_mask_bytes, val);
    EIG_HIP(hipStreamSynchronize(s));
    A.box_val = val;
  }
  box_classes(A, nx, ny, nz, z0, nzg);
  A.box_nx = (int)nx;
  A.box_ny = (int)ny;
  A.box_nz = (int)nz;
  A.box_glo = glo;
  A.box_ghi = ghi;
  for (int k = 0; k < A.sym_nd; ++k)
  {
    A.box_dz[k] = dz[k];
    A.box_dxy[k] = dy[k] * kBoxHX + dx[k];
    A.box_dx[k] = dx[k];
    A.box_dy[k] = dy[k];
  }
  if (A.box_ctab || A.sym_nd > kBoxMaxNd)
  {
    // the class kernels read no box image; past kBoxMaxNd offsets there is no box-image kernel
    EIG_HIP(hipFree(A.box_val));
    A.box_val = nullptr;
    if (!A.box_ctab) return false;  // (box_state stays -1)
  }
  else
    A.device_bytes += (i64)A.sym_nd * n * (i64)sizeof(double);
  A.box_state = 1;
  return true;
}

// Columns per workgroup of the box-image kernels: eig_mat_tune(EIG_TUNE_BOX_COLS), else 32.
int box_cols(const eig_mat_s &A) { return A.tune_box_cols == 16 ? 16 : 32; }

// Y = A X (EPI store) or the Chebyshev step into Xold (EPI cheb) for m % 32 == 0 columns on the box
// kernel; false when the matrix has no box geometry (the caller takes the band march).
static bool launch_box(const eig_mat_s &A, i64 m, const double *X, double *Y, const double *Xold, const double *Bv,
                       const double *dinv, double omega, double gamma, int epi, hipStream_t s, BoxDot bd = {})
{
  if (m <= 0 || m % 8 != 0 || !box_prepare(A)) return false;
  if (epi >= kBoxChebFirst && !A.box_ctab) return false;  // (row-class only)
  if ((epi == kBoxStoreDot || epi == kBoxStoreDotGram) && !A.box_ctab) return false;
  if (epi == kBoxStoreDotGram && m != 8) return false;
  // a rank's slab (A.ctx->distributed()): the product and the Chebyshev step only, the window's ghost
  // planes as planes -1 / nz, every window-layout vector from its owned rows (own_offset)
  const bool slab = A.ctx->distributed();
  if (slab && epi != kBoxStore && epi != kBoxCheb) return false;
  const i64 own8 = slab ? A.own_offset * 8 : 0;
  if (A.box_ctab)
  {
    // row-class kernels: one launch, blockIdx.y = column block.  z runs of about 32 planes (a run
    // re-reads two halo planes, so shorter runs cost bytes; longer ones balance worse), but at least
    // one workgroup per CU on small grids and no run shorter than 8 planes (EIG_TUNE_BOX_SEGS sweeps,
    // profiles/r03aw_box_segs.jsonl: 128^3 m = 8 55.3 -> 46.8 us, 256^3 m = 32 1554 -> 1500 us)
    BoxGeom g;
    g.nx = A.box_nx;
    g.ny = A.box_ny;
    g.nz = A.box_nz;
    g.zlo = A.box_glo;
    g.zhi = A.box_ghi;
    g.gz0 = slab ? (int)(A.row_begin / ((i64)A.box_nx * A.box_ny)) : 0;
    g.gnz = slab ? (int)(A.nb_rows_global / ((i64)A.box_nx * A.box_ny)) : A.box_nz;
    g.P = g.nx * g.ny;
    g.ntx = (g.nx + kCTX - 1) / kCTX;
    g.nty = (g.ny + kCTY - 1) / kCTY;
    const i64 per_seg = (i64)g.ntx * g.nty * (m / 8);
    const i64 fill = std::min<i64>(g.nz / 8, (A.ctx->num_cu + per_seg - 1) / per_seg);
    g.nseg = (int)std::max<i64>({1, (g.nz + 31) / 32, fill});
    if (A.tune_box_segs > 0) g.nseg = std::min(g.nz, A.tune_box_segs);
    g.nd = A.sym_nd;
    for (int k = 0; k < 27; ++k)
    {
      g.dz[k] = k < A.sym_nd ? A.box_dz[k] : 0;
      g.dxy[k] = k < A.sym_nd ? A.box_dy[k] * kCHX + A.box_dx[k] : 0;
    }
    const dim3 grid((unsigned)(g.ntx * g.nty * g.nseg), (unsigned)(m / 8));
    // kBoxStoreDot: one ticket and grid.x x 8 partials per column block
    if (epi == kBoxStoreDot && ((i64)grid.x * 8 * grid.y > (i64)kMaxRedBlocks * kMaxRedVals || grid.y > kNumTickets))
      return false;
    if (epi == kBoxStoreDotGram && ((i64)grid.x * 72 + 8 * 72 > (i64)kMaxRedBlocks * kMaxRedVals || grid.y != 1))
      return false;
    // the stencil's shape: compile-time kernels for the 7-point and the Kuhn 15-point stencils,
    // a runtime offset loop for any other
    unsigned shape = 0;
    for (int k = 0; k < A.sym_nd; ++k)
      shape |= 1u << ((A.box_dz[k] + 1) * 9 + (A.box_dy[k] + 1) * 3 + (A.box_dx[k] + 1));
    auto go = [&](auto shape_tag) {
      constexpr unsigned S = decltype(shape_tag)::value;
      const double *ct = (const double *)A.box_ctab;
      const unsigned *cm = (const unsigned *)A.box_cmask;
      if (slab)  // (kBoxStore / kBoxCheb only, from the owned rows)
      {
        if (epi == kBoxCheb)
          hipLaunchKernelGGL((k_boxc_mv8<kBoxCheb, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X + own8,
                             Y + own8, Xold ? Xold + own8 : nullptr, Bv + own8, omega, gamma, bd);
        else
          hipLaunchKernelGGL((k_boxc_mv8<kBoxStore, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X + own8,
                             Y + own8, (const double *)nullptr, (const double *)nullptr, 0.0, 0.0, bd);
        return;
      }
      if (epi == kBoxCheb)
        hipLaunchKernelGGL((k_boxc_mv8<kBoxCheb, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y, Xold,
                           Bv, omega, gamma, bd);
      else if (epi == kBoxChebFirst)
        hipLaunchKernelGGL((k_boxc_mv8<kBoxChebFirst, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y,
                           (const double *)nullptr, Bv, omega, gamma, bd);
      else if (epi == kBoxChebFirstAdd)
        hipLaunchKernelGGL((k_boxc_mv8<kBoxChebFirstAdd, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y,
                           (const double *)nullptr, Bv, omega, gamma, bd);
      else if (epi == kBoxResidCopy)
        hipLaunchKernelGGL((k_boxc_mv8<kBoxResidCopy, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y,
                           Xold, Bv, 0.0, 0.0, bd);
      else if (epi == kBoxResidAcc)
        hipLaunchKernelGGL((k_boxc_mv8<kBoxResidAcc, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y,
                           Xold, Bv, 0.0, 0.0, bd);
      else if (epi == kBoxChebSecond)
        hipLaunchKernelGGL((k_boxc_mv8<kBoxChebSecond, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y,
                           (const double *)nullptr, Bv, omega, gamma, bd);
      else if (epi == kBoxResid)
        hipLaunchKernelGGL((k_boxc_mv8<kBoxResid, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y,
                           (const double *)nullptr, Bv, 0.0, 0.0, bd);
      else if (epi == kBoxStoreDot)
        hipLaunchKernelGGL((k_boxc_mv8<kBoxStoreDot, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y,
                           (const double *)nullptr, (const double *)nullptr, 0.0, 0.0, bd);
      else if (epi == kBoxStoreDotGram)
        hipLaunchKernelGGL((k_boxc_mv8<kBoxStoreDotGram, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y,
                           (const double *)nullptr, (const double *)nullptr, 0.0, 0.0, bd);
      else
        hipLaunchKernelGGL((k_boxc_mv8<kBoxStore, S>), grid, dim3(kCThreads), 0, s, g, A.window, ct, cm, X, Y,
                           (const double *)nullptr, (const double *)nullptr, 0.0, 0.0, bd);
    };
    // (the image's offsets ascend, i.e. run in the shape's bit order: box_prepare builds them so)
    if (A.box_geomask && shape == kShape7 && A.sym_nd == 7)
      go(std::integral_constant<unsigned, kShape7>{});
    else if (A.box_geomask && shape == kShapeKuhn && A.sym_nd == 15)
      go(std::integral_constant<unsigned, kShapeKuhn>{});
    else if (A.box_geomask && shape == kShape27 && A.sym_nd == 27)
      go(std::integral_constant<unsigned, kShape27>{});
    else
      go(std::integral_constant<unsigned, 0u>{});
    EIG_HIP(hipGetLastError());
    return true;
  }
  if (m % 32 != 0) return false;  // the box-image kernel takes 32 columns per pass
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
  if (A.tune_box_segs > 0) g.nseg = std::min(g.nz, A.tune_box_segs);
  g.nd = A.sym_nd;
  g.xmap = A.tune_box_map == 1 && (tiles * g.nseg) % 8 == 0;
  g.zlo = A.box_glo;
  g.zhi = A.box_ghi;
  for (int k = 0; k < 27; ++k)
  {
    g.dz[k] = k < A.sym_nd ? A.box_dz[k] : 0;
    g.dxy[k] = k < A.sym_nd ? A.box_dxy[k] : 0;
  }
  const uint32_t *m32 = A.sym_mask_bytes == 4 ? static_cast<const uint32_t *>(A.sym_mask) : nullptr;
  const uint8_t *m8 = A.sym_mask_bytes == 1 ? static_cast<const uint8_t *>(A.sym_mask) : nullptr;
  const i64 ld = A.window;
  unsigned shape = 0;
  for (int k = 0; k < A.sym_nd; ++k)
    shape |= 1u << ((A.box_dz[k] + 1) * 9 + (A.box_dy[k] + 1) * 3 + (A.box_dx[k] + 1));
  // EIG_TUNE_BOX_COLS: 16 = the push-order kernel (two 16-column workgroups per tile), 32 = k_box_mv32
  const bool push = box_cols(A) == 16 && !slab;
  auto go = [&](auto shape_tag) {
    constexpr unsigned S = decltype(shape_tag)::value;
    for (i64 c0 = 0; c0 < m; c0 += 32)
    {
      // 4 column blocks of ld rows x 8, from the owned rows (one rank: own_offset 0)
      const i64 off = c0 * ld + own8;
      if (push)
      {
        const int items = tiles * g.nseg;
        const dim3 pgrid((unsigned)(16 * ((items + 7) / 8)));
        if (epi == kBoxCheb)
          hipLaunchKernelGGL((k_box_mv16p<kBoxCheb, S>), pgrid, dim3(kPThreads), 0, s, g, ld, items,
                             (const double *)A.box_val, m32, m8, X + off, Y + off, Xold ? Xold + off : nullptr,
                             Bv + off, dinv, omega, gamma);
        else if (epi == kBoxResid)
          hipLaunchKernelGGL((k_box_mv16p<kBoxResid, S>), pgrid, dim3(kPThreads), 0, s, g, ld, items,
                             (const double *)A.box_val, m32, m8, X + off, Y + off, (const double *)nullptr,
                             Bv + off, (const double *)nullptr, 0.0, 0.0);
        else
          hipLaunchKernelGGL((k_box_mv16p<kBoxStore, S>), pgrid, dim3(kPThreads), 0, s, g, ld, items,
                             (const double *)A.box_val, m32, m8, X + off, Y + off, (const double *)nullptr,
                             (const double *)nullptr, (const double *)nullptr, 0.0, 0.0);
        continue;
      }
      const dim3 grid((unsigned)(tiles * g.nseg));
      if (epi == kBoxCheb)
        hipLaunchKernelGGL((k_box_mv32<kBoxCheb, S>), grid, dim3(kBoxThreads), 0, s, g, ld, (const double *)A.box_val,
                           m32, m8, X + off, Y + off, Xold ? Xold + off : nullptr, Bv + off, dinv, omega, gamma);
      else if (epi == kBoxResid)
        hipLaunchKernelGGL((k_box_mv32<kBoxResid, S>), grid, dim3(kBoxThreads), 0, s, g, ld, (const double *)A.box_val,
                           m32, m8, X + off, Y + off, (const double *)nullptr, Bv + off, (const double *)nullptr, 0.0,
                           0.0);
      else
        hipLaunchKernelGGL((k_box_mv32<kBoxStore, S>), grid, dim3(kBoxThreads), 0, s, g, ld, (const double *)A.box_val,
                           m32, m8, X + off, Y + off, (const double *)nullptr, (const double *)nullptr,
                           (const double *)nullptr, 0.0, 0.0);
    }
  };
  if (A.box_geomask && shape == kShape7 && A.sym_nd == 7)
    go(std::integral_constant<unsigned, kShape7>{});
  else if (A.box_geomask && shape == kShapeKuhn && A.sym_nd == 15)
    go(std::integral_constant<unsigned, kShapeKuhn>{});
  else
    go(std::integral_constant<unsigned, 0u>{});
  EIG_HIP(hipGetLastError());
  return true;
}

bool launch_box_spmm(const eig_mat_s &A, i64 m, const double *X, double *Y, hipStream_t s)
{
  return launch_box(A, m, X, Y, nullptr, nullptr, nullptr, 0.0, 0.0, kBoxStore, s);
}

// Y = A X and dp[j] = X_j . Y_j (8 per column block) in one launch: the row-class kernel only
// (false otherwise: the caller runs the product and dot_diag separately).  red: the context's
// reduction workspace, its tickets 0 .. m / 8 - 1.
bool launch_box_spmm_dot(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, ReduceWS red,
                         hipStream_t s)
{
  if (m <= 0 || m % 8 != 0 || !box_prepare(A) || !A.box_ctab) return false;
  BoxDot bd;
  bd.dp = dp;
  bd.part = red.partials;
  bd.tick = red.ticket(0);
  return launch_box(A, m, X, Y, nullptr, nullptr, nullptr, 0.0, 0.0, kBoxStoreDot, s, bd);
}

// Y = A X, dp (8 dots) and gram (the 8 x 8 window Gram of Y) in one launch, m = 8: the row-class
// kernel only (false otherwise).  Uses the reduction workspace's partials (grid.x x 72 + 8 x 72) and
// ticket 0.
bool launch_box_spmm_dot_gram(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, double *gram,
                              ReduceWS red, hipStream_t s, unsigned *zero_word)
{
  if (m != 8 || !box_prepare(A) || !A.box_ctab) return false;
  BoxDot bd;
  bd.dp = dp;
  bd.part = red.partials;
  bd.tick = red.ticket(0);
  bd.gram = gram;
  bd.zero_word = zero_word;
  return launch_box(A, m, X, Y, nullptr, nullptr, nullptr, 0.0, 0.0, kBoxStoreDotGram, s, bd);
}

bool launch_box_resid(const eig_mat_s &A, i64 m, const double *X, const double *B, double *R, hipStream_t s)
{
  return launch_box(A, m, X, R, nullptr, B, nullptr, 0.0, 0.0, kBoxResid, s);
}

// R = B - A E and Xacc = E (copy) or Xacc += E (row-class image only; false otherwise).
bool launch_box_resid_acc(const eig_mat_s &A, i64 m, const double *E, const double *B, double *R, double *Xacc,
                          bool copy, hipStream_t s)
{
  return launch_box(A, m, E, R, Xacc, B, nullptr, 0.0, 0.0, copy ? kBoxResidCopy : kBoxResidAcc, s);
}

bool launch_box_cheb(const eig_mat_s &M, i64 m, const double *Xk, double *Xold, const double *B, const double *dinv,
                     double omega, double gamma, hipStream_t s, double *Xnew)
{
  EIG_CHECK(Xold || Xnew, EIG_ERR_ARG, "box Chebyshev step: x_{k-1} = 0 needs a separate output buffer");
  return launch_box(M, m, Xk, Xnew ? Xnew : Xold, Xold, B, dinv, omega, gamma, kBoxCheb, s);
}

// The first Chebyshev step from x_0 = 0, x_1 = gamma D^-1 B never stored: Y = x_2 straight from B
// (row-class image only; false otherwise -- the caller then runs k_cheb_init and launch_box_cheb).
bool launch_box_cheb_first(const eig_mat_s &M, i64 m, const double *B, double omega, double gamma, double *Y,
                           hipStream_t s)
{
  return launch_box(M, m, B, Y, nullptr, B, nullptr, omega, gamma, kBoxChebFirst, s);
}

// Y += x_2 of the degree-2 solve from B (the same x_2 as launch_box_cheb_first, added in place).
bool launch_box_cheb_first_add(const eig_mat_s &M, i64 m, const double *B, double omega, double gamma, double *Y,
                               hipStream_t s)
{
  return launch_box(M, m, B, Y, nullptr, B, nullptr, omega, gamma, kBoxChebFirstAdd, s);
}

// The second step, x_3 from x_2 = X2 and x_1 = gamma D^-1 B (formed per row, not read): Y = x_3.
bool launch_box_cheb_second(const eig_mat_s &M, i64 m, const double *X2, const double *B, double omega, double gamma,
                            double *Y, hipStream_t s)
{
  return launch_box(M, m, X2, Y, nullptr, B, nullptr, omega, gamma, kBoxChebSecond, s);
}

}  // namespace eigmi
