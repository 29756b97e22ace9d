// k_spmv.hip -- sparse matrix x vector on the SELL-C image (gfx950).
//
// Replaces BCRSMatrix::mv (dune-istl; called at arpack_geneo_wrapper.hh:275 through multMvB)
// and the b = 1 product matmul_sparse_tallskinny_naive (kernels_cpp.hh:596-621).
//
// Layout (internal.h): slices of C = 64 R block rows, one wavefront per slice; lane l owns the R
// adjacent rows l R .. l R + R - 1.  Entry k of slice row r sits at slice_ptr[s] + k C + r
// (column-major over the slice), so the k-th (value, column) of a lane's R rows is one R-wide
// vector load and a wave-instruction reads 512 R bytes contiguous.  Every row keeps its stored
// (ascending-column) order and accumulates from 0.0, mul then add (-ffp-contract=off): y is
// bitwise BCRSMatrix::mv.  Padding entries carry column -1 and are skipped.
//
// Work split: a workgroup of 4 waves walks a CONTIGUOUS chunk of slices (waves interleaved), so
// rows that share x lines stay in one CU / one XCD's L2; 2048 workgroups (8 per CU) are resident.
#include "internal.h"
#include "reduce_dev.h"
#include "xch_dev.h"

namespace eigmi {

constexpr int kWaves = kStreamThreads / 64;

template <int R>
struct Vec;
template <>
struct Vec<1> {
  typedef double d;
  typedef i32 i;
};
template <>
struct Vec<2> {
  typedef double d __attribute__((ext_vector_type(2)));
  typedef i32 i __attribute__((ext_vector_type(2)));
};
template <>
struct Vec<4> {
  typedef double d __attribute__((ext_vector_type(4)));
  typedef i32 i __attribute__((ext_vector_type(4)));
};

template <int R>
__device__ __forceinline__ double lane_get(const typename Vec<R>::d &v, int q)
{
  if constexpr (R == 1) return v;
  else return v[q];
}
template <int R>
__device__ __forceinline__ i32 lane_geti(const typename Vec<R>::i &v, int q)
{
  if constexpr (R == 1) return v;
  else return v[q];
}

// XCD-aware work-item order for the plane marches: workgroups are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH "Workgroup dispatch"), so workgroup b takes logical item swizzled_block(b) and
// each XCD walks ONE contiguous eighth of the items -- a column's +-plane neighbours then sit in
// the same XCD's L2.  Bijective for any grid size (the first G % 8 groups hold one workgroup more).
// (The slice kernels take plain contiguous chunks: measured faster there -- the 256 MB MALL
// already serves their plane re-reads.)
__device__ __forceinline__ i64 swizzled_block()
{
  const int G = gridDim.x, bid = blockIdx.x;
  if (G < 16) return bid;
  const int q = G >> 3, r = G & 7, x = bid & 7, i = bid >> 3;
  return (i64)(x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

__device__ __forceinline__ void chunk_of(i64 count, i64 &b, i64 &e)
{
  const i64 G = gridDim.x;
  const i64 per = (count + G - 1) / G;
  b = (i64)blockIdx.x * per;
  e = b + per;
  if (e > count) e = count;
}

// Slice order of the row kernels: an XCD-aware sweep.  Workgroups are dealt round-robin over the 8
// XCDs, so XCD x takes the x-th eighth of the launch's slices and its workgroups sweep it together
// (grid-stride inside the eighth): the rows in flight on one XCD stay within a window of (its
// workgroups x 4) slices, and the gathered x rows of a banded (e.g. RCM-ordered) matrix are that
// window +- the bandwidth, which the XCD's L2 can hold.  Measured against contiguous per-workgroup
// chunks (256^3, tools/gpu_csr2.sh): scrambled + RCM SpMV 313 -> 305 us, K1 371 -> 359 us, fused
// step 671 -> 634 us; 7-point SELL image SpMV 268 -> 261 us.  Wave w of a workgroup takes slices
// it0, it0 + step, ... < end.  (Fewer than 8 workgroups: contiguous chunks.)
__device__ __forceinline__ void slice_sweep(i64 count, int wave, i64 &it0, i64 &end, i64 &step)
{
  const int G = gridDim.x;
  if (G < 8)
  {
    i64 b, e;
    chunk_of(count, b, e);
    it0 = b + wave;
    end = e;
    step = kWaves;
    return;
  }
  const int x = blockIdx.x & 7, i = blockIdx.x >> 3;
  const int Gx = (G - x + 7) >> 3;  // workgroups on XCD x
  it0 = count * x / 8 + (i64)i * kWaves + wave;
  end = count * (x + 1) / 8;
  step = (i64)Gx * kWaves;
}

// Gathered operand x[g]: a plain vector, or the fused Lanczos step's u_k = t_{k-1} - c u_{k-1}
// formed on the fly from the interleaved (t, u) pair vector (mul then sub, -ffp-contract=off:
// bitwise what the step stores for u_k).
struct XPlain {
  const double *__restrict__ x;
  typedef double raw;
  __device__ __forceinline__ const void *ptr() const { return x; }
  __device__ __forceinline__ double operator()(i64 g) const { return x[g]; }
  __device__ __forceinline__ raw load(i64 g) const { return x[g]; }
  __device__ __forceinline__ double val(raw v) const { return v; }
};
// (t, u) interleaved: one 16-B gather fetches both operands of an entry.
typedef double dpair __attribute__((ext_vector_type(2)));
struct XPair {
  const dpair *__restrict__ p;
  double c;
  typedef dpair raw;
  __device__ __forceinline__ const void *ptr() const { return p; }
  __device__ __forceinline__ double operator()(i64 g) const
  {
    const dpair v = p[g];
    return v.x - c * v.y;
  }
  __device__ __forceinline__ raw load(i64 g) const { return p[g]; }
  __device__ __forceinline__ double val(raw v) const { return v.x - c * v.y; }
};

// Whole-wave lane shifts on the DPP path (GFX9 wave_shr:1 / wave_shl:1, VALU moves, no LDS):
// lane_prev(v) in lane l is v of lane l - 1, lane_next(v) is v of lane l + 1 (lane 0 / 63 get 0 and
// are patched by the caller).
__device__ __forceinline__ int dpp_prev(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, true); }
__device__ __forceinline__ int dpp_next(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xf, 0xf, true); }
template <bool NEXT>
__device__ __forceinline__ double lane_shift(double v)
{
  const long long b = __double_as_longlong(v);
  const int lo = NEXT ? dpp_next((int)b) : dpp_prev((int)b);
  const int hi = NEXT ? dpp_next((int)(b >> 32)) : dpp_prev((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <bool NEXT>
__device__ __forceinline__ dpair lane_shift(dpair v)
{
  return dpair{lane_shift<NEXT>(v.x), lane_shift<NEXT>(v.y)};
}

// acc[q] = sum_k a[k][q] * x[c[k][q]] for the R rows of this lane, k ascending.  KC entries are
// prefetched per round (8 (value, column) loads in flight per lane for every R).
template <int R, class X>
__device__ __forceinline__ void rows_dot(const double *__restrict__ val, const i32 *__restrict__ col, const X &x,
                                         i64 base, int width, int lane, double (&acc)[R])
{
  constexpr int C = 64 * R;
  constexpr int KC = 8 / R;
  typedef typename Vec<R>::d dv;
  typedef typename Vec<R>::i iv;
#pragma unroll
  for (int q = 0; q < R; ++q) acc[q] = 0.0;
  // slice base pointers are wave-uniform (scalar); per-lane offsets are 32-bit
  const double *vs = val + base;
  const i32 *cs = col + base;
  for (int k0 = 0; k0 < width; k0 += KC)
  {
    dv a[KC];
    iv c[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k)
    {
      if (k0 + k < width)
      {
        const int idx = (k0 + k) * C + lane * R;
        c[k] = __builtin_nontemporal_load(reinterpret_cast<const iv *>(cs + idx));
        a[k] = __builtin_nontemporal_load(reinterpret_cast<const dv *>(vs + idx));
      }
      else
      {
        c[k] = (iv)(-1);
        a[k] = (dv)(0.0);
      }
    }
    double xv[KC][R];
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int q = 0; q < R; ++q)
      {
        const i32 cc = lane_geti<R>(c[k], q);
        xv[k][q] = (cc >= 0) ? x(cc) : 0.0;
      }
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int q = 0; q < R; ++q)
        if (lane_geti<R>(c[k], q) >= 0) acc[q] += lane_get<R>(a[k], q) * xv[k][q];
  }
}

// Stencil slice: entry k of row r is stored iff bit k of mask[r]; its column is r + own + delta_k
// (window-local).  Offsets ascend, so each row still accumulates in ascending-column order.
template <int R, class X>
__device__ __forceinline__ void rows_dot_stencil(const double *__restrict__ val, const i32 *__restrict__ delta,
                                                 const uint8_t *__restrict__ mask, const X &x,
                                                 i64 base, int width, int lane, i64 xrow0, i64 xlast,
                                                 double (&acc)[R])
{
  constexpr int C = 64 * R;
  constexpr int KC = 8 / R;
  typedef typename Vec<R>::d dv;
#pragma unroll
  for (int q = 0; q < R; ++q) acc[q] = 0.0;
  const double *vs = val + base;
  unsigned m[R];
#pragma unroll
  for (int q = 0; q < R; ++q) m[q] = mask[lane * R + q];
  for (int k0 = 0; k0 < width; k0 += KC)
  {
    dv a[KC];
    int dk[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k)
    {
      dk[k] = (k0 + k < width) ? delta[k0 + k] : 0;  // wave-uniform (scalar) loads
      a[k] = (k0 + k < width) ? __builtin_nontemporal_load(reinterpret_cast<const dv *>(vs + (k0 + k) * C + lane * R))
                              : (dv)(0.0);
    }
    // gather addresses do not depend on the mask (clamped into the window instead), so the x loads
    // issue together with the value loads; the mask only gates the accumulation below.
    double xv[KC][R];
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int q = 0; q < R; ++q)
      {
        i64 g = xrow0 + q + dk[k];
        g = g < 0 ? 0 : (g > xlast ? xlast : g);
        xv[k][q] = x(g);
      }
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int q = 0; q < R; ++q)
        if ((m[q] >> (k0 + k)) & 1u) acc[q] += lane_get<R>(a[k], q) * xv[k][q];
  }
}

// Symmetric band image (internal.h, eig_mat_s::sym_*): the stored diagonals of the upper triangle,
// one window-indexed array each; the entry at offset -d of row w is the entry at +d of row w - d.
struct SymImg {
  const double *val;  // nup arrays of ld doubles
  const void *mask;   // owned row r: bit k = row stores the entry at off[k] (u8 or u32 per row)
  i64 ld;
  int nd;                 // offsets, ascending = ISTL column order
  // near offsets {-1, 0, +1} (the lane-shift path): off[klo..khi) are the ones present; km1 / k0 /
  // kp1 their mask bits (-1 = absent), j0 / j1 the arrays of |d| = 0 / 1 (-1 = absent)
  int klo, khi, km1, k0, kp1, j0, j1;
  i32 off[kSymMaxOff];
  i32 dj[kSymMaxOff];     // array index of |off[k]|
};

// Offsets off[kb..ke) of row w: one coalesced value load each (at w for d >= 0, at w + d for d < 0:
// the mirrored upper entry, re-read from L2 / MALL after the rows d earlier streamed it) plus one
// coalesced gather; the mask gates the accumulation.
template <int KC, class X>
__device__ __forceinline__ void sym_span(const SymImg &S, int kb, int ke, unsigned m, i64 w, i64 wv, const X &x,
                                         i64 xl, double &acc)
{
  for (int k0 = kb; k0 < ke; k0 += KC)
  {
    double a[KC], xv[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k)
    {
      const bool in = k0 + k < ke;
      const int d = in ? S.off[k0 + k] : 0;
      i64 g = w + d;
      g = g < 0 ? 0 : (g > xl ? xl : g);
      const i64 va = (i64)(in ? S.dj[k0 + k] : 0) * S.ld + (d < 0 ? g : wv);
      a[k] = in ? S.val[va] : 0.0;
      xv[k] = in ? x(g) : 0.0;
    }
#pragma unroll
    for (int k = 0; k < KC; ++k)
      if ((m >> (k0 + k)) & 1u) acc += a[k] * xv[k];
  }
}

// Row r (window index w = own + r) of the symmetric band image, one row per lane; a row sums
// exactly its stored entries in ascending-column order (bitwise BCRSMatrix::mv when the matrix is
// bitwise symmetric, which build_sym checks).  `centre` returns the row's own operand x[w] (the
// fused step takes its (t, u) from it).
// NEAR: the offsets -1 / 0 / +1 share one centre load -- the neighbours' operands and the
// mirrored -1 value come from the adjacent lanes by DPP lane shifts (lanes 0 / 63 load theirs):
// 3 gathers + 1 value load fewer per row, i.e. ~30 % fewer L1 requests for a 7-point stencil.
template <class MT, int KC, bool NEAR, class X>
__device__ __forceinline__ void row_sym(const SymImg &S, i64 r, i64 w, int lane, const X &x, i64 xl, double &acc,
                                        typename X::raw &centre)
{
  acc = 0.0;
  const unsigned m = static_cast<const MT *>(S.mask)[r];
  const i64 wc = w > xl ? xl : w;
  if constexpr (!NEAR)
  {
    sym_span<KC>(S, 0, S.nd, m, w, w, x, xl, acc);
    centre = x.load(wc);
  }
  else
  {
    // near loads first: they fly while the far-negative span waits for its own
    const double a0 = S.j0 >= 0 ? S.val[(i64)S.j0 * S.ld + w] : 0.0;
    const double ap = S.val[(i64)S.j1 * S.ld + w];
    const typename X::raw pc = x.load(wc);
    typename X::raw el, er;
    double ae = 0.0;
    const i64 wl = w - 1 < 0 ? 0 : (w - 1 > xl ? xl : w - 1), wr = w + 1 > xl ? xl : w + 1;
    if (lane == 0)
    {
      el = x.load(wl);
      ae = S.val[(i64)S.j1 * S.ld + wl];
    }
    if (lane == 63) er = x.load(wr);
    sym_span<KC>(S, 0, S.klo, m, w, w, x, xl, acc);
    typename X::raw pl = lane_shift<false>(pc), pr = lane_shift<true>(pc);
    double am = lane_shift<false>(ap);
    if (lane == 0)
    {
      pl = el;
      am = ae;
    }
    if (lane == 63) pr = er;
    if (S.km1 >= 0 && ((m >> S.km1) & 1u)) acc += am * x.val(pl);
    if (S.k0 >= 0 && ((m >> S.k0) & 1u)) acc += a0 * x.val(pc);
    if (S.kp1 >= 0 && ((m >> S.kp1) & 1u)) acc += ap * x.val(pr);
    sym_span<KC>(S, S.khi, S.nd, m, w, w, x, xl, acc);
    centre = pc;
  }
}

struct SellB1 {
  const i64 *slice_ptr;
  const double *val;
  const i32 *col;
  const i32 *st_width;  // null when the image has no stencil slices
  const i32 *st_delta;
  const uint8_t *st_mask;
  i64 xlast;  // window length - 1 (gather clamp)
  SymImg sym;
};

// Image modes: every slice explicit, every slice stencil, or mixed (per-slice wave-uniform branch);
// kSym8 / kSym32: the symmetric band image with u8 / u32 row masks (R = 1 only); kSymN8 / kSymN32:
// the same with the lane-shift path for the offsets -1 / 0 / +1.
enum { kExplicit = 0, kStencil = 1, kMixed = 2, kSym8 = 3, kSym32 = 4, kSymN8 = 5, kSymN32 = 6 };
template <int MODE>
constexpr bool is_sym()
{
  return MODE >= kSym8;
}
template <int MODE>
using sym_mask_t = typename std::conditional<MODE == kSym8 || MODE == kSymN8, uint8_t, uint32_t>::type;
template <int MODE>
constexpr bool sym_near()
{
  return MODE == kSymN8 || MODE == kSymN32;
}

// Row sums of slice s for this lane's R rows.
template <int R, int MODE, class X>
__device__ __forceinline__ void slice_dot(const SellB1 &A, i64 s, const X &x, i64 own, int lane, double (&acc)[R])
{
  constexpr int C = 64 * R;
  if constexpr (is_sym<MODE>())
  {
    if constexpr (R == 1)  // (the launchers pick these modes only for R = 1 images)
    {
      const i64 r = s * 64 + lane;
      typename X::raw centre;
      row_sym<sym_mask_t<MODE>, 4, sym_near<MODE>()>(A.sym, r, own + r, lane, x, A.xlast, acc[0], centre);
    }
    return;
  }
  else
  {
  const i64 base = A.slice_ptr[s];
  const int width = (int)((A.slice_ptr[s + 1] - base) / C);
  const bool st = (MODE == kStencil) || (MODE == kMixed && A.st_width[s] > 0);
  if (MODE != kExplicit && st)
    rows_dot_stencil<R, X>(A.val, A.st_delta + 8 * s, A.st_mask + s * C, x, base, width, lane,
                        own + s * C + (i64)lane * R, A.xlast, acc);
  else
    rows_dot<R, X>(A.val, A.col, x, base, width, lane, acc);
  }
}

static SellB1 sell_b1(const eig_mat_s &A)
{
  SellB1 b{A.slice_ptr, A.val, A.col, A.st_width, A.st_delta, A.st_mask, A.window - 1, {}};
  if (A.sym_val)
  {
    b.sym.val = A.sym_val;
    b.sym.mask = A.sym_mask;
    b.sym.ld = A.sym_ld;
    b.sym.nd = A.sym_nd;
    for (int k = 0; k < kSymMaxOff; ++k)
    {
      b.sym.off[k] = k < A.sym_nd ? A.sym_off[k] : 0;
      b.sym.dj[k] = k < A.sym_nd ? A.sym_dj[k] : 0;
    }
    b.sym.klo = b.sym.khi = A.sym_nd;
    b.sym.km1 = b.sym.k0 = b.sym.kp1 = b.sym.j0 = b.sym.j1 = -1;
    for (int k = A.sym_nd - 1; k >= 0; --k)
    {
      const int d = A.sym_off[k];
      if (d >= -1) b.sym.klo = k;
      if (d > 1) b.sym.khi = k;
      if (d == -1) b.sym.km1 = k;
      if (d == 0) b.sym.k0 = k, b.sym.j0 = A.sym_dj[k];
      if (d == 1) b.sym.kp1 = k;
      if (d == 1 || d == -1) b.sym.j1 = A.sym_dj[k];
    }
  }
  return b;
}

// Band-image kernels on this matrix: 0 = none (the SELL / stencil kernels: EIG_MAT_NO_BAND), 1 =
// every offset through its own gather (EIG_MAT_BAND_GATHER), 2 = the lane-shift path (default).
static int sym_kernels(const eig_mat_s &A)
{
  return (A.kflags & EIG_MAT_NO_BAND) ? 0 : (A.kflags & EIG_MAT_BAND_GATHER) ? 1 : 2;
}

static bool is_sym_mode(int mode) { return mode >= kSym8; }

static int image_mode(const eig_mat_s &A)
{
  const int sk = A.sym_val ? sym_kernels(A) : 0;
  if (sk)
  {
    bool near = false;  // offsets +-1 present: the lane-shift path applies
    for (int k = 0; k < A.sym_nd; ++k) near = near || A.sym_off[k] == 1 || A.sym_off[k] == -1;
    if (sk == 2 && near) return A.sym_mask_bytes == 1 ? kSymN8 : kSymN32;
    return A.sym_mask_bytes == 1 ? kSym8 : kSym32;
  }
  if (A.n_stencil_slices == 0) return kExplicit;
  return A.n_stencil_slices == A.nslices ? kStencil : kMixed;
}

// Explicit-column slices, software-pipelined (CPF; eig_mat_tune EIG_TUNE_SELL_CPF): the NEXT slice's
// first 8 column indices are loaded while this slice's gathers are in flight, so a slice issues its
// value loads and its gathers together -- one memory round trip per slice instead of two (column
// index, then the gather it addresses).  Products and their order are rows_dot's (bitwise).
__device__ __forceinline__ void sell_cols8(const SellB1 &A, i64 s, int lane, i32 (&c)[8])
{
  const i64 base = A.slice_ptr[s];
  const int width = (int)((A.slice_ptr[s + 1] - base) >> 6);
  const i32 *cs = A.col + base;
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = k < width ? __builtin_nontemporal_load(cs + k * 64 + lane) : -1;
}

// the explicit-column slices' cross-slice column prefetch (eig_mat_tune EIG_TUNE_SELL_CPF: 1 on; 0 and
// 2 (automatic) off -- a measurement switch.  Scrambled + RCM Poisson 256^3, same-box A/B
// (profiles/r05zf_csr.jsonl): fused step 402-403 -> 436-437 us, eig_mv 308 -> 315 us: the extra
// registers cost a wave per SIMD, and those waves hid the column round trip already)
static bool sell_cpf(const eig_mat_s &A, bool fused)
{
  (void)fused;
  return A.tune_sell_cpf == 1;
}

// One explicit slice with its first 8 column indices already in registers (cc): the value loads
// and the gathers issue together, then the next slice's columns (sn >= 0) into cn, then the
// products in rows_dot's order (and its later rounds for rows wider than 8 entries).
template <class X>
__device__ __forceinline__ double sell_row_cpf(const SellB1 &A, i64 s, const X &x, int lane, const i32 (&cc)[8],
                                               i64 sn, i32 (&cn)[8])
{
  const i64 base = A.slice_ptr[s];
  const int width = (int)((A.slice_ptr[s + 1] - base) >> 6);
  const double *vs = A.val + base;
  double a[8], xv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
  {
    a[k] = k < width ? __builtin_nontemporal_load(vs + k * 64 + lane) : 0.0;
    xv[k] = cc[k] >= 0 ? x(cc[k]) : 0.0;
  }
  if (sn >= 0) sell_cols8(A, sn, lane, cn);
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (cc[k] >= 0) acc += a[k] * xv[k];
  for (int k0 = 8; k0 < width; k0 += 8)
  {
    i32 c2[8];
    double a2[8], x2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
    {
      const bool in = k0 + k < width;
      c2[k] = in ? __builtin_nontemporal_load(A.col + base + (k0 + k) * 64 + lane) : -1;
      a2[k] = in ? __builtin_nontemporal_load(vs + (k0 + k) * 64 + lane) : 0.0;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) x2[k] = c2[k] >= 0 ? x(c2[k]) : 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (c2[k] >= 0) acc += a2[k] * x2[k];
  }
  return acc;
}

// 8 waves per SIMD (8 workgroups per CU) except the mixed image, which carries both row paths.
template <int MODE>
constexpr int min_waves()
{
  return MODE == kMixed ? 1 : 8;
}

// y[own + r] = (A x)[r], 1x1 blocks (x: window base).
template <int R, int MODE, bool CPF = false>
__global__ __launch_bounds__(kStreamThreads, CPF ? 6 : min_waves<MODE>()) void k_spmv_b1(i64 nrows, i64 own, SellB1 A,
                                                               const i32 *__restrict__ slices, i64 first, i64 count,
                                                               const double *__restrict__ x, double *__restrict__ y)
{
  constexpr int C = 64 * R;
  // wave index through readfirstlane: the slice loop, slice_ptr loads and row bases stay scalar
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  i64 it0, end, step;
  slice_sweep(count, wave, it0, end, step);
  if constexpr (CPF && R == 1 && (MODE == kExplicit || MODE == kMixed))
  {
    // explicit slices software-pipelined (sell_row_cpf): the next slice's columns fly with this
    // slice's gathers; stencil slices of a mixed image as slice_dot
    auto sid = [&](i64 it) { return slices ? (i64)slices[first + it] : first + it; };
    auto expl = [&](i64 s) { return MODE == kExplicit || A.st_width[s] <= 0; };  // (explicit: width -1)
    i32 cn[8];
    if (it0 < end && expl(sid(it0))) sell_cols8(A, sid(it0), lane, cn);
    for (i64 it = it0; it < end; it += step)
    {
      const i64 s = sid(it);
      const i64 sn = it + step < end && expl(sid(it + step)) ? sid(it + step) : -1;
      double acc;
      if (expl(s))
      {
        i32 cc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) cc[k] = cn[k];
        acc = sell_row_cpf(A, s, XPlain{x}, lane, cc, sn, cn);
      }
      else
      {
        if (sn >= 0) sell_cols8(A, sn, lane, cn);
        double a1[1];
        slice_dot<1, MODE>(A, s, XPlain{x}, own, lane, a1);
        acc = a1[0];
      }
      const i64 r0 = s * C + lane;
      if (r0 < nrows) y[own + r0] = acc;
    }
    return;
  }
  for (i64 it = it0; it < end; it += step)
  {
    const i64 s = slices ? (i64)slices[first + it] : first + it;
    double acc[R];
    slice_dot<R, MODE>(A, s, XPlain{x}, own, lane, acc);
    const i64 r0 = s * C + (i64)lane * R;
#pragma unroll
    for (int q = 0; q < R; ++q)
      if (r0 + q < nrows) y[own + r0 + q] = acc[q];
  }
}

// General br x bc blocks (C = 64): lane = block row, per block br*bc values column-major over lanes.
template <int BR, int BC>
__global__ __launch_bounds__(kStreamThreads) void k_spmv_blk(i64 nbrows, const i64 *__restrict__ slice_ptr,
                                                             const i32 *__restrict__ slices, i64 first, i64 count,
                                                             const double *__restrict__ val,
                                                             const i32 *__restrict__ col,
                                                             const double *__restrict__ x, double *__restrict__ y)
{
  constexpr int BB = BR * BC;
  // wave index through readfirstlane: the slice loop, slice_ptr loads and row bases stay scalar
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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
template <int R, int MODE>
__global__ __launch_bounds__(kStreamThreads, min_waves<MODE>()) void k_lanczos_spmv_b1(
    i64 nrows, i64 own, SellB1 A, const i32 *__restrict__ slices, i64 first, i64 count,
    const double *__restrict__ u, const double *__restrict__ up, double *__restrict__ t, int j,
    const double *__restrict__ nsum,
    double *__restrict__ dot_out, double *__restrict__ beta_out, const double *__restrict__ carry,
    double *partials, unsigned *ticket)
{
  constexpr int C = 64 * R;
  __shared__ double tot[1];
  // wave index through readfirstlane: the slice loop, slice_ptr loads and row bases stay scalar
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double beta = sqrt(nsum[j]);
  const double sig = 1.0 / beta;
  const double gam = (j > 0) ? beta * (1.0 / sqrt(nsum[j - 1])) : 0.0;
  i64 it0, end, step;
  slice_sweep(count, wave, it0, end, step);
  double d = 0.0;
  for (i64 it = it0; it < end; it += step)
  {
    const i64 s = slices ? (i64)slices[first + it] : first + it;
    const i64 r0 = s * C + (i64)lane * R;
    // epilogue operands issued before the row loop so their latency hides under the matrix stream
    double upv[R], uv[R];
#pragma unroll
    for (int q = 0; q < R; ++q)
    {
      const bool ok = r0 + q < nrows;
      upv[q] = (ok && j > 0) ? up[own + r0 + q] : 0.0;
      uv[q] = ok ? u[own + r0 + q] : 0.0;
    }
    double acc[R];
    slice_dot<R, MODE>(A, s, XPlain{u}, own, lane, acc);
#pragma unroll
    for (int q = 0; q < R; ++q)
    {
      const i64 r = r0 + q;
      if (r < nrows)
      {
        double ti = acc[q] * sig;
        if (j > 0) ti = ti - gam * upv[q];
        t[own + r] = ti;
        d += ti * uv[q];
      }
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

// ---------------------------------------------------------------------------------------------
// Fused one-reduction Lanczos step.  u_k = t_{k-1} - c u_{k-1} is formed inside the
// gathers of the SpMV that needs it (XPair), and its squared norm is PREDICTED from the previous
// step's reductions instead of being reduced before the SpMV:
//   c = dsum/m,  nt_k = tsq - c dsum       (m = measured ||u_{k-1}||^2, reduced when u_{k-1} was
//                                             formed; using it keeps the prediction error at
//                                             rounding level -- tsq - alpha^2 alone diverges)
//   t_k = ((A u_k) - mu u_k) sig_k - gam_k u_{k-1},  sig_k = 1/sqrt(nt_k)
//   (dsum_k, tsq_k, m_k) = (t_k . u_k, t_k . t_k, u_k . u_k)   -> ONE allreduce of 3 doubles
// Guard against cancellation (nt_k = ||t||^2 - (t.u)^2/||u||^2 loses digits when |alpha| >> beta):
//  * the step runs on A - mu I, mu = trace(A)/n (a constant inside the spectrum): the Krylov space,
//    beta and alpha - mu are unchanged, but |alpha - mu| stays of the order of the spectral width
//    however far the operator is shifted (A + 1e6 I costs nothing extra);
//  * when the prediction still keeps less than kFusedTau of tsq (nt <= tau tsq, incl. nt <= 0 and
//    NaN), the launch REPAIRS instead of stepping: it forms u_k explicitly into the output pairs
//    (u_k, u_{k-1}) and reduces its exact norm; the next launch then takes step k with c = 0 and
//    the exact nt_k (the same per-row code: x - 0 y = x).  The decision is made on the device from
//    the allreduced sums (identical on every rank), so no step synchronises with the host; the
//    host tops the launch count up afterwards (drivers.cpp).  Launch L reads its logical step j
//    and mode from ctl[2L], ctl[2L+1] and block 0 writes those of launch L+1.
// Same formulas as orc_lanczos_fused (oracle.cc).
// ---------------------------------------------------------------------------------------------
constexpr double kFusedTau = 1e-2;
enum { kFusedStep = 0, kFusedPost = 1, kFusedHalt = 2, kFusedRepair = 3, kFusedNoop = 4 };

struct FusedArgs {
  double *nsum, *alpha, *beta;  // per logical step
  const double *fred;           // per launch: 3 allreduced sums
  int *ctl;                     // per launch: (logical step j, mode) at its start
  double *aux;                  // per launch: (rn, rm) handed from a repair to the next launch
  const double *mu2;            // (sum of the diagonal, rows), allreduced: mu = mu2[0] / mu2[1]
  double *pn;                   // per launch: nsum[j - 1] of its step (LanczosState::pn)
  int L;                        // launch index
  int force;                    // 1: repair even if the prediction is sound (exact final beta)
  int xch;                      // kXchPublish: the last workgroup allreduces the sums through the
                                // peers' mailboxes (xch_dev.h) instead of an allreduce launch after
  Mailbox mb;                   // (xch != 0) this rank's mailbox
};

struct FusedStep {
  int j, act;
  double c, nt, ap, bk, gam, sig, mu, rn, rm;
};

// Prologue of a fused launch (every thread; wave- and grid-uniform); block 0 / thread 0 stores the
// step's scalars and the next launch's control word.  Returns the action.
__device__ __forceinline__ FusedStep fused_begin(const FusedArgs &f)
{
  FusedStep s;
  // every operand the prologue may need, loaded together (addresses depend on L only: one memory
  // round trip before the launch's streams start, instead of ctl -> nsum[j - 1])
  const int cj = f.ctl[2 * f.L], mode = f.ctl[2 * f.L + 1];
  const double mu0 = f.mu2[0], mu1 = f.mu2[1];
  const int Lp = f.L > 0 ? f.L - 1 : 0;
  const double fd = f.fred[3 * Lp], fq = f.fred[3 * Lp + 1], fm = f.fred[3 * Lp + 2];
  const double ax0 = f.aux[2 * f.L], ax1 = f.aux[2 * f.L + 1], pnl = f.pn[f.L], ns0 = f.nsum[0];
  s.j = cj;
  s.mu = mu0 / mu1;
  s.c = s.ap = s.bk = s.gam = s.rn = s.rm = 0.0;
  s.nt = 1.0;
  const int j = s.j;
  if (mode == kFusedHalt) s.act = kFusedHalt;
  else if (f.force && (j == 0 || mode != kFusedStep)) s.act = kFusedNoop;
  else if (mode == kFusedPost)
  {
    const double mex = fm;
    s.rn = ax0;
    s.rm = ax1;
    s.nt = mex;
    if (!(mex > 0.0)) s.act = kFusedHalt;  // u_j = 0: invariant subspace
    else
    {
      s.bk = sqrt(mex) * s.rn / s.rm;
      s.gam = s.bk / s.rm;
      s.act = kFusedPost;
    }
  }
  else if (j == 0)
  {
    s.nt = ns0;
    s.act = kFusedStep;
  }
  else
  {
    const double d = fd, q = fq, m = fm;
    s.rn = sqrt(pnl);
    s.rm = sqrt(m);
    s.c = d / m;
    s.ap = s.c * s.rn + s.mu;
    s.nt = q - s.c * d;
    if (f.force || !(s.nt > kFusedTau * q)) s.act = kFusedRepair;
    else
    {
      s.bk = sqrt(s.nt) * s.rn / s.rm;
      s.gam = s.bk / s.rm;
      s.act = kFusedStep;
    }
  }
  s.sig = 1.0 / sqrt(s.nt);
  if (blockIdx.x == 0 && threadIdx.x == 0)  // (both launches of a split step store the same values)
  {
    int nj = j, nm = kFusedStep;
    switch (s.act)
    {
      case kFusedStep:
        if (j > 0)
        {
          f.nsum[j] = s.nt;
          f.alpha[j - 1] = s.ap;
          f.beta[j] = s.bk;
        }
        else
          f.beta[0] = sqrt(s.nt);
        nj = j + 1;
        break;
      case kFusedPost:
        f.nsum[j] = s.nt;
        f.beta[j] = s.bk;
        nj = j + 1;
        break;
      case kFusedRepair:
        f.alpha[j - 1] = s.ap;
        f.aux[2 * f.L + 2] = s.rn;
        f.aux[2 * f.L + 3] = s.rm;
        nm = kFusedPost;
        break;
      case kFusedHalt:
        if (mode == kFusedPost)
        {
          f.nsum[j] = 0.0;
          f.beta[j] = 0.0;
        }
        nm = kFusedHalt;
        break;
      default:  // kFusedNoop
        nm = mode;
        if (mode == kFusedPost)
        {
          f.aux[2 * f.L + 2] = f.aux[2 * f.L];
          f.aux[2 * f.L + 3] = f.aux[2 * f.L + 1];
        }
        break;
    }
    f.ctl[2 * f.L + 2] = nj;
    f.ctl[2 * f.L + 3] = nm;
    // nsum[j' - 1] for the next launch: the norm this launch fixed (step / post: nsum[j]); otherwise
    // the logical step does not advance and the value carries over
    f.pn[f.L + 1] = (s.act == kFusedStep || s.act == kFusedPost) ? s.nt : pnl;
  }
  return s;
}

// Launch with nothing to compute (halted recurrence, or a forced repair with nothing to repair):
// the reduction slot reads zero.
// (The host forces a repair only after reading a stepping state, so kFusedNoop is defensive.)
__device__ __forceinline__ void fused_idle(double *out)
{
  if (blockIdx.x == 0 && threadIdx.x < 3) out[threadIdx.x] = 0.0;
}

// End of a fused launch: the grid reduction of the three sums (plus a split step's carry) into
// out; with kXchPublish the last workgroup first allreduces them with the peers through their
// mailboxes (xch_dev.h), so out holds the global sums when the kernel ends.  An idle launch takes
// this path with zero sums when it exchanges (every rank idles at the same launch).
template <int U>
__device__ __forceinline__ void fused_finish(double (&v)[3], double *partials, unsigned *ticket, double *tot,
                                             double *out, const double *carry, const FusedArgs &fa)
{
  if (grid_sum<3, kStreamThreads, U>(v, partials, ticket, tot))
  {
    if (fa.xch & kXchPublish)
    {
      if (carry)
      {
        if (threadIdx.x < 3) tot[threadIdx.x] += carry[threadIdx.x];
        __syncthreads();
      }
      xch_exchange(fa.mb, tot);
      if (threadIdx.x < 3) out[threadIdx.x] = tot[threadIdx.x];
    }
    else if (threadIdx.x < 3)
      out[threadIdx.x] = carry ? (carry[threadIdx.x] + tot[threadIdx.x]) : tot[threadIdx.x];
  }
}

// Repair launch body for rows [r0, r1) (owned-row indices, grid-stride): u = t - c u_prev into the
// output pair (u, u_prev), and ||u||^2.  The same mul-then-sub as the gathers (XPair), so the step
// that follows multiplies exactly the u_k the unrepaired step would have formed.
__device__ __forceinline__ double fused_repair_rows(i64 r0, i64 r1, i64 own, double c, const dpair *__restrict__ P,
                                                    dpair *__restrict__ Pout)
{
  double m2 = 0.0;
  const i64 stride = (i64)gridDim.x * blockDim.x;
  for (i64 r = r0 + (i64)blockIdx.x * blockDim.x + threadIdx.x; r < r1; r += stride)
  {
    const dpair p = P[own + r];
    const double u = p.x - c * p.y;
    Pout[own + r] = dpair{u, p.y};
    m2 += u * u;
  }
  return m2;
}

// Fused step, one stencil slice, one row per lane: gathers the (t, u) pairs at the slice's offsets
// (16-B loads, clamped addresses as rows_dot_stencil), accumulates sum a (t - c u) in offset order
// and takes the row's own (t, u) from the delta = 0 gather instead of a separate load.  KC entries
// in flight per round.  Same arithmetic and order as the generic path (bitwise equal).
template <int KC>
__device__ __forceinline__ void fused_row_stencil(const SellB1 &A, i64 s, const dpair *__restrict__ P, double c,
                                                  i64 own, int lane, double &acc, double &tv, double &uv)
{
  const i64 base = A.slice_ptr[s];
  const int width = (int)((A.slice_ptr[s + 1] - base) >> 6);
  const i32 *dl = A.st_delta + 8 * s;
  const unsigned m = A.st_mask[s * 64 + lane];
  const double *vs = A.val + base;
  const i64 xrow0 = own + s * 64 + lane;
  const i64 xl = A.xlast;
  acc = 0.0;
  bool centre = false;  // wave-uniform: the offset list holds delta = 0
  for (int k0 = 0; k0 < width; k0 += KC)
  {
    double a[KC];
    dpair pr[KC];
    int dk[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k)
    {
      const bool in = k0 + k < width;
      dk[k] = in ? dl[k0 + k] : 0;
      a[k] = in ? __builtin_nontemporal_load(vs + (k0 + k) * 64 + lane) : 0.0;
    }
#pragma unroll
    for (int k = 0; k < KC; ++k)
    {
      i64 g = xrow0 + dk[k];
      g = g < 0 ? 0 : (g > xl ? xl : g);
      pr[k] = (k0 + k < width) ? P[g] : dpair{0.0, 0.0};
    }
#pragma unroll
    for (int k = 0; k < KC; ++k)
    {
      if (k0 + k < width && dk[k] == 0)
      {
        tv = pr[k].x;
        uv = pr[k].y;
        centre = true;
      }
      if ((m >> (k0 + k)) & 1u) acc += a[k] * (pr[k].x - c * pr[k].y);
    }
  }
  if (!centre)
  {
    const i64 g = xrow0 > xl ? xl : xrow0;
    const dpair pv = P[g];
    tv = pv.x;
    uv = pv.y;
  }
}

// Register budget for 8 waves / SIMD (W): stencil rows take 4 entries per round to fit 64 VGPRs
// (measured: 5 waves with 8 entries per round and 6 waves were no faster).
// (explicit-column and mixed images: 6 waves / SIMD; at 8 their row loops spill 36 / 46 VGPRs to
// scratch, whose write-back is the write traffic PMC showed beyond the pair stores.  Stencil
// images: 7 (at 8: 20 B of scratch per lane; 3-D Poisson 256^3 on the SELL stencil image 353.2 ->
// 333.3 us, tools/stencil_fused.py)
template <int MODE>
constexpr int fused_b1_waves()
{
  return (MODE == kExplicit || MODE == kMixed) ? 6 : MODE == kStencil ? 7 : 8;
}

template <int R, int MODE, bool CPF = false>
__global__ __launch_bounds__(kStreamThreads, CPF ? 5 : fused_b1_waves<MODE>()) void k_lanczos_fused_b1(
    i64 nrows, i64 own, SellB1 A, const i32 *__restrict__ slices, i64 first, i64 count,
    const dpair *__restrict__ P, dpair *__restrict__ Pout, FusedArgs fa, double *__restrict__ out,
    const double *__restrict__ carry, double *partials, unsigned *ticket)
{
  constexpr int C = 64 * R;
  constexpr int W = 8;
  __shared__ double tot[3];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const FusedStep fs = fused_begin(fa);
  if (fs.act == kFusedHalt || fs.act == kFusedNoop)
  {
    double z[3] = {0.0, 0.0, 0.0};
    if (fa.xch & kXchPublish) fused_finish<2>(z, partials, ticket, tot, out, nullptr, fa);
    else fused_idle(out);
    return;
  }
  const double c = fs.c, gam = fs.gam, sig = fs.sig, mu = fs.mu;
  const int k = fs.j;
  i64 it0, end, step;
  slice_sweep(count, wave, it0, end, step);
  if (fs.act == kFusedRepair)
  {
    // this launch's rows: its slices
    double m2 = 0.0;
    for (i64 it = it0; it < end; it += step)
    {
      const i64 s = slices ? (i64)slices[first + it] : first + it;
#pragma unroll
      for (int q = 0; q < R; ++q)
      {
        const i64 r = s * C + (i64)lane * R + q;
        if (r < nrows)
        {
          const dpair p = P[own + r];
          const double u = p.x - c * p.y;
          Pout[own + r] = dpair{u, p.y};
          m2 += u * u;
        }
      }
    }
    double v[3] = {0.0, 0.0, m2};
    fused_finish<2>(v, partials, ticket, tot, out, carry, fa);
    return;
  }
  const XPair xc{P, c};
  double d = 0.0, q2 = 0.0, m2 = 0.0;
  auto sid = [&](i64 it) { return slices ? (i64)slices[first + it] : first + it; };
  auto expl = [&](i64 s) { return MODE == kExplicit || A.st_width[s] <= 0; };  // (explicit: width -1)
  constexpr bool kCpf = CPF && R == 1 && (MODE == kExplicit || MODE == kMixed);
  i32 cn[8];
  if constexpr (kCpf)
  {
    if (it0 < end && expl(sid(it0))) sell_cols8(A, sid(it0), lane, cn);
  }
  for (i64 it = it0; it < end; it += step)
  {
    const i64 s = sid(it);
    const i64 r0 = s * C + (i64)lane * R;
    double tv[R], uv[R], acc[R];
    if constexpr (kCpf)
    {
      const bool more = it + step < end;
      if (expl(s))
      {
        i32 cc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) cc[k] = cn[k];
        const dpair pv = r0 < nrows ? P[own + r0] : dpair{0.0, 0.0};
        const i64 sn = more && expl(sid(it + step)) ? sid(it + step) : -1;
        acc[0] = sell_row_cpf(A, s, xc, lane, cc, sn, cn);
        tv[0] = pv.x;
        uv[0] = pv.y;
      }
      else
      {
        if (more && expl(sid(it + step))) sell_cols8(A, sid(it + step), lane, cn);
        fused_row_stencil<(W >= 8 ? 4 : 8)>(A, s, P, c, own, lane, acc[0], tv[0], uv[0]);
      }
    }
    else if constexpr (is_sym<MODE>())
    {
      if constexpr (R == 1)
      {
        dpair pc;
        // far spans: 4 entries per round (2 on the lane-shift path, whose near operands stay live
        // across the far-negative span) at 8 waves / SIMD, 8 at 5
        constexpr int KC = W >= 8 ? (sym_near<MODE>() ? 2 : 4) : 8;
        row_sym<sym_mask_t<MODE>, KC, sym_near<MODE>()>(A.sym, r0, own + r0, lane, xc, A.xlast, acc[0], pc);
        tv[0] = pc.x;
        uv[0] = pc.y;
      }
    }
    else if (R == 1 && MODE != kExplicit && (MODE == kStencil || A.st_width[s] > 0))
    {
      fused_row_stencil<(W >= 8 ? 4 : 8)>(A, s, P, c, own, lane, acc[0], tv[0], uv[0]);
    }
    else
    {
#pragma unroll
      for (int q = 0; q < R; ++q)
      {
        const bool ok = r0 + q < nrows;
        const dpair pv = ok ? P[own + r0 + q] : dpair{0.0, 0.0};
        tv[q] = pv.x;
        uv[q] = pv.y;
      }
      slice_dot<R, MODE>(A, s, xc, own, lane, acc);
    }
#pragma unroll
    for (int q = 0; q < R; ++q)
    {
      const i64 r = r0 + q;
      if (r < nrows)
      {
        const double uk = tv[q] - c * uv[q];
        double ti = (acc[q] - mu * uk) * sig;
        if (k > 0) ti = ti - gam * uv[q];
        Pout[own + r] = dpair{ti, uk};
        d += ti * uk;
        q2 += ti * ti;
        m2 += uk * uk;
      }
    }
  }
  double v[3] = {d, q2, m2};
  fused_finish<2>(v, partials, ticket, tot, out, carry, fa);
}

// ---------------------------------------------------------------------------------------------
// Plane-marching fused step (2.5-D blocking of the symmetric band image).  When the band's widest
// offset D (= N^2 for a 3-D 7-point grid, N for 2-D) is a multiple of 64 and every other offset is
// narrower, rows split into "planes" of D rows and a wave owns one 64-row column of a run of
// planes: lane l handles rows c*64 + l + z*D for z = z0 .. z1-1.  The -D neighbour of a row is then
// the row the same lane handled one iteration earlier and the +D neighbour the one it handles
// next, so the far pair operands and the mirrored -D value ride in registers: each (t, u) pair is
// loaded once (as the +D operand, then carried as the centre and as the -D operand) and each
// upper value once.  Offsets in (-D, D) other than -1/0/+1 are gathered (their rows were just
// streamed by the neighbouring columns of the same plane, on the same XCD: L2 hits); -1/0/+1 use
// the lane shifts.  Per-row arithmetic and order are those of row_sym (bitwise the same t, u);
// only the assignment of rows to waves differs, so the three reductions sum in another order.
// Work items (column, plane run) are spread so each XCD takes one contiguous plane run across all
// columns (swizzled_block): the column neighbours of a row share the XCD's L2.
// ---------------------------------------------------------------------------------------------
struct MarchPlan {
  i64 D;        // rows per plane (the band's widest offset)
  i64 zb;       // first plane marched
  i64 nplanes;  // planes marched: zb .. zb + nplanes - 1 (whole launch: ceil(rows / D) from 0)
  i64 mrows;    // rows covered by the row mask (nslices * 64)
  int ncol;     // D / 64
  int nseg;     // plane runs per column
  // first entries of the far spans (-D, -1) and (+1, +D): offset (0 = empty span) and band array
  i32 dn, dq;
  const double *Un, *Uq;
  // uniform band (eig_mat_s::sym_uniform): the band values of the +D, 0, +1, far-span (dn / dq)
  // arrays, taken instead of the array loads by the UNI kernels
  double cD, c0, c1, cn, cq;
  // geometric row masks (eig_mat_s::sym_geo, uniform bands only): the nx x ny x nz grid whose
  // in-grid neighbours are exactly the stored entries -- the march derives each row's mask from
  // its coordinates instead of loading it; gz0 = the global plane of the rank's first row
  int gx, gy, gz, gz0;
  int uni;  // the march variant the launch takes (march_uniform: 0 arrays, 1 loaded masks, 2..9 geometric)
  // results stored with plain (MALL-allocating) stores instead of nontemporal ones: the vectors of a
  // small grid stay in the 256 MB memory-side cache for the next launch (geo2 kernels)
  int tstore;
  // box marches (variant 12): band array of the upper offset at 27-box position (a+1) 9 + (b+1) 3 + (c+1),
  // -1 when the stencil does not store it
  signed char kj[27];
  const double *pack;
  // eig_mat_tune(EIG_TUNE_CACHE) bits for the value march (measurement): 2 = the value streams with the
  // default cache policy instead of nontemporal, 4 = the +D pair stream nontemporal
  int cache;
  // geo2 value marches: 4 = a workgroup's 4 waves march the same 64 x of 4 consecutive y lines (their
  // +-nx gathers then mostly read lines their sibling waves just loaded on the same CU) instead of the
  // 4 x runs of one line; 0 = the item order (eig_mat_tune EIG_TUNE_MARCH_LINES)
  int lines;
};
// store helper of the geo2 epilogues: temporal when the plan says the vectors fit the MALL
template <class T>
__device__ __forceinline__ void march_store(const MarchPlan &mp, T v, T *p)
{
  if (mp.tstore)
    *p = v;
  else
    __builtin_nontemporal_store(v, p);
}

// Geometric uniform-band march with the +D operand loaded PF + 1 planes ahead (UNI = 2 + PF;
// eig_mat_tune(EIG_TUNE_MARCH_PREFETCH)).  The plain march waits for every load of plane z --
// including the +D pair that only arrives from HBM -- and, at the loop head, for the store of
// plane z - 1 (one vmcnt counter, in order), so a wave has one plane's memory in flight.  Here the
// plane's loads are issued gathers first, prefetch last, so the waits for the L2 gathers leave the
// prefetch in flight; the prefetch slots rotate through a loop unrolled PF + 1 times (no register
// moves of in-flight loads); the edge operand is loaded by every lane (lanes 1..62 fetch lane 0's,
// one cache line) so no divergent branch merges pending loads; and there is no row test (a
// geometric image covers whole planes: every marched row exists).  Products, sums and their order
// are those of march_rows<UNI = 2>: bitwise the same results.
template <int PF, bool PG, class X, class EPI>
__device__ __forceinline__ void march_rows_geo(const SellB1 &A, const MarchPlan &mp, i64 own, int lane, int wave,
                                               const X &x, EPI &epi)
{
  typedef typename X::raw raw;
  const SymImg &S = A.sym;
  const int xl = (int)A.xlast, D = (int)mp.D, own32 = (int)own;
  const int nd = S.nd;
  const int item = (int)swizzled_block() * kWaves + wave;
  if (item >= mp.ncol * mp.nseg) return;
  const int col = item % mp.ncol, seg = item / mp.ncol;
  const int z0 = (int)(mp.zb + seg * mp.nplanes / mp.nseg), z1 = (int)(mp.zb + (seg + 1) * mp.nplanes / mp.nseg);
  auto cx = [&](int g) -> unsigned { return g < 0 ? 0u : (unsigned)(g > xl ? xl : g); };
  const int kn0 = 1, kp0 = S.khi, kp1 = nd - 1;
  unsigned gxy = 0;
  {
    const int pr = col * 64 + lane, gxc = pr % mp.gx, gyc = pr / mp.gx;
    unsigned b = 0;
    int k = 1;
    if (mp.dn) b |= (gyc > 0 ? 1u : 0u) << k++;
    b |= (gxc > 0 ? 1u : 0u) << k++;
    b |= 1u << k++;
    b |= (gxc < mp.gx - 1 ? 1u : 0u) << k++;
    if (mp.dq) b |= (gyc < mp.gy - 1 ? 1u : 0u) << k++;
    gxy = b;
  }
  int w = own32 + col * 64 + lane + z0 * D;
  const int eoff = lane == 63 ? 1 : -1 - lane;  // lane 63: row w + 1; the others: lane 0's row w - 1
  // slots: plane z's pair (the centre), z + 1 (the +D operand), ..., z + PF + 1 (in flight); body k
  // of a trip reads slots k and k + 1 and loads into slot k + PF + 1 (mod PF + 2): no slot is copied
  constexpr int NS = PF + 2;
  struct Gath {
    raw eg, xn, xq;
  };
  auto gather = [&](int wg, Gath &g) {
    g.eg = x.load(cx(wg + eoff));
    if (mp.dn) g.xn = x.load(cx(wg + mp.dn));
    if (mp.dq) g.xq = x.load(cx(wg + mp.dq));
  };
  double pmv = x.val(x.load(cx(w - D)));
  raw sl[NS];
  Gath gs[2];
#pragma unroll
  for (int k = 0; k <= PF; ++k) sl[k] = x.load(cx(w + k * D));
  if constexpr (PG) gather(w, gs[0]);
  // PG: plane z + 1's gathers are issued in body z (before its prefetch), so the wait for them in
  // body z + 1 leaves the loads of body z + 1 in flight as well
  auto body = [&](int z, const raw &pcur, const raw &pd, raw &pf, Gath &gc, Gath &gn) {
    if constexpr (PG)
      gather(w + D, gn);
    else
      gather(w, gc);
    pf = x.load(cx(w + (PF + 1) * D));
    const int zg = z + mp.gz0;
    const unsigned m = gxy | (zg > 0 ? 1u : 0u) | (zg < mp.gz - 1 ? 1u << kp1 : 0u);
    double acc = 0.0;
    if (m & 1u) acc += mp.cD * pmv;
    if (mp.dn && ((m >> kn0) & 1u)) acc += mp.cn * x.val(gc.xn);
    const double vc = x.val(pcur);
    double vl = lane_shift<false>(vc), vr = lane_shift<true>(vc);
    const double ve = x.val(gc.eg);
    if (lane == 0) vl = ve;
    if (lane == 63) vr = ve;
    if (S.km1 >= 0 && ((m >> S.km1) & 1u)) acc += mp.c1 * vl;
    if (S.k0 >= 0 && ((m >> S.k0) & 1u)) acc += mp.c0 * vc;
    if (S.kp1 >= 0 && ((m >> S.kp1) & 1u)) acc += mp.c1 * vr;
    if (mp.dq && ((m >> kp0) & 1u)) acc += mp.cq * x.val(gc.xq);
    if ((m >> kp1) & 1u) acc += mp.cD * x.val(pd);
    epi(w - own32, w, acc, pcur);
    pmv = vc;
    w += D;
  };
  // (NS bodies per trip; with PG the gather sets alternate, so NS must be even)
  static_assert(!PG || NS % 2 == 0, "gather prefetch: an even number of bodies per trip");
  int z = z0;
  for (; z + NS - 1 < z1; z += NS)
  {
#pragma unroll
    for (int k = 0; k < NS; ++k)
      body(z + k, sl[k], sl[(k + 1) % NS], sl[(k + PF + 1) % NS], gs[PG ? k & 1 : 0], gs[PG ? (k + 1) & 1 : 1]);
  }
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (z + k < z1)
      body(z + k, sl[k], sl[(k + 1) % NS], sl[(k + PF + 1) % NS], gs[PG ? k & 1 : 0], gs[PG ? (k + 1) & 1 : 1]);
}

// Raw buffer loads (32-bit byte offset, hardware range check: an offset at or past the descriptor's
// byte count, or any offset through a zero-record descriptor, returns 0 without a memory access).
__device__ __forceinline__ void bload(__amdgpu_buffer_rsrc_t r, unsigned off, dpair &v)
{
  v = __builtin_bit_cast(dpair, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ void bload(__amdgpu_buffer_rsrc_t r, unsigned off, double &v)
{
  v = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
}
__device__ __forceinline__ void bload_nt(__amdgpu_buffer_rsrc_t r, unsigned off, dpair &v)
{
  v = __builtin_bit_cast(dpair, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 2));
}
__device__ __forceinline__ void bload_nt(__amdgpu_buffer_rsrc_t r, unsigned off, double &v)
{
  v = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 2));
}
// lane l takes v of lane l - 1 (NEXT = false) or l + 1; the lane without a source keeps `old`
template <bool NEXT>
__device__ __forceinline__ double lane_shift_or(double v, double old)
{
  return __builtin_amdgcn_update_dpp(old, v, NEXT ? 0x130 : 0x138, 0xf, 0xf, false);
}

// Geometric uniform-band march without row masks or selects (UNI 7..9; grids whose x extent is a
// multiple of 64, so each wave's 64 rows share one y line and one plane, and windows under 2 GiB).
// Every stored offset of a row is its in-grid neighbour (verified at upload), so the only missing
// terms are at the grid faces -- and a missing neighbour's operand is made EXACTLY zero instead of
// being masked out: the -nx / +nx gathers of a wave on the first / last y line go through a
// zero-record buffer descriptor (wave-uniform choice), the +D operand of the last global plane too
// (plane-uniform), the -D operand of the first global plane is set to 0, and the lane-0 / lane-63
// edge operand of a wave at x = 0 / x = nx - 1 is an out-of-range offset (the other 62 lanes'
// edge loads are out of range as well: no traffic).  The value of a zero pair is +0 and the band
// constant times it is +-0; acc starts at +0 and can never become -0 under round-to-nearest, so
// acc + (+-0) == acc bit for bit (also for Inf / NaN acc): each row's sum, term order and rounding
// are those of march_rows<UNI = 2> -- bitwise the same results -- with ~half its VALU work (no
// mask bits, selects or 64-bit address clamps).  Prefetch slots as in march_rows_geo.
// pre(x): called once the wave's first loads are in flight (the fused step's scalar prologue runs
// under them; it sets x's scalars); false = the launch does not march (the loads are dropped).
struct MarchNoPre {
  template <class X>
  __device__ __forceinline__ bool operator()(X &) const { return true; }
};
// VAL (march variants 10 / 11: geometric bands whose values are not uniform): the band values are
// streamed from the symmetric band arrays instead -- the +D / 0 / +1 / +nx values of each row once
// (nontemporal), the mirrored -D value carried from the previous plane in a register, the mirrored
// -1 value by the same lane shift as the operands (lane 0 loads its own), the mirrored -nx value
// re-read at row w - nx (the +nx array, streamed 4 columns earlier on the same XCD: an L2 hit).
// A missing neighbour's value reads as 0.0 (its slot is unset, or the same zero-record / out-of-range
// load as its operand) and its operand as exactly zero, so its product is +-0 and the row's sum is
// that of the masked march bit for bit.  VAL = 2 (variant 11) issues the next plane's value streams
// one plane ahead (the last plane of a run issues none).
template <int PF, bool PG, int VAL, class X, class EPI, class PRE>
__device__ __forceinline__ void march_rows_geo2(const SellB1 &A, const MarchPlan &mp, i64 own, int lane, int wave,
                                                X x, EPI &epi, PRE &pre)
{
  typedef typename X::raw raw;
  constexpr unsigned SZ = sizeof(raw);
  const int D = (int)mp.D, own32 = (int)own;
  int col, seg;
  if (mp.lines == 4)
  {
    // workgroup -> (x run, group of 4 lines, plane run); wave -> line of the group
    const int nxc = mp.gx / 64, per = nxc * (mp.gy / 4);
    const int wg = (int)swizzled_block();
    if (wg >= per * mp.nseg) return;
    seg = wg / per;
    const int r = wg % per;
    col = ((r / nxc) * 4 + wave) * nxc + r % nxc;
  }
  else
  {
    const int item = (int)swizzled_block() * kWaves + wave;
    if (item >= mp.ncol * mp.nseg) return;
    col = item % mp.ncol;
    seg = item / mp.ncol;
  }
  const int z0 = (int)(mp.zb + seg * mp.nplanes / mp.nseg), z1 = (int)(mp.zb + (seg + 1) * mp.nplanes / mp.nseg);
  const unsigned nbytes = (unsigned)(A.xlast + 1) * SZ;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(x.ptr()), 0, (int)nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(x.ptr()), 0, 0, 0x00020000);
  // the wave's line: first x and its y (wave-uniform)
  const int x0 = (col * 64) % mp.gx, yw = (col * 64) / mp.gx;
  // (2-D grids have no +-nx offsets: both gathers read zeros through r0, and cn = cq = 0, so
  // their terms add +-0 -- no branch around a load in the loop)
  const __amdgpu_buffer_rsrc_t rn = mp.dn && yw > 0 ? rs : r0, rq = mp.dq && yw < mp.gy - 1 ? rs : r0;
  constexpr unsigned kOut = 0x80000000u;  // + any window offset (< 2 GiB): past the byte count
  const unsigned eoff = lane == 0 ? (x0 > 0 ? 0u - SZ : kOut) : lane == 63 ? (x0 + 64 < mp.gx ? SZ : kOut) : kOut;
  const unsigned dnb = (unsigned)mp.dn * SZ, dqb = (unsigned)mp.dq * SZ, Db = (unsigned)D * SZ;
  int w = own32 + col * 64 + lane + z0 * D;
  unsigned vo = (unsigned)w * SZ;
  const int zg0 = z0 + mp.gz0;
  constexpr int NS = PF + 2;
  struct Gath {
    raw eg, xn, xq;
  };
  auto gather = [&](unsigned v, Gath &g) {
    bload(rs, v + eoff, g.eg);
    bload(rn, v + dnb, g.xn);
    bload(rq, v + dqb, g.xq);
  };
  // VAL: one descriptor per band array (8-B slots, window-indexed like the operands); vv = w * 8
  const SymImg &S = A.sym;
  const unsigned vbytes = (unsigned)S.ld * 8u;
  auto arr = [&](int j, bool on) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(S.val + (i64)(j >= 0 ? j : 0) * S.ld), 0,
                                             on && j >= 0 ? (int)vbytes : 0, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t vD = arr(S.dj[S.nd - 1], VAL), v0 = arr(S.j0, VAL), v1 = arr(S.j1, VAL),
                               vq = arr(S.dj[S.khi], VAL && mp.dq), vn = arr(S.dj[S.khi], VAL && mp.dn && yw > 0);
  const unsigned eov = lane == 0 && x0 > 0 ? 0u - 8u : kOut;  // lane 0: the mirrored -1 value at w - 1
  const unsigned dnv = (unsigned)mp.dn * 8u, Dv = (unsigned)D * 8u;
  unsigned vv = (unsigned)w * 8u;
  struct Vals {
    double aD, a0, ap, aq, an, ae;
  };
  const __amdgpu_buffer_rsrc_t vz = arr(0, false);
  const double *pD = S.val + (i64)S.dj[S.nd - 1] * S.ld, *p1 = S.val + (i64)(S.j1 >= 0 ? S.j1 : 0) * S.ld;
  const double *p0 = S.j0 >= 0 ? S.val + (i64)S.j0 * S.ld : nullptr, *pq = S.val + (i64)S.dj[S.khi] * S.ld;
  auto vload = [&](unsigned o, Vals &v, bool on) {  // on: wave-uniform (false: zeros, no traffic)
    if constexpr (VAL == 5)
    {
      // variant 15: the pack through 64-bit global addresses (wave-uniform / lane-0 conditions
      // instead of range-checked descriptors)
      const i64 r = (i64)(o >> 3);
      const dpair *P01 = reinterpret_cast<const dpair *>(mp.pack), *P23 = P01 + S.ld;
      const dpair p0 = (mp.cache & 2) ? P01[r] : __builtin_nontemporal_load(P01 + r);
      const dpair p1 = P23[r];
      v.aD = p0.x;
      v.a0 = p0.y;
      v.ap = p1.x;
      v.aq = p1.y;
      v.an = mp.dn && yw > 0 ? P23[r + mp.dn].y : 0.0;
      v.ae = lane == 0 && x0 > 0 ? P23[r - 1].x : 0.0;
    }
    else if constexpr (VAL == 4)
    {
      // (measurement variant 14: the same loads through 64-bit global addresses, as the plain march)
      const i64 r = (i64)(o >> 3);
      v.aD = on ? __builtin_nontemporal_load(pD + r) : 0.0;
      v.a0 = on && p0 ? __builtin_nontemporal_load(p0 + r) : 0.0;
      v.ap = on ? __builtin_nontemporal_load(p1 + r) : 0.0;
      v.aq = on && mp.dq ? pq[r] : 0.0;
      v.an = on && mp.dn && yw > 0 ? pq[r + mp.dn] : 0.0;
      v.ae = on && lane == 0 && x0 > 0 ? p1[r - 1] : 0.0;
    }
    else
    {
      v.aD = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(on ? vD : vz, (int)o, 0, 2));
      v.a0 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(on ? v0 : vz, (int)o, 0, 2));
      v.ap = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(on ? v1 : vz, (int)o, 0, 2));
      v.aq = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(on ? vq : vz, (int)o, 0, 0));
      v.an = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(on ? vn : vz, (int)(o + dnv), 0, 0));
      v.ae = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(on ? v1 : vz, (int)(o + eov), 0, 0));
    }
  };
  constexpr bool VPF = VAL == 2;  // value streams one plane ahead
  Vals vs[2];
  double amD = 0.0;  // VAL: the mirrored -D value (the +D value of the row below)
  raw pm{};
  if (zg0 > 0)
  {
    bload(rs, vo - Db, pm);  // (plane 0 of the grid: no -D neighbour)
    if constexpr (VAL) amD = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(vD, (int)(vv - Dv), 0, 0));
  }
  raw sl[NS];
  bload(rs, vo, sl[0]);
#pragma unroll
  for (int k = 1; k <= PF; ++k) bload(zg0 + k < mp.gz ? rs : r0, vo + (unsigned)k * Db, sl[k]);
  Gath gs[2];
  if constexpr (PG) gather(vo, gs[0]);
  if constexpr (VPF) vload(vv, vs[0], true);
  if (!pre(x)) return;
  double pmv = zg0 > 0 ? x.val(pm) : 0.0;
  auto body = [&](int z, const raw &pcur, const raw &pd, raw &pf, Gath &gc, Gath &gn, Vals &vc_, Vals &vn_) {
    if constexpr (PG)
      gather(vo + Db, gn);
    else
      gather(vo, gc);
    if constexpr (VAL == 1 || VAL >= 4) vload(vv, vc_, true);
    const int zg = z + mp.gz0;
    if (VAL == 5 && (mp.cache & 4))
      bload_nt(zg + PF + 1 < mp.gz ? rs : r0, vo + (unsigned)(PF + 1) * Db, pf);
    else
      bload(zg + PF + 1 < mp.gz ? rs : r0, vo + (unsigned)(PF + 1) * Db, pf);
    if constexpr (VPF) vload(vv + Dv, vn_, z + 1 < z1);
    double acc = 0.0;
    const double vc = x.val(pcur), ve = x.val(gc.eg);
    const double vl = lane_shift_or<false>(vc, ve), vr = lane_shift_or<true>(vc, ve);
    if constexpr (VAL)
    {
      const double am = lane_shift_or<false>(vc_.ap, vc_.ae);
      acc += amD * pmv;
      acc += vc_.an * x.val(gc.xn);
      acc += am * vl;
      acc += vc_.a0 * vc;
      acc += vc_.ap * vr;
      acc += vc_.aq * x.val(gc.xq);
      acc += vc_.aD * x.val(pd);
      amD = vc_.aD;
    }
    else
    {
      acc += mp.cD * pmv;
      acc += mp.cn * x.val(gc.xn);
      acc += mp.c1 * vl;
      acc += mp.c0 * vc;
      acc += mp.c1 * vr;
      acc += mp.cq * x.val(gc.xq);
      acc += mp.cD * x.val(pd);
    }
    epi(w - own32, w, acc, pcur);
    pmv = vc;
    w += D;
    vo += Db;
    vv += Dv;
  };
  static_assert(!PG || NS % 2 == 0, "gather prefetch: an even number of bodies per trip");
  static_assert(!VPF || NS % 2 == 0, "value prefetch: an even number of bodies per trip");
  int z = z0;
  for (; z + NS - 1 < z1; z += NS)
  {
#pragma unroll
    for (int k = 0; k < NS; ++k)
      body(z + k, sl[k], sl[(k + 1) % NS], sl[(k + PF + 1) % NS], gs[PG ? k & 1 : 0], gs[PG ? (k + 1) & 1 : 1],
           vs[VPF ? k & 1 : 0], vs[VPF ? (k + 1) & 1 : 1]);
  }
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (z + k < z1)
      body(z + k, sl[k], sl[(k + 1) % NS], sl[(k + PF + 1) % NS], gs[PG ? k & 1 : 0], gs[PG ? (k + 1) & 1 : 1],
           vs[VPF ? k & 1 : 0], vs[VPF ? (k + 1) & 1 : 1]);
}

// Value march with TWO grid lines per wave (march variant 22; round 6): lane = x of a 64-x run, the
// wave's rows (x, y0) and (x, y0 + 1) of every plane it marches (y0 even; mp.ncol counts line PAIRS).
// Per plane and lane, two rows of variant 15 (the pair pack through 64-bit addresses, the +D operand
// loaded, the centre and -D carried), except that each line's neighbour across the pair comes from
// registers: line y0's +nx operand is line y0 + 1's centre, line y0 + 1's -nx operand is line y0's
// centre and its mirrored -nx value a(w + nx, w) = a(w, w + nx) is line y0's own (+1, +nx) pack
// entry.  Gathered: line y0 - 1's operand and mirrored value, line y0 + 2's operand -- half of the
// gathers of variant 15, whose mirrored value gathers cost 13 us at 256^3 (section 4e ablation).  Every
// row sums the same products in the same order as variant 15 (bitwise its rows); the launch's three
// sums add the rows in another order (each lane adds its two rows per plane).
// The 2-line fused march is the default on ranks of at least EIG_MARCH_2L_MIN_ROWS rows: 256^3 (16.8 M
// rows) 206.5-206.8 us vs 223.5 us for variant 15 (profiles/r06e_sweep256_2lines.jsonl, 0.65 of HBM),
// but 2 M-row grids (128^3, one rank's 256^2 x 32 slab) 28.2-28.4 vs 27.7-27.9 us: fewer, longer
// wave chains cost more there than the halved gathers save.  256^2 slabs (profiles/r06m_threshold.jsonl):
// 4 M rows 47.1 vs 46.1 us, 6 M rows 84.3 vs 89.8 us, 8 M rows 111.7 vs 116.7 us; with two plane runs
// per column on wide planes (march_plan, round 6) 4 M rows 45.6 vs 46.0 us, 2 M rows 27.6 either way --
// the threshold is 4 M.
constexpr bool kMarch2lDefault = true;
constexpr bool is_march2l(int uni) { return uni == 22 || uni == 23 || uni == 24; }

template <class X, class EPI, class PRE>
__device__ __forceinline__ void march_rows_geo2_2l(const SellB1 &A, const MarchPlan &mp, i64 own, int lane, int wave,
                                                   X x, EPI &epi, PRE &pre)
{
  typedef typename X::raw raw;
  constexpr unsigned SZ = sizeof(raw);
  const int D = (int)mp.D, own32 = (int)own, gx = mp.gx;
  const int item = (int)swizzled_block() * kWaves + wave;
  if (item >= mp.ncol * mp.nseg) return;
  const int col2 = item % mp.ncol, seg = item / mp.ncol;
  const int xcols = gx / 64;
  const int x0 = (col2 % xcols) * 64, y0 = (col2 / xcols) * 2;
  const int z0 = (int)(mp.zb + seg * mp.nplanes / mp.nseg), z1 = (int)(mp.zb + (seg + 1) * mp.nplanes / mp.nseg);
  const unsigned nbytes = (unsigned)(A.xlast + 1) * SZ;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(x.ptr()), 0, (int)nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(x.ptr()), 0, 0, 0x00020000);
  // line y0 - 1 (operand + mirrored value gathered) and line y0 + 2 (operand gathered)
  const bool has_n = mp.dn && y0 > 0, has_q = mp.dq && y0 + 2 < mp.gy;
  const __amdgpu_buffer_rsrc_t rn = has_n ? rs : r0, rq = has_q ? rs : r0;
  constexpr unsigned kOut = 0x80000000u;
  const unsigned eoff = lane == 0 ? (x0 > 0 ? 0u - SZ : kOut) : lane == 63 ? (x0 + 64 < gx ? SZ : kOut) : kOut;
  const unsigned dnb = (unsigned)mp.dn * SZ, dqb = (unsigned)mp.dq * SZ, Db = (unsigned)D * SZ, nxb = (unsigned)gx * SZ;
  int w = own32 + y0 * gx + x0 + lane + z0 * D;  // line y0's row; line y0 + 1's at w + gx
  unsigned vo = (unsigned)w * SZ;
  const int zg0 = z0 + mp.gz0;
  const SymImg &S = A.sym;
  const dpair *P01 = reinterpret_cast<const dpair *>(mp.pack), *P23 = P01 + S.ld;
  const bool le = lane == 0 && x0 > 0;  // lane 0's mirrored -1 value (row x0 - 1) exists
  double amD0 = 0.0, amD1 = 0.0;
  raw pm0{}, pm1{};
  if (zg0 > 0)
  {
    bload(rs, vo - Db, pm0);
    bload(rs, vo + nxb - Db, pm1);
    amD0 = P01[w - D].x;
    amD1 = P01[w + gx - D].x;
  }
  raw c0, c1;
  bload(rs, vo, c0);
  bload(rs, vo + nxb, c1);
  if (!pre(x)) return;
  double pmv0 = zg0 > 0 ? x.val(pm0) : 0.0, pmv1 = zg0 > 0 ? x.val(pm1) : 0.0;
  for (int z = z0; z < z1; ++z)
  {
    const int zg = z + mp.gz0;
    raw eg0, eg1, xn0, xq1, d0, d1;
    bload(rs, vo + eoff, eg0);
    bload(rs, vo + nxb + eoff, eg1);
    bload(rn, vo + dnb, xn0);
    bload(rq, vo + nxb + dqb, xq1);
    const dpair p0a = (mp.cache & 2) ? P01[w] : __builtin_nontemporal_load(P01 + w), p0b = P23[w];
    const dpair p1a = (mp.cache & 2) ? P01[w + gx] : __builtin_nontemporal_load(P01 + w + gx), p1b = P23[w + gx];
    const double an0 = has_n ? P23[w + mp.dn].y : 0.0;
    const double ae0 = le ? P23[w - 1].x : 0.0, ae1 = le ? P23[w + gx - 1].x : 0.0;
    const __amdgpu_buffer_rsrc_t rd = zg + 1 < mp.gz ? rs : r0;
    bload(rd, vo + Db, d0);
    bload(rd, vo + nxb + Db, d1);
    const double vc0 = x.val(c0), vc1 = x.val(c1);
    double acc0 = 0.0, acc1 = 0.0;
    {
      const double ve = x.val(eg0);
      const double vl = lane_shift_or<false>(vc0, ve), vr = lane_shift_or<true>(vc0, ve);
      const double am = lane_shift_or<false>(p0b.x, ae0);
      acc0 += amD0 * pmv0;
      acc0 += an0 * x.val(xn0);
      acc0 += am * vl;
      acc0 += p0a.y * vc0;
      acc0 += p0b.x * vr;
      acc0 += p0b.y * vc1;  // +nx: line y0 + 1's centre
      acc0 += p0a.x * x.val(d0);
    }
    {
      const double ve = x.val(eg1);
      const double vl = lane_shift_or<false>(vc1, ve), vr = lane_shift_or<true>(vc1, ve);
      const double am = lane_shift_or<false>(p1b.x, ae1);
      acc1 += amD1 * pmv1;
      acc1 += p0b.y * vc0;  // -nx: line y0's centre, mirrored value = line y0's +nx entry
      acc1 += am * vl;
      acc1 += p1a.y * vc1;
      acc1 += p1b.x * vr;
      acc1 += p1b.y * x.val(xq1);
      acc1 += p1a.x * x.val(d1);
    }
    epi(w - own32, w, acc0, c0);
    epi(w + gx - own32, w + gx, acc1, c1);
    pmv0 = vc0;
    pmv1 = vc1;
    amD0 = p0a.x;
    amD1 = p1a.x;
    c0 = d0;
    c1 = d1;
    w += D;
    vo += Db;
  }
}

// Box march for the P1 Kuhn 15-point stencil (march variant 12; config C5's K and M, any values): the
// band's offsets are a D + b nx + c with (a, b, c) in the Kuhn edge set {0, +-e_i, +-(e_i + e_j),
// +-(1, 1, 1)} and every row stores exactly its in-grid neighbours among them (eig_mat_s::sym_box27,
// checked at upload).  A wave owns 64 consecutive x of one grid line (nx a multiple of 64) and marches
// z, keeping the operand lines it needs in registers as values x.val (the fused step's u_k):
//   plane z - 1: lines y - 1, y        plane z: y - 1, y, y + 1        plane z + 1: y, y + 1
// each line with one edge register (lane 0: the row at x0 - 1, lane 63: x0 + 64; DPP lane shifts take
// it as the "old" operand).  Per plane only plane z + 1's three lines are loaded (y: the stream, y +- 1:
// gathers the neighbouring columns streamed, L2 hits); the rest are carried (z + 1 -> z -> z - 1).
// Values: the row's 8 upper band arrays streamed once (0, +1, +nx, +nx+1, +D, +D+1, +D+nx, +D+nx+1);
// the mirrored lower entries from the rows below: -1 by the lane shift of the +1 stream, -D / -D-1
// carried from the previous plane's +D / +D+1 streams, -nx / -nx-1 / -D-nx / -D-nx-1 gathered at line
// y - 1 (planes z and z - 1).  Missing neighbours read as exact zeros (zero-record descriptors for
// lines / planes outside the grid, out-of-range edge offsets at x = 0 / nx - 1), so each row sums its
// stored entries in ascending-column order bit for bit as the reference row loop.
constexpr unsigned kKuhn15 = (1u << 0) | (1u << 1) | (1u << 3) | (1u << 4) | (1u << 9) | (1u << 10) | (1u << 12) |
                             (1u << 13) | (1u << 14) | (1u << 16) | (1u << 17) | (1u << 22) | (1u << 23) |
                             (1u << 25) | (1u << 26);
// KP (march variant 16): the values from the Kuhn pack (mp.pack: four arrays of value pairs (0, +1),
// (+nx, +nx+1), (+D, +D+1), (+D+nx, +D+nx+1) per window row -- 4 instead of 8 16-B/8-B streams and
// 2 instead of 4 gathers) through 64-bit global addresses, lane 0's edge values by exec-masked loads.
// LX (march variant 20, the pack): a workgroup's 4 waves march the SAME 64 x of 4 consecutive lines
// y0 .. y0 + 3 (instead of 4 x-runs of one line), and every line a wave streams -- its operand line of
// plane z + 1 and its pack pairs (+nx, +nx+1) of plane z and (+D+nx, +D+nx+1) of plane z - 1 -- goes
// through LDS to the waves of lines y +- 1 (double-buffered, one barrier per plane): only lines
// y0 - 1 and y0 + 4 are still gathered from L2, 2 of the 8 line gathers per plane of the workgroup
// (the gathers that miss L2 were the Kuhn step's 1.32x read excess, profiles/r04af_kuhn_*).  Lines
// per grid a multiple of 4; the same products in the same order as variant 16 (bitwise).
template <bool KP, bool LX, class X, class EPI, class PRE>
__device__ __forceinline__ void march_rows_kuhn(const SellB1 &A, const MarchPlan &mp, i64 own, int lane, int wave,
                                                X x, EPI &epi, PRE &pre)
{
  typedef typename X::raw raw;
  constexpr unsigned SZ = sizeof(raw);
  constexpr unsigned kOut = 0x80000000u;
  const int D = (int)mp.D, own32 = (int)own, gx = mp.gx;
  int col, seg;
  if constexpr (LX)
  {
    // workgroup -> (x run, group of 4 lines, plane run); workgroup-uniform, so every wave of it reaches
    // the same barriers
    const int nxc = gx / 64, per = nxc * (mp.gy / 4);
    const int wg = (int)swizzled_block();
    if (wg >= per * mp.nseg) return;
    seg = wg / per;
    const int r = wg % per;
    col = ((r / nxc) * 4 + wave) * nxc + r % nxc;
  }
  else
  {
    const int item = (int)swizzled_block() * kWaves + wave;
    if (item >= mp.ncol * mp.nseg) return;
    col = item % mp.ncol;
    seg = item / mp.ncol;
  }
  const int z0 = (int)(mp.zb + seg * mp.nplanes / mp.nseg), z1 = (int)(mp.zb + (seg + 1) * mp.nplanes / mp.nseg);
  const unsigned nbytes = (unsigned)(A.xlast + 1) * SZ;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(x.ptr()), 0, (int)nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(x.ptr()), 0, 0, 0x00020000);
  const int x0 = (col * 64) % gx, yw = (col * 64) / gx;
  const __amdgpu_buffer_rsrc_t rm = yw > 0 ? rs : r0, rp = yw < mp.gy - 1 ? rs : r0;  // lines y - 1, y + 1
  const unsigned eoff = lane == 0 ? (x0 > 0 ? 0u - SZ : kOut) : lane == 63 ? (x0 + 64 < gx ? SZ : kOut) : kOut;
  const unsigned nxb = (unsigned)gx * SZ, Db = (unsigned)D * SZ;
  int w = own32 + col * 64 + lane + z0 * D;
  unsigned vo = (unsigned)w * SZ;
  const int zg0 = z0 + mp.gz0;
  // value arrays (8-B window-indexed slots): one descriptor per upper array, zero-record where absent
  const SymImg &S = A.sym;
  const unsigned vbytes = (unsigned)S.ld * 8u;
  auto arr = [&](int pos, bool on) {
    const int j = mp.kj[pos];
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(S.val + (i64)(j >= 0 ? j : 0) * S.ld), 0,
                                             on && j >= 0 ? (int)vbytes : 0, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t a0d = arr(13, true), a1d = arr(14, true), aNd = arr(16, true), aN1d = arr(17, true),
                               aDd = arr(22, true), aD1d = arr(23, true), aDNd = arr(25, true), aDN1d = arr(26, true),
                               aNm = arr(16, yw > 0), aN1m = arr(17, yw > 0), vz = arr(13, false);
  const unsigned eov = lane == 0 && x0 > 0 ? 0u - 8u : kOut;  // lane 0: the value slot at x0 - 1
  const unsigned nxv = (unsigned)gx * 8u, Dv = (unsigned)D * 8u;
  unsigned vv = (unsigned)w * 8u;
  auto ld8 = [&](__amdgpu_buffer_rsrc_t r, unsigned o) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)o, 0, 0));
  };
  auto ld8nt = [&](__amdgpu_buffer_rsrc_t r, unsigned o) {  // once-read streams: nontemporal
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)o, 0, 2));
  };
  // operand lines: raw loads first (the fused prologue sets x.c meanwhile), values after
  const bool below = zg0 > 0;
  raw rAm, rAme, rA0, rA0e, rBm, rBme, rB0, rB0e, rBp, rBpe;
  {
    const __amdgpu_buffer_rsrc_t p0 = below ? rs : r0, pm = below ? rm : r0;
    bload(pm, vo - Db - nxb, rAm);
    bload(pm, vo - Db - nxb + eoff, rAme);
    bload(p0, vo - Db, rA0);
    bload(p0, vo - Db + eoff, rA0e);
  }
  bload(rm, vo - nxb, rBm);
  bload(rm, vo - nxb + eoff, rBme);
  bload(rs, vo, rB0);
  bload(rs, vo + eoff, rB0e);
  bload(rp, vo + nxb, rBp);
  bload(rp, vo + nxb + eoff, rBpe);
  // Kuhn pack: array q of pairs at byte 16 (q ld + w), one descriptor (32-bit offsets)
  const __amdgpu_buffer_rsrc_t kp = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(KP && mp.pack ? mp.pack : S.val), 0, KP && mp.pack ? (int)(8u * vbytes) : 0, 0x00020000);
  const unsigned kq = 2u * vbytes;  // bytes per pair array
  auto kl = [&](int q, unsigned row_off) {  // pair of array q at byte offset row_off (= 16 row)
    return __builtin_bit_cast(dpair, __builtin_amdgcn_raw_buffer_load_b128(kp, (int)(row_off + (unsigned)q * kq), 0, 0));
  };
  auto kle = [&](int q, unsigned row_off, bool on) {  // lane 0's edge value (.y); others: out of range
    const unsigned o = on ? row_off + (unsigned)q * kq + 8u : kOut;
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(kp, (int)o, 0, 0));
  };
  // the once-read pair streams (0, +1) and (+D, +D+1): default cache policy.  Measured against
  // nontemporal loads at 256^3 (P1 K, profiles/r04v_p1k.jsonl, r04w_p1k.jsonl): fused step 336.0 vs
  // 340.1 us and 337.0 vs 349.2 us on two boxes, eig_mv 282.9 vs 285.9 us -- although FETCH_SIZE
  // rises (100.7 vs 97.6 B per row; why the default policy is faster is not established)
  auto klnt = [&](int q, unsigned row_off) {
    return __builtin_bit_cast(dpair, __builtin_amdgcn_raw_buffer_load_b128(kp, (int)(row_off + (unsigned)q * kq), 0, 0));
  };
  const unsigned nxk = 2u * nxv, Dk = 2u * Dv;
  const bool le = lane == 0 && x0 > 0;  // lane 0's value edge (row x0 - 1) exists
  double aDp = 0.0, aD1p = 0.0, aD1pe = 0.0;
  if constexpr (KP)
  {
    if (below)
    {
      const dpair k2 = kl(2, 2u * vv - Dk);
      aDp = k2.x;
      aD1p = k2.y;
      aD1pe = kle(2, 2u * vv - Dk - 16u, le);
    }
  }
  else
  {
    aDp = below ? ld8(aDd, vv - Dv) : 0.0;
    aD1p = below ? ld8(aD1d, vv - Dv) : 0.0;
    aD1pe = below ? ld8(aD1d, vv - Dv + eov) : 0.0;
  }
  // LX: the line exchange (raw operand line of plane z + 1, pack pairs (+nx, +nx+1) of plane z and
  // (+D+nx, +D+nx+1) of plane z - 1 per wave), double-buffered by plane parity
  __shared__ raw lx_c[LX ? 2 : 1][LX ? kWaves : 1][64];
  __shared__ dpair lx_k1[LX ? 2 : 1][LX ? kWaves : 1][64], lx_k3[LX ? 2 : 1][LX ? kWaves : 1][64];
  const bool lx_lo = LX && wave > 0, lx_hi = LX && wave < kWaves - 1;  // line y - 1 / y + 1 in this workgroup
  dpair k3prev = {0.0, 0.0};  // LX: this line's (+D+nx, +D+nx+1) pair of the previous plane
  if constexpr (LX && KP)
  {
    if (below) k3prev = kl(3, 2u * vv - Dk);
  }
  if (!pre(x)) return;
  double Am = x.val(rAm), Ame = x.val(rAme), A0 = x.val(rA0), A0e = x.val(rA0e), Bm = x.val(rBm), Bme = x.val(rBme),
         Bp = x.val(rBp), Bpe = x.val(rBpe);
  double B0 = x.val(rB0), B0e = x.val(rB0e);
  raw pB0 = rB0;
  for (int z = z0; z < z1; ++z)
  {
    const int zg = z + mp.gz0;
    const bool up = zg + 1 < mp.gz, dn = zg > 0;
    raw rC0, rC0e, rCp, rCpe, rCm, rCme;
    {
      const __amdgpu_buffer_rsrc_t q0 = up ? rs : r0, qp = up ? rp : r0, qm = up ? rm : r0;
      bload(q0, vo + Db, rC0);
      bload(q0, vo + Db + eoff, rC0e);
      if (!lx_hi) bload(qp, vo + Db + nxb, rCp);
      bload(qp, vo + Db + nxb + eoff, rCpe);
      if (!lx_lo) bload(qm, vo + Db - nxb, rCm);
      bload(qm, vo + Db - nxb + eoff, rCme);
    }
    // the row's upper values (once-read streams nontemporal; +nx.. arrays are re-read by line y + 1)
    double a0, a1, aN, aN1, aD, aD1, aDN, aDN1, a1e = 0.0, aD1e = 0.0;
    double aNl = 0.0, aN1l = 0.0, aN1le = 0.0, aDNl = 0.0, aDN1l = 0.0, aDN1le = 0.0;
    if constexpr (KP)
    {
      const unsigned ko = 2u * vv;
      const dpair k0 = klnt(0, ko), k1 = kl(1, ko), k2 = klnt(2, ko), k3 = kl(3, ko);
      a0 = k0.x, a1 = k0.y, aN = k1.x, aN1 = k1.y, aD = k2.x, aD1 = k2.y, aDN = k3.x, aDN1 = k3.y;
      a1e = kle(0, ko - 16u, le);
      aD1e = kle(2, ko - 16u, le);
      // mirrored lower entries at line y - 1 (plane z: -nx, -nx-1; plane z - 1: -D-nx, -D-nx-1): the
      // wave-uniform line / plane conditions pick an out-of-range offset (zeros, no traffic)
      const bool ym = yw > 0, dm = dn && yw > 0;
      dpair kn = {0.0, 0.0}, kd = {0.0, 0.0};
      if (!lx_lo)
      {
        kn = __builtin_bit_cast(dpair,
                                __builtin_amdgcn_raw_buffer_load_b128(kp, (int)(ym ? ko - nxk + kq : kOut), 0, 0));
        kd = __builtin_bit_cast(
            dpair, __builtin_amdgcn_raw_buffer_load_b128(kp, (int)(dm ? ko - Dk - nxk + 3u * kq : kOut), 0, 0));
      }
      aN1le = kle(1, ko - nxk - 16u, le && ym);
      aDN1le = kle(3, ko - Dk - nxk - 16u, le && dm);
      if constexpr (LX)
      {
        // this wave's lines to the workgroup, then the neighbours' from it
        const int b = z & 1;
        lx_c[b][wave][lane] = rC0;
        lx_k1[b][wave][lane] = k1;
        lx_k3[b][wave][lane] = k3prev;
        k3prev = k3;
        __syncthreads();
        if (lx_hi) rCp = lx_c[b][wave + 1][lane];
        if (lx_lo)
        {
          rCm = lx_c[b][wave - 1][lane];
          kn = lx_k1[b][wave - 1][lane];
          kd = dn ? lx_k3[b][wave - 1][lane] : dpair{0.0, 0.0};
        }
      }
      aNl = kn.x, aN1l = kn.y;
      aDNl = kd.x, aDN1l = kd.y;
    }
    else
    {
      a0 = ld8nt(a0d, vv), a1 = ld8nt(a1d, vv), aN = ld8(aNd, vv), aN1 = ld8(aN1d, vv);
      aD = ld8nt(aDd, vv), aD1 = ld8nt(aD1d, vv), aDN = ld8(aDNd, vv), aDN1 = ld8(aDN1d, vv);
      a1e = ld8(a1d, vv + eov), aD1e = ld8(aD1d, vv + eov);
      // mirrored lower entries at line y - 1 (plane z: -nx, -nx-1; plane z - 1: -D-nx, -D-nx-1)
      aNl = ld8(aNm, vv - nxv), aN1l = ld8(aN1m, vv - nxv), aN1le = ld8(aN1m, vv - nxv + eov);
      const __amdgpu_buffer_rsrc_t dnm = dn && yw > 0 ? aDNd : vz, dn1m = dn && yw > 0 ? aDN1d : vz;
      aDNl = ld8(dnm, vv - Dv - nxv), aDN1l = ld8(dn1m, vv - Dv - nxv), aDN1le = ld8(dn1m, vv - Dv - nxv + eov);
    }
    const double C0 = x.val(rC0), C0e = x.val(rC0e), Cp = x.val(rCp), Cpe = x.val(rCpe);
    double acc = 0.0;
    acc += lane_shift_or<false>(aDN1l, aDN1le) * lane_shift_or<false>(Am, Ame);  // (-1, -1, -1)
    acc += aDNl * Am;                                                            // (-1, -1,  0)
    acc += lane_shift_or<false>(aD1p, aD1pe) * lane_shift_or<false>(A0, A0e);    // (-1,  0, -1)
    acc += aDp * A0;                                                             // (-1,  0,  0)
    acc += lane_shift_or<false>(aN1l, aN1le) * lane_shift_or<false>(Bm, Bme);    // ( 0, -1, -1)
    acc += aNl * Bm;                                                             // ( 0, -1,  0)
    acc += lane_shift_or<false>(a1, a1e) * lane_shift_or<false>(B0, B0e);        // ( 0,  0, -1)
    acc += a0 * B0;                                                              // ( 0,  0,  0)
    acc += a1 * lane_shift_or<true>(B0, B0e);                                    // ( 0,  0, +1)
    acc += aN * Bp;                                                              // ( 0, +1,  0)
    acc += aN1 * lane_shift_or<true>(Bp, Bpe);                                   // ( 0, +1, +1)
    acc += aD * C0;                                                              // (+1,  0,  0)
    acc += aD1 * lane_shift_or<true>(C0, C0e);                                   // (+1,  0, +1)
    acc += aDN * Cp;                                                             // (+1, +1,  0)
    acc += aDN1 * lane_shift_or<true>(Cp, Cpe);                                  // (+1, +1, +1)
    epi(w - own32, w, acc, pB0);
    // carry z + 1 -> z -> z - 1
    Am = Bm, Ame = Bme, A0 = B0, A0e = B0e;
    Bm = x.val(rCm), Bme = x.val(rCme);
    B0 = C0, B0e = C0e, pB0 = rC0;
    Bp = Cp, Bpe = Cpe;
    aDp = aD, aD1p = aD1, aD1pe = aD1e;
    w += D;
    vo += Db;
    vv += Dv;
  }
}

// The rows of this wave's work item, in plane order: epi(r, w, acc, centre) gets each row's sum
// and its own operand x[w] (raw: a double, or the (t, u) pair of the fused step).
// The first entry of both far spans is issued with the row's streams, so a 7-point row waits
// once.  SPAN1: each far span holds at most one offset (3-D 7-point, 2-D 5-point), so the generic
// span loops are compiled out.  (Measured and dropped: issuing the far spans offset group by
// offset group after the near math; prefetching the next plane's streams, or its far-span
// operands, one iteration ahead -- both spill in the fused kernel and gave nothing in the others;
// y-line workgroup grouping with a barrier per plane; temporal result stores.)
// UNI (uniform band, SPAN1 only): the band values come from the plan's constants -- the values the
// arrays hold at every slot the mask admits -- so only the row mask and the operands are streamed;
// the same products and sums in the same order, bit for bit.  (Measured and dropped for UNI: issuing
// plane z + 1's mask / gathers / edge operand before plane z's arithmetic -- 256^3 fused step 145 vs
// 137 us at the 7 waves / SIMD it needs, 128^3 28.0 vs 30.7: profiles/r03bc_latency.jsonl.)
template <class MT, int KC, bool SPAN1, int UNI, class X, class EPI, class PRE = MarchNoPre>
__device__ __forceinline__ void march_rows(const SellB1 &A, const MarchPlan &mp, i64 own, int lane, int wave,
                                           const X &x, EPI &epi, PRE &&pre = PRE{})
{
  static_assert(!UNI || SPAN1 || UNI == 12 || UNI == 16 || UNI == 19 || UNI == 20 || is_march2l(UNI),
                "uniform-band march: far spans of at most one offset");
  if constexpr (UNI == 12 || UNI == 16 || UNI == 19 || UNI == 20)
  {
    march_rows_kuhn<UNI != 12, UNI == 20>(A, mp, own, lane, wave, x, epi, pre);
    return;
  }
  else if constexpr (is_march2l(UNI))
  {
    march_rows_geo2_2l(A, mp, own, lane, wave, x, epi, pre);
    return;
  }

  else if constexpr (UNI >= 3)
  {
    // 3, 4, 5: +D operand 1, 2, 3 planes ahead; 6: 3 planes ahead and the gathers one plane ahead
    if constexpr (UNI >= 10)  // 10, 11: the value march (band arrays streamed), 11 one plane ahead, 13 packed
      march_rows_geo2<0, false, UNI == 14 ? 4 : UNI == 15 || UNI == 18 ? 5 : UNI - 9>(A, mp, own, lane, wave, x, epi, pre);
    else if constexpr (UNI >= 7)  // 7, 8, 9: march_rows_geo2 with the prefetches of 3, 4, 6
      march_rows_geo2<UNI == 9 ? 2 : UNI - 7, UNI == 9, 0>(A, mp, own, lane, wave, x, epi, pre);
    else
      march_rows_geo<UNI == 6 ? 2 : UNI - 3, UNI == 6>(A, mp, own, lane, wave, x, epi);
    return;
  }
  constexpr bool GEO = UNI == 2;
  typedef typename X::raw raw;
  // 32-bit row / window indices (window < 2^31, enforced at upload) keep the address math short
  const SymImg &S = A.sym;
  const int xl = (int)A.xlast, D = (int)mp.D, ldl = (int)(S.ld - 1), own32 = (int)own, mrows = (int)mp.mrows;
  const int nd = S.nd;
  const double *UD = S.val + (i64)S.dj[nd - 1] * S.ld;
  const double *U1 = S.val + (i64)S.j1 * S.ld;
  const double *U0 = S.val + (i64)(S.j0 >= 0 ? S.j0 : 0) * S.ld;
  const MT *mask = static_cast<const MT *>(S.mask);
  const int item = (int)swizzled_block() * kWaves + wave;
  if (item >= mp.ncol * mp.nseg) return;
  const int col = item % mp.ncol, seg = item / mp.ncol;
  const int z0 = (int)(mp.zb + seg * mp.nplanes / mp.nseg), z1 = (int)(mp.zb + (seg + 1) * mp.nplanes / mp.nseg);
  auto cx = [&](int g) -> unsigned { return g < 0 ? 0u : (unsigned)(g > xl ? xl : g); };
  auto cv = [&](int g) -> unsigned { return g < 0 ? 0u : (unsigned)(g > ldl ? ldl : g); };
  const int kn0 = 1, kn1 = S.klo, kp0 = S.khi, kp1 = nd - 1;  // far spans (-D, -1) and (+1, +D)
  // GEO: the lane's row keeps its (x, y) in every plane; bit k of the mask = the neighbour at
  // off[k] lies in the grid (verified row by row at upload)
  unsigned gxy = 0;
  if constexpr (GEO)
  {
    const int pr = col * 64 + lane, gxc = pr % mp.gx, gyc = pr / mp.gx;
    // offsets ascending: -D, (-nx), -1, 0, +1, (+nx), +D -- the far-span bits only when present
    unsigned b = 0;
    int k = 1;
    if (mp.dn) b |= (gyc > 0 ? 1u : 0u) << k++;
    b |= (gxc > 0 ? 1u : 0u) << k++;
    b |= 1u << k++;
    b |= (gxc < mp.gx - 1 ? 1u : 0u) << k++;
    if (mp.dq) b |= (gyc < mp.gy - 1 ? 1u : 0u) << k++;
    gxy = b;
  }
  struct Stream {
    unsigned m;
    double aD, a0, ap;
    raw pD;
  };
  // streams read exactly once (the row mask, the 0 / +1 / +D band values): nontemporal loads keep
  // them from evicting the (t, u) / band lines the neighbouring columns re-read from L2
  auto ld1 = [&](const double *p, unsigned i) { return __builtin_nontemporal_load(p + i); };
  auto load_stream = [&](int w, int z, Stream &st) {
    const int r = w - own32;
    const unsigned wv = (unsigned)(w > ldl ? ldl : w);
    if constexpr (GEO)
    {
      const int zg = z + mp.gz0;  // (z: the wave's plane on this rank)
      st.m = gxy | (zg > 0 ? 1u : 0u) | (zg < mp.gz - 1 ? 1u << kp1 : 0u);
    }
    else
      st.m = r < mrows ? (unsigned)__builtin_nontemporal_load(mask + (unsigned)r) : 0u;
    st.pD = x.load(cx(w + D));
    if constexpr (UNI)
    {
      st.aD = mp.cD;
      st.a0 = mp.c0;
      st.ap = mp.c1;
    }
    else
    {
      st.aD = ld1(UD, wv);
      st.a0 = S.j0 >= 0 ? ld1(U0, wv) : 0.0;
      st.ap = ld1(U1, wv);
    }
  };
  // carried operands: the -D operand (as its value x.val), its mirrored matrix entry, the centre
  int w = own32 + col * 64 + lane + z0 * D;
  double pmv = x.val(x.load(cx(w - D)));
  double amD = UNI ? mp.cD : UD[cv(w - D)];
  raw pcur = x.load(cx(w));
  Stream cur;
  const bool edge = lane == 0 || lane == 63;
  for (int z = z0; z < z1; ++z, w += D)
  {
    const int r = w - own32;
    const unsigned wv = (unsigned)(w > ldl ? ldl : w);
    load_stream(w, z, cur);
    // lanes 0 / 63: the row across the wave edge (one load for both), and lane 0's mirrored -1 entry
    raw eg;
    double ae = 0.0;
    if (edge) eg = x.load(cx(lane == 0 ? w - 1 : w + 1));
    if (lane == 0) ae = UNI ? mp.c1 : U1[cv(w - 1)];
    double an = 0.0, aq = 0.0;
    raw xn, xq;
    if (mp.dn)
    {
      const unsigned g = cx(w + mp.dn);  // (negative offset: the mirrored slot at the gathered row)
      an = UNI ? mp.cn : mp.Un[g];
      xn = x.load(g);
    }
    if (mp.dq)
    {
      aq = UNI ? mp.cq : mp.Uq[wv];
      xq = x.load(cx(w + mp.dq));
    }
    const unsigned m = cur.m;
    double acc = 0.0;
    if (m & 1u) acc += amD * pmv;
    if (mp.dn && ((m >> kn0) & 1u)) acc += an * x.val(xn);
    if (!SPAN1) sym_span<KC>(S, kn0 + 1, kn1, m, w, wv, x, xl, acc);
    // neighbours' operand VALUES shifted across lanes (x.val per lane, then moved: the same bits
    // as evaluating x.val on the shifted raw operand, at half the registers for pairs)
    const double vc = x.val(pcur);
    double vl = lane_shift<false>(vc), vr = lane_shift<true>(vc);
    double am = lane_shift<false>(cur.ap);
    if (edge)
    {
      const double ve = x.val(eg);
      if (lane == 0)
      {
        vl = ve;
        am = ae;
      }
      else
        vr = ve;
    }
    if (S.km1 >= 0 && ((m >> S.km1) & 1u)) acc += am * vl;
    if (S.k0 >= 0 && ((m >> S.k0) & 1u)) acc += cur.a0 * vc;
    if (S.kp1 >= 0 && ((m >> S.kp1) & 1u)) acc += cur.ap * vr;
    if (mp.dq && ((m >> kp0) & 1u)) acc += aq * x.val(xq);
    if (!SPAN1) sym_span<KC>(S, kp0 + 1, kp1, m, w, wv, x, xl, acc);
    if ((m >> kp1) & 1u) acc += cur.aD * x.val(cur.pD);
    epi(r, w, acc, pcur);
    pmv = vc;
    pcur = cur.pD;
    amD = cur.aD;
  }
}

// y[own + r] = (A x)[r] on the plane march (BCRSMatrix::mv; bitwise k_spmv_b1).
// resident waves per SIMD of the eig_mv / K1 march kernels (the box march holds ~90 VGPRs)
constexpr int march_mv_waves(int uni) { return uni == 12 || uni == 16 || uni == 19 || uni == 20 || is_march2l(uni) ? 5 : 8; }

template <class MT, bool SPAN1, int UNI>
__global__ __launch_bounds__(kStreamThreads, march_mv_waves(UNI)) void k_spmv_march(i64 nrows, i64 own, SellB1 A, MarchPlan mp,
                                                                  const double *__restrict__ x,
                                                                  double *__restrict__ y)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto epi = [&](int r, int w, double acc, double) {
    if constexpr (UNI >= 7)
      march_store(mp, acc, y + (unsigned)w);  // (geometric: whole planes)
    else if (UNI >= 3 || r < nrows)
      __builtin_nontemporal_store(acc, y + (unsigned)w);
  };
  march_rows<MT, 2, SPAN1, UNI>(A, mp, own, lane, wave, XPlain{x}, epi);
}

// Classic Lanczos kernel 1 on the plane march (same per-row arithmetic as k_lanczos_spmv_b1; the
// row's own u_j is the march's centre operand).
template <class MT, bool SPAN1, int UNI>
__global__ __launch_bounds__(kStreamThreads, march_mv_waves(UNI)) void k_lanczos_spmv_march(
    i64 nrows, i64 own, SellB1 A, MarchPlan mp, const double *__restrict__ u, const double *__restrict__ up,
    double *__restrict__ t, int j, const double *__restrict__ nsum, double *__restrict__ dot_out,
    double *__restrict__ beta_out, double *partials, unsigned *ticket)
{
  __shared__ double tot[1];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double beta = sqrt(nsum[j]);
  const double sig = 1.0 / beta;
  const double gam = (j > 0) ? beta * (1.0 / sqrt(nsum[j - 1])) : 0.0;
  double d = 0.0;
  auto epi = [&](int r, int w, double acc, double uv) {
    if (r < nrows)
    {
      double ti = acc * sig;
      if (j > 0) ti = ti - gam * up[(unsigned)w];
      __builtin_nontemporal_store(ti, t + (unsigned)w);
      d += ti * uv;
    }
  };
  march_rows<MT, 2, SPAN1, UNI>(A, mp, own, lane, wave, XPlain{u}, epi);
  double v[1] = {d};
  if (grid_sum<1, kStreamThreads>(v, partials, ticket, tot))
  {
    if (threadIdx.x == 0)
    {
      dot_out[0] = tot[0];
      if (beta_out) beta_out[0] = beta;
    }
  }
}

// Fused one-reduction step on the plane march (per-row arithmetic of k_lanczos_fused_b1).  A repair
// launch (fused_begin) takes the rows of the planes this launch marches.  Built for 7 waves / SIMD
// (72 VGPRs; at 8 the pair operands spill: -5 %).
// resident waves per SIMD the fused march kernels are built for (registers: no spills)
constexpr int march_fused_waves(int uni)
{
  return uni == 22 ? 5 : uni == 23 ? 4 : uni == 24 ? 6 : uni == 18 ? 7 : uni == 16 || uni == 20 ? 4 : uni == 12 || uni == 19 ? 5 : uni == 11 ? 5 : uni == 10 || uni >= 13 ? 6 : uni == 6 || uni == 9 ? 4 : uni == 5 ? 5 : uni == 4 || uni == 8 ? 6
       : uni == 3 || uni == 7 ? 7 : uni ? 8 : 7;
}

template <class MT, bool SPAN1, int UNI>
__global__ __launch_bounds__(kStreamThreads, march_fused_waves(UNI)) void k_lanczos_fused_march(
    i64 nrows, i64 own, SellB1 A, MarchPlan mp, const dpair *__restrict__ P, dpair *__restrict__ Pout, FusedArgs fa,
    double *__restrict__ out, double *partials, unsigned *ticket)
{
  __shared__ double tot[3];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double d = 0.0, q2 = 0.0, m2 = 0.0;
  if constexpr (UNI >= 7)
  {
    // geo2: the scalar prologue runs while the wave's first plane loads are in flight (the march
    // calls `pre` after issuing them); waves without a work item run it after the march returns
    FusedStep fs{};
    bool begun = false;
    auto epi = [&](int, int w, double acc, dpair pc) {
      const double uk = pc.x - fs.c * pc.y;
      double ti = (acc - fs.mu * uk) * fs.sig;
      if (fs.j > 0) ti = ti - fs.gam * pc.y;
      march_store(mp, dpair{ti, uk}, Pout + (unsigned)w);
      d += ti * uk;
      q2 += ti * ti;
      m2 += uk * uk;
    };
    auto pre = [&](XPair &x) {
      fs = fused_begin(fa);
      begun = true;
      x.c = fs.c;
      return fs.act == kFusedStep || fs.act == kFusedPost;
    };
    march_rows<MT, 2, SPAN1, UNI>(A, mp, own, lane, wave, XPair{P, 0.0}, epi, pre);
    if (!begun) fs = fused_begin(fa);
    if (fs.act == kFusedHalt || fs.act == kFusedNoop)
    {
      if (!(fa.xch & kXchPublish))
      {
        fused_idle(out);
        return;
      }
      d = q2 = m2 = 0.0;
    }
    if (fs.act == kFusedRepair)
    {
      const i64 r0 = mp.zb * mp.D, r1 = std::min<i64>(nrows, (mp.zb + mp.nplanes) * mp.D);
      m2 = fused_repair_rows(r0, r1, own, fs.c, P, Pout);
    }
    double v[3] = {d, q2, m2};
    fused_finish<8>(v, partials, ticket, tot, out, nullptr, fa);
    return;
  }
  const FusedStep fs = fused_begin(fa);
  if (fs.act == kFusedHalt || fs.act == kFusedNoop)
  {
    double z[3] = {0.0, 0.0, 0.0};
    if (fa.xch & kXchPublish) fused_finish<8>(z, partials, ticket, tot, out, nullptr, fa);
    else fused_idle(out);
    return;
  }
  const double c = fs.c, gam = fs.gam, sig = fs.sig, mu = fs.mu;
  const int k = fs.j;
  if (fs.act == kFusedRepair)
  {
    const i64 r0 = mp.zb * mp.D, r1 = std::min<i64>(nrows, (mp.zb + mp.nplanes) * mp.D);
    m2 = fused_repair_rows(r0, r1, own, c, P, Pout);
  }
  else
  {
    auto epi = [&](int r, int w, double acc, dpair pc) {
      if (UNI >= 3 || r < nrows)  // (geometric images cover whole planes: no row test)
      {
        const double uk = pc.x - c * pc.y;
        double ti = (acc - mu * uk) * sig;
        if (k > 0) ti = ti - gam * pc.y;
        __builtin_nontemporal_store(dpair{ti, uk}, Pout + (unsigned)w);
        d += ti * uk;
        q2 += ti * ti;
        m2 += uk * uk;
      }
    };
    march_rows<MT, 2, SPAN1, UNI>(A, mp, own, lane, wave, XPair{P, c}, epi);
  }
  double v[3] = {d, q2, m2};
  fused_finish<8>(v, partials, ticket, tot, out, nullptr, fa);
}

// ---------------------------------------------------------------------------------------------
// Pipelined one-reduction step, row half (restatement orc_lanczos_pipelined).  The
// step's SpMV multiplies t_{k-1} (S = A t_{k-1}, a plain eig_mv launch), which needs no scalar of the
// previous launch, so on N GPUs it runs while that launch's 3-value allreduce is in flight.  This
// kernel then applies the scalars (fused_begin: the same modes, prediction and repairs as the fused
// step) row by row:
//   u_k = t_{k-1} - c u_{k-1},  z_k = S - c z_{k-1}  (= A u_k),  t_k = (z_k - mu u_k) sig - gam u_{k-1}
// T (t) is updated in place; UZ holds the (u, z) pairs.  A repair writes T = u_k and keeps UZ (the
// launch after it has c = 0: u = T, z = S = A u_k exactly).  Bytes: 32 B read + 24 B written per row.
// Rows [0, n) are owned rows (pointers already offset to the owned part).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kStreamThreads) void k_lanczos_pipe(i64 n, double *__restrict__ T,
                                                                 dpair *__restrict__ UZ,
                                                                 const double *__restrict__ S, FusedArgs fa,
                                                                 double *__restrict__ out, double *partials,
                                                                 unsigned *ticket)
{
  __shared__ double tot[3];
  const FusedStep fs = fused_begin(fa);
  if (fs.act == kFusedHalt || fs.act == kFusedNoop)
  {
    fused_idle(out);
    return;
  }
  const double c = fs.c, gam = fs.gam, sig = fs.sig, mu = fs.mu;
  const bool k0 = fs.j > 0;
  const i64 stride = (i64)gridDim.x * kStreamThreads;
  double d = 0.0, q2 = 0.0, m2 = 0.0;
  if (fs.act == kFusedRepair)
  {
    for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n; i += stride)
    {
      const double u = T[i] - c * UZ[i].x;
      T[i] = u;
      m2 += u * u;
    }
  }
  else
  {
    auto row = [&](double t, double s, dpair uz, double &tn, dpair &uzn) {
      const double u = t - c * uz.x;
      const double z = s - c * uz.y;
      double ti = (z - mu * u) * sig;
      if (k0) ti = ti - gam * uz.x;
      tn = ti;
      uzn = dpair{u, z};
      d += ti * u;
      q2 += ti * ti;
      m2 += u * u;
    };
    // two rows per lane: 16-B loads of T and S, two 16-B (u, z) pairs (4 items in flight per lane
    // with all loads issued first measured no faster: the launch is HBM-bound at 56 B per row)
    const i64 n2 = n >> 1;
    double2 *T2 = reinterpret_cast<double2 *>(T);
    const double2 *S2 = reinterpret_cast<const double2 *>(S);
    for (i64 i = (i64)blockIdx.x * kStreamThreads + threadIdx.x; i < n2; i += stride)
    {
      const double2 t = T2[i], s = S2[i];
      const dpair a = UZ[2 * i], b = UZ[2 * i + 1];
      double2 tn;
      dpair an, bn;
      row(t.x, s.x, a, tn.x, an);
      row(t.y, s.y, b, tn.y, bn);
      T2[i] = tn;
      UZ[2 * i] = an;
      UZ[2 * i + 1] = bn;
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0)
    {
      double tn;
      dpair zn;
      row(T[n - 1], S[n - 1], UZ[n - 1], tn, zn);
      T[n - 1] = tn;
      UZ[n - 1] = zn;
    }
  }
  double v[3] = {d, q2, m2};
  if (grid_sum<3, kStreamThreads>(v, partials, ticket, tot))
  {
    if (threadIdx.x < 3) out[threadIdx.x] = tot[threadIdx.x];
  }
}

// ---------------------------------------------------------------------------------------------
// a2 SpMM Y = A X for one 8-column block of a MultiVector<double,8> (kernels_cpp.hh:626-657) on the
// band-image plane march.  Lane = (row rq = lane >> 2 of a 16-row wave column, column pair
// cp = lane & 3): every operand load of the wave reads 16 consecutive X rows = 1 KiB contiguous,
// the 4 lanes of a row share the row's band values and mask byte (one cache line per wave).  The
// wave marches its 16-row column through the planes like march_rows: the -D / centre operands are
// carried, the +D operand loaded once; the +-1 operands (and the mirrored -1 value) come from the
// lanes 4 apart by ds_bpermute (rows 0 / 15 of the wave load theirs); the +-N operands are L2 hits.
// Per column, each row sums its stored entries in ascending-column order with separately rounded
// products and sums: bitwise the reference loop.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double lane_from(double v, int src_lane)
{
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)b);
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// One column block per workgroup (blockIdx.y): sharing the band stream between 2 / 4 blocks measured
// equal / 6 % slower (m = 32 at 256^3) -- the vector streams bound the launch.
// DOT: also dp[8 qb + j] = X_j . Y_j over the rows (StandardLargest's :84-85 in one launch): each
// lane adds its row's own operand x its result, one deterministic grid sum per column block
// (partials part + grid.x * 8 qb, ticket tick + qb kTicketStride); Y is unchanged.
// DOT = 2: also the window Gram of Y (one column block, m = 8: StandardLargest's next MGS starts from
// it, k_mgs_la_gram) -- dots and Gram in one two-level grid sum (reduce_dev.h quad_gram_block).
template <class MT, int DOT = 0>
__global__ __launch_bounds__(kStreamThreads, DOT == 2 ? 5 : DOT ? 6 : 8) void k_spmm8_march(i64 nrows, i64 own, i64 ld, SellB1 A,
                                                                   MarchPlan mp, const double *__restrict__ X,
                                                                   double *__restrict__ Y, double *dp = nullptr,
                                                                   double *part = nullptr, unsigned *tick = nullptr,
                                                                   double *gram = nullptr, unsigned *zero_word = nullptr)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int qb = (int)blockIdx.y;  // column block
  const int rq = lane >> 2, cp = lane & 3;
  const SymImg &S = A.sym;
  const int xl = (int)A.xlast, D = (int)mp.D, ldl = (int)(S.ld - 1), own32 = (int)own, mrows = (int)mp.mrows;
  const int nd = S.nd;
  const double *UD = S.val + (i64)S.dj[nd - 1] * S.ld;
  const double *U1 = S.val + (i64)S.j1 * S.ld;
  const double *U0 = S.val + (i64)(S.j0 >= 0 ? S.j0 : 0) * S.ld;
  const MT *mask = static_cast<const MT *>(S.mask);
  const int item = (int)swizzled_block() * kWaves + wave;
  // (DOT: a wave past the last item joins the workgroup's reduction with an empty march)
  const bool live = item < mp.ncol * mp.nseg;
  if (!DOT && !live) return;
  const int col = item % mp.ncol, seg = item / mp.ncol;
  const int z0 = (int)(mp.zb + seg * mp.nplanes / mp.nseg);
  const int z1 = live ? (int)(mp.zb + (seg + 1) * mp.nplanes / mp.nseg) : z0;
  dpair dsum{0.0, 0.0};
  double gacc[2][8] = {};  // DOT == 2: this lane's share of the window Gram
  // column block qb, column pair cp: row g's operand at Xb[g]
  const dpair *Xb = reinterpret_cast<const dpair *>(X + (i64)qb * ld * 8) + cp;
  dpair *Yb = reinterpret_cast<dpair *>(Y + (i64)qb * ld * 8) + cp;
  auto xat = [&](int g) { return Xb[(unsigned)(g < 0 ? 0 : (g > xl ? xl : g)) * 4u]; };
  auto cv = [&](int g) -> unsigned { return g < 0 ? 0u : (unsigned)(g > ldl ? ldl : g); };
  auto fma2 = [](dpair acc, double a, dpair x) { return dpair{acc.x + a * x.x, acc.y + a * x.y}; };
  const int kn0 = 1, kn1 = S.klo, kp0 = S.khi, kp1 = nd - 1;
  const bool top = rq == 0, bot = rq == 15;
  int w = own32 + col * 16 + rq + z0 * D;
  dpair pm = xat(w - D);
  double amD = UD[cv(w - D)];
  dpair pcur = xat(w);
  for (int z = z0; z < z1; ++z, w += D)
  {
    const int r = w - own32;
    const unsigned wv = (unsigned)(w > ldl ? ldl : w);
    const unsigned m = r < mrows ? (unsigned)__builtin_nontemporal_load(mask + (unsigned)r) : 0u;
    const double aD = __builtin_nontemporal_load(UD + wv);
    const dpair pD = xat(w + D);
    const double a0 = S.j0 >= 0 ? __builtin_nontemporal_load(U0 + wv) : 0.0;
    const double ap = __builtin_nontemporal_load(U1 + wv);
    dpair eg;
    double ae = 0.0;
    if (top || bot) eg = xat(top ? w - 1 : w + 1);
    if (top) ae = U1[cv(w - 1)];
    double an = 0.0, aq = 0.0;
    dpair xn, xq;
    if (mp.dn)
    {
      const int g = w + mp.dn;
      an = mp.Un[cv(g)];
      xn = xat(g);
    }
    if (mp.dq)
    {
      aq = mp.Uq[wv];
      xq = xat(w + mp.dq);
    }
    dpair acc{0.0, 0.0};
    if (m & 1u) acc = fma2(acc, amD, pm);
    if (mp.dn && ((m >> kn0) & 1u)) acc = fma2(acc, an, xn);
    for (int k = kn0 + 1; k < kn1; ++k)  // (further far-negative offsets: generic gathers)
      if ((m >> k) & 1u)
      {
        const int g = w + S.off[k];
        acc = fma2(acc, S.val[(i64)S.dj[k] * S.ld + cv(g)], xat(g));
      }
    // rows w -/+ 1: lanes 4 apart (same column pair); the wave's first / last row loads its own
    const int up = (lane - 4) & 63, dn = (lane + 4) & 63;
    dpair pl{lane_from(pcur.x, up), lane_from(pcur.y, up)}, pr{lane_from(pcur.x, dn), lane_from(pcur.y, dn)};
    double am = lane_from(ap, up);
    if (top)
    {
      pl = eg;
      am = ae;
    }
    if (bot) pr = eg;
    if (S.km1 >= 0 && ((m >> S.km1) & 1u)) acc = fma2(acc, am, pl);
    if (S.k0 >= 0 && ((m >> S.k0) & 1u)) acc = fma2(acc, a0, pcur);
    if (S.kp1 >= 0 && ((m >> S.kp1) & 1u)) acc = fma2(acc, ap, pr);
    if (mp.dq && ((m >> kp0) & 1u)) acc = fma2(acc, aq, xq);
    for (int k = kp0 + 1; k < kp1; ++k)
      if ((m >> k) & 1u) acc = fma2(acc, S.val[(i64)S.dj[k] * S.ld + wv], xat(w + S.off[k]));
    if ((m >> kp1) & 1u) acc = fma2(acc, aD, pD);
    if (r < nrows)
    {
      __builtin_nontemporal_store(acc, Yb + (unsigned)w * 4u);
      if (DOT)
      {
        dsum.x += pcur.x * acc.x;
        dsum.y += pcur.y * acc.y;
      }
    }
    if constexpr (DOT == 2) quad_gram_add(gacc, r < nrows ? acc.x : 0.0, r < nrows ? acc.y : 0.0);  // (a quad = a row)
    pm = pcur;
    pcur = pD;
    amD = aD;
  }
  if constexpr (DOT == 2)
  {
    __shared__ double gs[kStreamThreads / 64 * 72], gv[72], gt[72];
    quad_gram_block<kStreamThreads>(gacc, dsum.x, dsum.y, gs, gv);
    if (grid_sum2<kStreamThreads>(gv, 72, part, part + (size_t)gridDim.x * 72, tick, blockIdx.x, gridDim.x, gt))
    {
      if (threadIdx.x < 64) gram[threadIdx.x] = gt[threadIdx.x];
      if (threadIdx.x < 8) dp[threadIdx.x] = gt[64 + threadIdx.x];
      if (threadIdx.x == 0 && zero_word) *zero_word = 0u;  // (the next MGS's barrier word)
    }
  }
  else if constexpr (DOT)
  {
    __shared__ double tot[8];
    double v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q)
    {
      v[2 * q] = q == cp ? dsum.x : 0.0;
      v[2 * q + 1] = q == cp ? dsum.y : 0.0;
    }
    if (grid_sum_n<8, kStreamThreads>(v, part + (size_t)qb * gridDim.x * 8, tick + (size_t)qb * kTicketStride, tot,
                                      blockIdx.x, gridDim.x))
    {
      if (threadIdx.x < 8) dp[qb * 8 + threadIdx.x] = tot[threadIdx.x];
    }
  }
}

bool launch_spmm_march(const eig_mat_s &A, i64 m, const double *X, double *Y, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// General band march for the 8-column SpMM and the fused Chebyshev step (k_spmm8_marchg).  The
// carried offset P is the widest band offset that is a multiple of 16 with -P stored too (3-D P1
// on the Kuhn split: P = N^2 + N); the others split into four spans of gathered offsets -- S1 below
// -P, S2 in (-P, -1), S3 in (+1, +P), S4 above +P -- of at most kGSpan offsets each, loaded
// predicated and unrolled (gathered operand + band value, the mirrored slot for negative offsets),
// S1 / S2 with the row's streams and S3 / S4 after the near terms.  Accumulation in ascending
// offset order: S1, -P, S2, -1, 0, +1, S3, +P, S4.  EPI = kStore: separately rounded products
// and sums over the stored entries (bitwise the reference SpMM); kGCheb: fused multiply-adds and
// the Chebyshev update of k_sell_mv8q's kCheb epilogue (tolerance-checked).
// ---------------------------------------------------------------------------------------------
constexpr int kGSpan = 3;
enum { kGStore = 0, kGCheb = 1 };

struct GSpans {
  int kPm, kPp;                      // mask bits of -P / +P
  int s1b, s1e, s2b, s2e, s3b, s3e, s4b, s4e;
};

template <class X>
__device__ __forceinline__ void gspan_load(const SymImg &S, int kb, int ke, int w, unsigned wv, int xl, int ldl,
                                           const X &xat, double (&a)[kGSpan], dpair (&x)[kGSpan])
{
#pragma unroll
  for (int k = 0; k < kGSpan; ++k)
  {
    const bool in = kb + k < ke;
    const int d = in ? S.off[kb + k] : 0;
    int g = w + d;
    g = g < 0 ? 0 : (g > xl ? xl : g);
    const unsigned gv = (unsigned)(g > ldl ? ldl : g);
    a[k] = in ? S.val[(i64)S.dj[kb + k] * S.ld + (d < 0 ? gv : wv)] : 0.0;
    x[k] = in ? xat(g) : dpair{0.0, 0.0};
  }
}

template <int EPI>
__device__ __forceinline__ dpair gacc(dpair acc, double a, dpair x)
{
  if (EPI == kGStore) return dpair{acc.x + a * x.x, acc.y + a * x.y};
  return dpair{__builtin_fma(a, x.x, acc.x), __builtin_fma(a, x.y, acc.y)};
}

template <int EPI>
__device__ __forceinline__ void gspan_acc(int kb, int ke, unsigned m, const double (&a)[kGSpan],
                                          const dpair (&x)[kGSpan], dpair &acc)
{
#pragma unroll
  for (int k = 0; k < kGSpan; ++k)
    if (kb + k < ke && ((m >> (kb + k)) & 1u)) acc = gacc<EPI>(acc, a[k], x[k]);
}

template <class MT, int EPI>
__global__ __launch_bounds__(kStreamThreads, 6) void k_spmm8_marchg(
    i64 nrows, i64 own, i64 ld, SellB1 A, MarchPlan mp, GSpans sp, const double *__restrict__ X,
    double *__restrict__ Y, const double *__restrict__ Bv, const double *__restrict__ dinv, double omega,
    double gamma)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rq = lane >> 2, cp = lane & 3;
  const SymImg &S = A.sym;
  const int xl = (int)A.xlast, P = (int)mp.D, ldl = (int)(S.ld - 1), own32 = (int)own, mrows = (int)mp.mrows;
  const double *UP = S.val + (i64)S.dj[sp.kPp] * S.ld;
  const double *U1 = S.val + (i64)S.j1 * S.ld;
  const double *U0 = S.val + (i64)(S.j0 >= 0 ? S.j0 : 0) * S.ld;
  const MT *mask = static_cast<const MT *>(S.mask);
  // (Measured and dropped at 256^3, m = 32: the workgroup's 4 waves on the 4 column blocks of one
  // item, so the band values / mask / D^-1 are fetched once per 4 blocks -- 6.62 vs 6.73 ms, with
  // any number of plane runs per column; rocprof: L2 misses on the gathered X rows dominate.)
  // (Measured and dropped: a persistent schedule with XCD-owned column ranges walked by 128-768
  // resident waves per XCD -- slower at every count, 7.5-19.5 ms: the march is latency-bound per
  // wave and wants full occupancy.)
  const int item = (int)swizzled_block() * kWaves + wave;
  if (item >= mp.ncol * mp.nseg) return;
  const int col = item % mp.ncol, seg = item / mp.ncol, blk = (int)blockIdx.y;
  const int z0 = (int)(mp.zb + seg * mp.nplanes / mp.nseg), z1 = (int)(mp.zb + (seg + 1) * mp.nplanes / mp.nseg);
  const i64 boff = (i64)blk * ld * 8;
  const dpair *Xb = reinterpret_cast<const dpair *>(X + boff) + cp;
  dpair *Yb = reinterpret_cast<dpair *>(Y + boff) + cp;
  const dpair *Bb = EPI == kGCheb ? reinterpret_cast<const dpair *>(Bv + boff) + cp : nullptr;
  auto xat = [&](int g) { return Xb[(unsigned)(g < 0 ? 0 : (g > xl ? xl : g)) * 4u]; };
  auto cv = [&](int g) -> unsigned { return g < 0 ? 0u : (unsigned)(g > ldl ? ldl : g); };
  const bool top = rq == 0, bot = rq == 15;
  int w = own32 + col * 16 + rq + z0 * P;
  dpair pm = xat(w - P);
  double amP = UP[cv(w - P)];
  dpair pcur = xat(w);
  for (int z = z0; z < z1; ++z, w += P)
  {
    const int r = w - own32;
    const unsigned wv = (unsigned)(w > ldl ? ldl : w);
    const unsigned m = r < mrows ? (unsigned)__builtin_nontemporal_load(mask + (unsigned)r) : 0u;
    const double aP = __builtin_nontemporal_load(UP + wv);
    const dpair pP = xat(w + P);
    const double a0 = S.j0 >= 0 ? __builtin_nontemporal_load(U0 + wv) : 0.0;
    const double ap = __builtin_nontemporal_load(U1 + wv);
    dpair eg;
    double ae = 0.0;
    if (top || bot) eg = xat(top ? w - 1 : w + 1);
    if (top) ae = U1[cv(w - 1)];
    double a1[kGSpan], a2[kGSpan];
    dpair x1[kGSpan], x2[kGSpan];
    gspan_load(S, sp.s1b, sp.s1e, w, wv, xl, ldl, xat, a1, x1);
    gspan_load(S, sp.s2b, sp.s2e, w, wv, xl, ldl, xat, a2, x2);
    dpair acc{0.0, 0.0};
    gspan_acc<EPI>(sp.s1b, sp.s1e, m, a1, x1, acc);
    if ((m >> sp.kPm) & 1u) acc = gacc<EPI>(acc, amP, pm);
    gspan_acc<EPI>(sp.s2b, sp.s2e, m, a2, x2, acc);
    const int up = (lane - 4) & 63, dn = (lane + 4) & 63;
    dpair pl{lane_from(pcur.x, up), lane_from(pcur.y, up)}, pr{lane_from(pcur.x, dn), lane_from(pcur.y, dn)};
    double am = lane_from(ap, up);
    if (top)
    {
      pl = eg;
      am = ae;
    }
    if (bot) pr = eg;
    if (S.km1 >= 0 && ((m >> S.km1) & 1u)) acc = gacc<EPI>(acc, am, pl);
    if (S.k0 >= 0 && ((m >> S.k0) & 1u)) acc = gacc<EPI>(acc, a0, pcur);
    if (S.kp1 >= 0 && ((m >> S.kp1) & 1u)) acc = gacc<EPI>(acc, ap, pr);
    gspan_load(S, sp.s3b, sp.s3e, w, wv, xl, ldl, xat, a1, x1);
    gspan_load(S, sp.s4b, sp.s4e, w, wv, xl, ldl, xat, a2, x2);
    gspan_acc<EPI>(sp.s3b, sp.s3e, m, a1, x1, acc);
    if ((m >> sp.kPp) & 1u) acc = gacc<EPI>(acc, aP, pP);
    gspan_acc<EPI>(sp.s4b, sp.s4e, m, a2, x2, acc);
    if (r < nrows)
    {
      if (EPI == kGStore)
        __builtin_nontemporal_store(acc, Yb + (unsigned)w * 4u);
      else
      {
        const double di = __builtin_nontemporal_load(dinv + r);
        const dpair bb = __builtin_nontemporal_load(Bb + (unsigned)w * 4u);
        const dpair xo = __builtin_nontemporal_load(Yb + (unsigned)w * 4u);
        const double gd = gamma * di;
        const double o0 = omega * (pcur.x + gd * (bb.x - acc.x) - xo.x) + xo.x;
        const double o1 = omega * (pcur.y + gd * (bb.y - acc.y) - xo.y) + xo.y;
        __builtin_nontemporal_store(dpair{o0, o1}, Yb + (unsigned)w * 4u);
      }
    }
    pm = pcur;
    pcur = pP;
    amP = aP;
  }
}

// Final beta of a fused run (eig_lanczos_tridiag): after the forced repair launch L-1 (or a repair
// the recurrence took itself), the exact ||u_j||^2 is in fred[3(L-1)+2] and (rn, rm) in aux[2L..]:
// beta[j] = sqrt(mex) rn / rm, nsum[j] = mex -- the values the post-repair step would store.
__global__ void k_fused_tail(double *nsum, double *beta, const double *fred, const int *ctl, const double *aux, int L)
{
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int j = ctl[2 * L], mode = ctl[2 * L + 1];
  if (mode == kFusedPost)
  {
    const double mex = fred[3 * (L - 1) + 2];
    nsum[j] = mex;
    beta[j] = mex > 0.0 ? sqrt(mex) * aux[2 * L] / aux[2 * L + 1] : 0.0;
  }
  else if (j == 0)
    beta[0] = sqrt(nsum[0]);
}

// Grid = min(work, resident workgroups): every workgroup takes one contiguous chunk, so a grid
// larger than what the CUs hold at once would leave a tail of late chunks.
template <class K>
static int grid_for_slices(K kernel, i64 count, int num_cu)
{
  static thread_local std::pair<const void *, int> cache{nullptr, 0};
  int per_cu = 0;
  if (cache.first == (const void *)kernel) per_cu = cache.second;
  else
  {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kStreamThreads, 0) != hipSuccess || per_cu < 1)
      per_cu = 4;
    cache = {(const void *)kernel, per_cu};
  }
  const i64 cap = (i64)per_cu * num_cu;
  const i64 need = (count + kWaves - 1) / kWaves;
  if (need < 1) return 1;
  return (int)(need < cap ? need : cap);
}

// The packed value image of march variants 13 / 15: two arrays of value pairs, (+D, 0) and (+1, +nx)
// per window row (the 5-point 2-D band: +nx = 0), so a wave reads each with one 16-B load per lane
// of 1 KB contiguous; built from the band arrays at first use, freed by a shift.
__global__ void k_sym_pack(i64 ld, const double *__restrict__ UD, const double *__restrict__ U0,
                           const double *__restrict__ U1, const double *__restrict__ Uq, double *__restrict__ out)
{
  for (i64 w = (i64)blockIdx.x * blockDim.x + threadIdx.x; w < ld; w += (i64)gridDim.x * blockDim.x)
  {
    reinterpret_cast<dpair *>(out)[w] = dpair{UD[w], U0 ? U0[w] : 0.0};
    reinterpret_cast<dpair *>(out)[ld + w] = dpair{U1[w], Uq ? Uq[w] : 0.0};
  }
}
// Kuhn pack (march variant 16): four pair arrays, (0, +1), (+nx, +nx+1), (+D, +D+1), (+D+nx, +D+nx+1)
__global__ void k_kuhn_pack(i64 ld, const double *__restrict__ val, int4 ja, int4 jb, double *__restrict__ out)
{
  const int j0[4] = {ja.x, ja.z, jb.x, jb.z}, j1[4] = {ja.y, ja.w, jb.y, jb.w};
  for (i64 w = (i64)blockIdx.x * blockDim.x + threadIdx.x; w < ld; w += (i64)gridDim.x * blockDim.x)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      reinterpret_cast<dpair *>(out)[(i64)q * ld + w] = dpair{val[(i64)j0[q] * ld + w], val[(i64)j1[q] * ld + w]};
}
static bool march_kuhn(const eig_mat_s &A);
void sym_pack_fill(eig_mat_s &A, hipStream_t s)
{
  if (A.sym_box27 == kKuhn15)
  {
    // band array of each upper Kuhn offset (the 27-box positions 13 14 | 16 17 | 22 23 | 25 26)
    const i64 D = (i64)A.sym_gx * A.sym_gy;
    int j[27];
    for (int q = 0; q < 27; ++q) j[q] = 0;
    for (int k = 0; k < A.sym_nd; ++k)
      for (int q = 13; q < 27; ++q)
        if ((i64)(q / 9 - 1) * D + (i64)((q / 3) % 3 - 1) * A.sym_gx + (q % 3 - 1) == A.sym_off[k]) j[q] = A.sym_dj[k];
    hipLaunchKernelGGL(k_kuhn_pack, dim3(2048), dim3(256), 0, s, A.sym_ld, A.sym_val,
                       make_int4(j[13], j[14], j[16], j[17]), make_int4(j[22], j[23], j[25], j[26]), A.sym_pack);
    EIG_HIP(hipGetLastError());
    return;
  }
  const SellB1 b = sell_b1(A);
  const SymImg &S = b.sym;
  const double *UD = S.val + (i64)S.dj[S.nd - 1] * S.ld, *U1 = S.val + (i64)S.j1 * S.ld;
  const double *U0 = S.j0 >= 0 ? S.val + (i64)S.j0 * S.ld : nullptr;
  const double *Uq = S.khi < S.nd - 1 ? S.val + (i64)S.dj[S.khi] * S.ld : nullptr;
  hipLaunchKernelGGL(k_sym_pack, dim3(2048), dim3(256), 0, s, S.ld, UD, U0, U1, Uq, A.sym_pack);
  EIG_HIP(hipGetLastError());
}

// The value pack, built at the first launch that marches on it (never by a plan made for a query:
// eig_mat_get_info, kernel names, byte models).  eig_lanczos_capture builds it before capturing,
// so no graph records the pack kernel; a shift refills the same buffer in place.
const double *sym_pack_prepare(const eig_mat_s &Ac)
{
  eig_mat_s &A = const_cast<eig_mat_s &>(Ac);
  if (A.sym_pack) return A.sym_pack;
  const i64 bytes = A.sym_ld * (A.sym_box27 == kKuhn15 ? 64 : 32);
  EIG_HIP(hipMalloc(&A.sym_pack, (size_t)bytes));
  A.sym_pack_bytes = bytes;
  A.device_bytes += bytes;
  sym_pack_fill(A, A.ctx->stream);
  return A.sym_pack;
}

// EIG_MAT_NO_MARCH: the plane-marching kernels are off for this matrix (the slice kernels run).
static bool march_enabled(const eig_mat_s &A) { return (A.kflags & EIG_MAT_NO_MARCH) == 0; }
static bool march_span1(const eig_mat_s &A)
{
  int klo = A.sym_nd, khi = A.sym_nd;
  for (int k = A.sym_nd - 1; k >= 0; --k)
  {
    if (A.sym_off[k] >= -1) klo = k;
    if (A.sym_off[k] > 1) khi = k;
  }
  return A.sym_mask_bytes == 1 && klo - 1 <= 1 && (A.sym_nd - 1) - khi <= 1;
}

// Far spans of at most one offset each (u8-mask bands only: at most 8 offsets, so (-D, -1) and
// (+1, +D) hold at most one offset each exactly when nd <= 7 with -1/0/+1 present).
// Uniform band values in the march kernels' arguments (EIG_MAT_NO_UNIFORM keeps the array loads).
// 0 = the arrays, 1 = uniform values + loaded row masks, 2 = uniform values + geometric row masks
// (the grid coordinates of the global rows: a rank's slab starts at global plane sym_gz0);
// 3 / 4 / 5: geometric, march_rows_geo with the +D operand 1 / 2 / 3 planes ahead, 6: 3 planes
// ahead and the gathers 1 plane ahead (eig_mat_tune(EIG_TUNE_MARCH_PREFETCH) = 1 forces 2, 2..5
// force 3..6; 0 = kGeoAuto).
// 7 / 8 / 9: march_rows_geo2 (no masks or selects; x extent a multiple of 64, window < 2 GiB) with
// the prefetches of 3 / 4 / 6 (tune values 6..8); a geo2 request on a grid that does not qualify
// takes the corresponding march_rows_geo variant.
// Automatic choice (measured: profiles/r03bj_march_variants.jsonl, r03bn_*, r03bp_*; tools/gpu.sh
// prefetch): geo2 without prefetch (7) where the grid allows it -- fused step 256^3 125.8 us at 8
// plane runs (plain march 130.0), 128^3 20.1 us (plain 30.2; with the MALL-resident plain stores,
// MarchPlan::tstore), one rank's 256^2 x 32 slab 20.5 us (plain 34.5); eig_mv 256^3 46.1 us (plain
// 59.4), 128^3 8.0 (12.1).  The prefetching geo2 variants (8, 9) are within a few per cent either
// way.  Grids geo2 does not take: march_rows_geo with the +D operand two planes ahead (4).
// 10 / 11: bands that are not uniform (or EIG_MAT_NO_UNIFORM) on a geo2 grid: the value march
// (march_rows_geo2<VAL>: the band arrays streamed, masks from the coordinates), 11 with the value
// streams and the +D operand one plane ahead (tune values 9 / 10; 1 = the plain masked march).
// 12: the P1 Kuhn box march (march_rows_kuhn; eig_mat_s::sym_box27 == kKuhn15, one rank).
static bool march_kuhn(const eig_mat_s &A)
{
  return A.sym_box27 == kKuhn15 && A.sym_nd == 15 && !A.ctx->distributed() && A.sym_gx % 64 == 0 &&
         A.window * 16 < (i64(1) << 31) && A.sym_ld * 8 < (i64(1) << 31) && A.tune_march_prefetch != 1;
}
bool kuhn_pack_fits(const eig_mat_s &A) { return A.sym_ld * 64 < (i64(1) << 31); }
// the Kuhn march on its value pack (16): fused step 256^3 346 us, eig_mv 292 us (the arrays, 12: 407 /
// 330 us; profiles/r04d_p1k.jsonl); tune value 14 = the arrays, 15 = the pack variant 19.
// The pack is read through one 32-bit buffer descriptor of 64 B per row: grids of 2^25 rows and
// more (e.g. 448^3, or 256 x 512 x 512, whose descriptor size would wrap to 0) take the arrays.
// Default 20 (the pack with the line exchange in LDS) where the lines come in groups of 4: 256^3 fused
// step 333.2 vs 340.8 us, eig_mv 278.7 vs 292.2 us (profiles/r05g_p1k.jsonl); tune value 13 = 16.
int kuhn_variant(const eig_mat_s &A)
{
  const int tp = A.tune_march_prefetch;
  if (tp == 14 || !kuhn_pack_fits(A)) return 12;
  if (tp == 15) return 19;
  return tp != 13 && A.sym_gy % 4 == 0 ? 20 : 16;
}
static int march_uniform(const eig_mat_s &A, bool fused = false, i64 nplanes = 0)
{
  if (march_kuhn(A)) return kuhn_variant(A);
  const bool geo2 = A.sym_geo && A.sym_gx % 64 == 0 && A.window * 16 < (i64(1) << 31);
  if (!A.sym_uniform || (A.kflags & EIG_MAT_NO_UNIFORM))
  {
    if (!geo2 || !march_span1(A) || A.sym_ld * 32 >= (i64(1) << 31) || A.tune_march_prefetch == 1) return 0;
    // automatic: the fused step on the value pack (15: 223.7 us at 256^3, one rank's 256^2 x 32 slab
    // 30.4 us; the arrays 226.8 / 31.7), eig_mv / K1 on the plain masked march (0: 152.1 us against 161.4 on
    // the pack): profiles/r04d_latency.jsonl, r04d_slab.jsonl
    const int tp = A.tune_march_prefetch;
    // 22: two grid lines per wave (7-point bands on grids of an even line count)
    const bool two = A.sym_nd == 7 && A.sym_gy % 2 == 0 && A.sym_gy > 0;
    if (tp >= 16 && tp <= 18) return two ? tp + 6 : 15;
    const bool big = A.nb_rows >= EIG_MARCH_2L_MIN_ROWS;
    return tp == 9 ? 10 : tp == 10 ? 11 : tp == 12 ? 14 : tp == 13 ? 15 : tp == 15 ? 18
         : fused ? (A.sym_nd == 7 ? (two && big && kMarch2lDefault ? 22 : 15) : 10) : 0;
  }
  if (!A.sym_geo) return 1;
  int u = A.tune_march_prefetch > 0 ? 1 + A.tune_march_prefetch : geo2 ? 7 : 4;
  if (u >= 7 && !geo2) u = u == 9 ? 6 : u - 4;
  return u;
}


// Launch a march kernel template KERN<MT, SPAN1> for the image's mask width (u8 masks only can
// have single-offset far spans).
#define EIG_MARCH_LAUNCH(KERN, MODE, G, ...)                                                               \
  do {                                                                                                    \
    if (mp.uni == 12)                                                                                     \
      hipLaunchKernelGGL((KERN<uint32_t, false, 12>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);     \
    else if (mp.uni == 16)                                                                                \
      hipLaunchKernelGGL((KERN<uint32_t, false, 16>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);     \
    else if (mp.uni == 20)                                                                                \
      hipLaunchKernelGGL((KERN<uint32_t, false, 20>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);     \
    else if (mp.uni == 19)                                                                                \
      hipLaunchKernelGGL((KERN<uint32_t, false, 19>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);     \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 14)                                          \
      hipLaunchKernelGGL((KERN<uint8_t, true, 14>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);       \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 15)                                          \
      hipLaunchKernelGGL((KERN<uint8_t, true, 15>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);       \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 22)                                          \
      hipLaunchKernelGGL((KERN<uint8_t, true, 22>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);       \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 23)                                          \
      hipLaunchKernelGGL((KERN<uint8_t, true, 23>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);       \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 24)                                          \
      hipLaunchKernelGGL((KERN<uint8_t, true, 24>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);       \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 18)                                          \
      hipLaunchKernelGGL((KERN<uint8_t, true, 18>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);       \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 11)                                          \
      hipLaunchKernelGGL((KERN<uint8_t, true, 11>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);       \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 10)                                          \
      hipLaunchKernelGGL((KERN<uint8_t, true, 10>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);       \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 9)                                      \
      hipLaunchKernelGGL((KERN<uint8_t, true, 9>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 8)                                 \
      hipLaunchKernelGGL((KERN<uint8_t, true, 8>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 7)                                 \
      hipLaunchKernelGGL((KERN<uint8_t, true, 7>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 6)                                 \
      hipLaunchKernelGGL((KERN<uint8_t, true, 6>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 5)                                 \
      hipLaunchKernelGGL((KERN<uint8_t, true, 5>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 4)                                 \
      hipLaunchKernelGGL((KERN<uint8_t, true, 4>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 3)                                 \
      hipLaunchKernelGGL((KERN<uint8_t, true, 3>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 2)                                 \
      hipLaunchKernelGGL((KERN<uint8_t, true, 2>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8 && march_span1(A) && mp.uni == 1)                                 \
      hipLaunchKernelGGL((KERN<uint8_t, true, 1>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8 && march_span1(A))                                                          \
      hipLaunchKernelGGL((KERN<uint8_t, true, 0>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);        \
    else if ((MODE) == kSymN8)                                                                            \
      hipLaunchKernelGGL((KERN<uint8_t, false, 0>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);       \
    else                                                                                                  \
      hipLaunchKernelGGL((KERN<uint32_t, false, 0>), dim3(G), dim3(kStreamThreads), 0, __VA_ARGS__);      \
  } while (0)

// Plane-marching plan for a whole-matrix launch on the lane-shift band image, or nseg = 0 when the
// band does not qualify: symmetric offset set with off[0] = -D, off[nd-1] = +D, D a multiple of 64,
// at least 4 planes.  Plane runs per column: enough items for one resident wave per SIMD slot
// (8 per SIMD), at most kMaxRedBlocks workgroups.
// Band geometry the march needs (independent of the matrix's kernel flags): widest offset D.
bool march_geometry(const eig_mat_s &A, i64 &D, int chunk)
{
  D = 0;
  if (!A.sym_val || A.sym_nd < 3) return false;
  bool near = false;
  for (int k = 0; k < A.sym_nd; ++k) near = near || A.sym_off[k] == 1 || A.sym_off[k] == -1;
  D = A.sym_off[A.sym_nd - 1];
  return near && D > 1 && D % chunk == 0 && A.sym_off[0] == -D;
}

// [zb, ze): plane range of a split launch (the interior planes of a distributed slab); ze < 0 =
// the whole matrix.
// chunk: rows per wave column (64 for the scalar kernels, 16 for the 8-column SpMM).
// pack: build the value pack the plan's variant streams (launch paths only; a query leaves it unbuilt)
static MarchPlan march_plan(const eig_mat_s &A, int mode, i64 zb = 0, i64 ze = -1, bool fused = false,
                            int chunk = 64, bool pack = false)
{
  MarchPlan mp{};
  if (mode != kSymN8 && mode != kSymN32) return mp;
  i64 D;
  const bool kuhn = chunk == 64 && march_kuhn(A);
  if (!march_enabled(A) || !(kuhn ? (D = (i64)A.sym_gx * A.sym_gy) > 0 : march_geometry(A, D, chunk))) return mp;
  if (ze < 0) ze = (A.nb_rows + D - 1) / D;
  const i64 nplanes = ze - zb;
  if (nplanes < 2 || (zb == 0 && nplanes < 4)) return mp;
  const i64 ncol = D / chunk;
  // about one work item per resident wave slot (8 per SIMD)
  const i64 resident = 8LL * 4 * A.ctx->num_cu;  // waves
  i64 nseg = std::max<i64>(1, (resident + ncol - 1) / ncol);
  nseg = std::min<i64>(nseg, nplanes);
  // the fused step prefers longer plane runs (fewer fronts in the XCDs' L2 at once) wherever the
  // grid is small; measured with eig_mat_tune sweeps (tools/gpu.sh latency, profiles/r03h_latency):
  //  * wide planes (>= 1024 columns: 256^2 per plane): 256^3 8 runs 220.8 us (7: 224.6, 6: 232.5,
  //    4: 267.3); one rank's 256^2 x 32 slab 2 runs 33.7 us (4: 35.5, 7: 36.7, 1: 47.3); the 16-plane
  //    slab 2 runs 21.7 us (1: 28.3, 4: 23.9, 7: 26.2)  ->  nplanes / 32 runs, at least 2, at most 8
  //  * narrower planes (128^3: 256 columns): 12 runs 34.9 us (16: 35.5, 28: 36.5, 32: 36.7)  ->
  //    runs of >= 10 planes, as long as that leaves a quarter of the resident slots busy (64^3, 64
  //    columns: 6 runs of 10 planes took 20.1 us, 64 runs of one plane 13.3)
  //  * (round 3, uniform-band march: 256^3 6 runs 129.8-134.0 us, 8 runs 133.6-137.1: at most 6)
  //  * round 6, the value pack marches (15, 22-24) on wide planes: TWO runs per column, i.e. long
  //    chains of half the planes each (profiles/r06q_*, r06r_runs_*: 256^3 2-line 193.2 us at 2 runs
  //    vs 208.3 at its former 16 (1: 268.2); 1-line 204.4 at 2 vs 225.2 at 8 (1: 255.8, 4: 261.6);
  //    256^2 slabs of 32 / 64 / 96 / 128 planes 27.6 / 45.6 / 77.9 / 102.2 us for the 2-line march
  //    at 2 runs, the best or equal of every count tried).  On 128^3 (256 columns) 2 runs are slow
  //    (52.3 us vs 28.3): the rule is for wide planes only.  The same holds for the P1 Kuhn march
  //    (profiles/r06t_runs_p1k.jsonl: fused step 312.5 us at 2 runs vs 333.9 at 8, 4: 380.9; eig_mv
  //    263.2 vs 280.0); not for the 7-point value eig_mv (151.9 vs 154.7 on one box, 152.8 vs 152.2 on
  //    another: r06r_runs_256.jsonl, r06u_runs_uniform_mv.jsonl) nor the uniform-band march (fused
  //    132.7 vs 132.1, eig_mv 61.3 vs 48.9).
  const int uni = march_uniform(A, fused, nplanes);
  const bool wide_pack = ncol >= 1024 && chunk == 64 && (kuhn || (fused && (uni == 15 || is_march2l(uni))));
  if (wide_pack)
    nseg = std::min<i64>(2, nplanes);
  else if (fused && ncol >= 1024)
    nseg = std::min<i64>(nplanes / 2 > 0 ? nplanes / 2 : 1,
                         std::max<i64>(2, std::min<i64>(uni == 7 || uni >= 10 ? 8 : 6, nplanes / 32)));
  else if (fused)  // (geo2 marches: runs of >= 16 planes -- 128^3 8 runs 24.3 us, 12: 25.3, 16: 26.4)
    nseg = std::min(nseg, std::max<i64>({1, nplanes / (uni >= 7 ? 16 : 10), (resident / 4 + ncol - 1) / ncol}));
  // variant 22 marches line PAIRS: half the items per plane run, so twice the runs for as many waves
  const i64 items_per_run = is_march2l(uni) ? ncol / 2 : ncol;
  if (is_march2l(uni) && !wide_pack) nseg = std::min<i64>(nplanes, 2 * nseg);
  if (A.tune_march_runs > 0) nseg = std::min<i64>(A.tune_march_runs, nplanes);  // eig_mat_tune
  while (nseg > 1 && (items_per_run * nseg + kWaves - 1) / kWaves > kMaxRedBlocks) --nseg;
  if ((items_per_run * nseg + kWaves - 1) / kWaves > kMaxRedBlocks) return mp;
  mp.D = D;
  int klo = A.sym_nd, khi = A.sym_nd;
  for (int k = A.sym_nd - 1; k >= 0; --k)
  {
    if (A.sym_off[k] >= -1) klo = k;
    if (A.sym_off[k] > 1) khi = k;
  }
  mp.dn = klo > 1 ? A.sym_off[1] : 0;
  mp.Un = A.sym_val + (i64)(klo > 1 ? A.sym_dj[1] : 0) * A.sym_ld;
  mp.dq = khi < A.sym_nd - 1 ? A.sym_off[khi] : 0;
  mp.Uq = A.sym_val + (i64)(khi < A.sym_nd - 1 ? A.sym_dj[khi] : 0) * A.sym_ld;
  for (int q = 0; q < 27; ++q) mp.kj[q] = -1;
  if (kuhn)
  {
    // band array of each upper box offset a D + b nx + c
    for (int k = 0; k < A.sym_nd; ++k)
      for (int q = 13; q < 27; ++q)
        if ((i64)(q / 9 - 1) * D + (i64)((q / 3) % 3 - 1) * A.sym_gx + (q % 3 - 1) == A.sym_off[k])
          mp.kj[q] = (signed char)A.sym_dj[k];
  }
  if (A.sym_geo || kuhn)
  {
    mp.gx = A.sym_gx;
    mp.gy = A.sym_gy;
    mp.gz = A.sym_gz;
    mp.gz0 = A.sym_gz0;
  }
  if (A.sym_uniform)
  {
    const int kD = A.sym_nd - 1;
    int kz = -1, k1 = -1;
    for (int k = 0; k < A.sym_nd; ++k)
    {
      if (A.sym_off[k] == 0) kz = k;
      if (A.sym_off[k] == 1) k1 = k;
    }
    mp.cD = A.sym_uc[A.sym_dj[kD]];
    mp.c0 = kz >= 0 ? A.sym_uc[A.sym_dj[kz]] : 0.0;
    mp.c1 = k1 >= 0 ? A.sym_uc[A.sym_dj[k1]] : 0.0;
    mp.cn = klo > 1 ? A.sym_uc[A.sym_dj[1]] : 0.0;
    mp.cq = khi < A.sym_nd - 1 ? A.sym_uc[A.sym_dj[khi]] : 0.0;
  }
  mp.uni = uni;
  mp.pack = pack && (uni == 15 || uni == 16 || uni == 18 || uni == 19 || uni == 20 || is_march2l(uni)) ? sym_pack_prepare(A) : nullptr;
  // measured (tools/march_copy.hip *_pp, profiles/r03bo_march_copy.jsonl): the step's ping-pong at
  // 128^3 (2 x 32 MB of pairs) 12.9 us with plain stores vs 17.6 us nontemporal; at 256^3 (2 x 268
  // MB) no difference either way -- plain stores where every vector a launch touches fits in half
  // of the 256 MB MALL
  // fused step only (eig_mv's y, written repeatedly beside the same x, measured slower: 128^3 9.6 vs
  // 8.0 us)
  mp.tstore = fused && uni >= 7 && (A.window * 16 * 3 <= (i64(128) << 20) || (A.tune_cache & 1));
  mp.cache = A.tune_cache;
  // line groups (geo2 value marches 10 / 11 / 14 / 15 on grids of whole 64-x runs and 4-line groups)
  mp.lines = A.tune_march_lines == 4 && !kuhn && uni >= 10 && uni <= 15 && uni != 12 && mp.gx % 64 == 0 &&
                     mp.gx > 0 && mp.gy % 4 == 0 && (i64)mp.gx * mp.gy == D
                 ? 4
                 : 0;
  mp.zb = zb;
  mp.nplanes = nplanes;
  mp.mrows = A.nslices * 64;
  mp.ncol = (int)items_per_run;
  mp.nseg = (int)nseg;
  return mp;
}

// eig_mat_info.march_variant: the variant a whole-matrix launch takes, -1 when it does not march
int march_variant(const eig_mat_s &A, bool fused)
{
  if (A.br != 1 || A.bc != 1) return -1;
  const MarchPlan mp = march_plan(A, image_mode(A), 0, -1, fused);
  return mp.nseg > 0 ? mp.uni : -1;
}

const i32 kMarchInteriorTag = 0;

void march_prepare(const eig_mat_s &A)
{
  if (A.br != 1 || A.bc != 1) return;
  const int mode = image_mode(A);
  for (bool fused : {false, true})
  {
    (void)march_plan(A, mode, 0, -1, fused, 64, true);
    if (A.mz1 > A.mz0) (void)march_plan(A, mode, A.mz0, A.mz1, fused, 64, true);
  }
}

bool march_split_active(const eig_mat_s &A)
{
  return A.mz1 > A.mz0 && march_plan(A, image_mode(A), A.mz0, A.mz1).nseg > 0;
}

// Plan for a launch: the whole matrix (slices == nullptr over all slices), the interior planes of a
// distributed slab (slices == &kMarchInteriorTag), or none (nseg = 0: the slice kernels run).
static MarchPlan launch_plan(const eig_mat_s &A, int mode, const i32 *slices, i64 first, i64 count,
                             bool fused = false)
{
  if (slices == &kMarchInteriorTag)
  {
    const MarchPlan mp = march_plan(A, mode, A.mz0, A.mz1, fused, 64, true);
    EIG_CHECK(mp.nseg > 0, EIG_ERR_ARG, "interior-plane launch without a march plan");
    return mp;
  }
  if (!slices && first == 0 && count == A.nslices) return march_plan(A, mode, 0, -1, fused, 64, true);
  return MarchPlan{};
}

void launch_spmv(const eig_mat_s &A, const double *x, double *y, const i32 *slices, i64 first, i64 count,
                 hipStream_t s, bool keep)
{
  if (count <= 0 && slices != &kMarchInteriorTag) return;
  const int ncu = A.ctx->num_cu;
  double *yo = y + A.own_offset;
  if (A.br == 1 && A.bc == 1)
  {
    const int mode = image_mode(A);
    MarchPlan mp = launch_plan(A, mode, slices, first, count);
    // keep: y is read by the very next launch (the pipelined step's S) -- plain stores on grids
    // whose vectors fit the MALL, as the fused step's (MarchPlan::tstore)
    if (keep && mp.uni >= 7 && A.window * 16 * 3 <= (i64(128) << 20)) mp.tstore = 1;
    if (mp.nseg > 0)
    {
      const unsigned G = (unsigned)((mp.ncol * (i64)mp.nseg + kWaves - 1) / kWaves);
      EIG_MARCH_LAUNCH(k_spmv_march, mode, G, s, A.nb_rows, A.own_offset, sell_b1(A), mp, x, y);
      return;
    }
  }
#define EIG_BLK(R_, C_)                                                                                 \
  if (A.br == R_ && A.bc == C_)                                                                         \
  {                                                                                                     \
    const int G = grid_for_slices(k_spmv_blk<R_, C_>, count, ncu);                                      \
    hipLaunchKernelGGL((k_spmv_blk<R_, C_>), dim3(G), dim3(kStreamThreads), 0, s, A.nb_rows, A.slice_ptr, \
                       slices, first, count, A.val, A.col, x, yo);                                      \
    return;                                                                                             \
  }
#define EIG_B1_(R_, M_, CPF_)                                                                            \
  {                                                                                                      \
    const int G = grid_for_slices(k_spmv_b1<R_, M_, CPF_>, count, ncu);                                  \
    hipLaunchKernelGGL((k_spmv_b1<R_, M_, CPF_>), dim3(G), dim3(kStreamThreads), 0, s, A.nb_rows,         \
                       A.own_offset, sell_b1(A), slices, first, count, x, y);                            \
  }
#define EIG_B1(R_, M_)                                                                                   \
  {                                                                                                      \
    if (sell_cpf(A, false) && (M_ == kExplicit || M_ == kMixed)) EIG_B1_(R_, M_, true)                   \
    else EIG_B1_(R_, M_, false)                                                                          \
  }
#define EIG_B1M(R_)                                                                                      \
  {                                                                                                      \
    const int m_ = image_mode(A);                                                                        \
    if (m_ == kExplicit) EIG_B1(R_, kExplicit)                                                           \
    else if (m_ == kStencil) EIG_B1(R_, kStencil)                                                        \
    else if (m_ == kSym8) EIG_B1(R_, kSym8)                                                              \
    else if (m_ == kSym32) EIG_B1(R_, kSym32)                                                            \
    else if (m_ == kSymN8) EIG_B1(R_, kSymN8)                                                            \
    else if (m_ == kSymN32) EIG_B1(R_, kSymN32)                                                            \
    else EIG_B1(R_, kMixed)                                                                              \
  }
  if (A.br == 1 && A.bc == 1)
  {
    EIG_B1M(1)
    return;
  }
#undef EIG_B1M
#undef EIG_B1
#undef EIG_B1_
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
  if (!carry)
  {
    const int mode = image_mode(A);
    const MarchPlan mp = launch_plan(A, mode, slices, first, count);
    if (mp.nseg > 0)
    {
      const unsigned G = (unsigned)((mp.ncol * (i64)mp.nseg + kWaves - 1) / kWaves);
      EIG_MARCH_LAUNCH(k_lanczos_spmv_march, mode, G, s, A.nb_rows, A.own_offset, sell_b1(A), mp, u, up, t, j,
                       st.nsum, dot_out, beta_out, red.partials, red.ticket(ticket));
      return;
    }
  }
#define EIG_LZ(R_, M_)                                                                                       \
  hipLaunchKernelGGL((k_lanczos_spmv_b1<R_, M_>),                                                           \
                     dim3(grid_for_slices(k_lanczos_spmv_b1<R_, M_>, count, A.ctx->num_cu)), dim3(kStreamThreads), \
                     0, s, A.nb_rows, A.own_offset, sell_b1(A), slices, first, count, u, up, t, j, st.nsum, dot_out, \
                     beta_out, carry, red.partials, red.ticket(ticket))
#define EIG_LZM(R_)                                                                                          \
  {                                                                                                          \
    const int m_ = image_mode(A);                                                                            \
    if (m_ == kExplicit) EIG_LZ(R_, kExplicit);                                                              \
    else if (m_ == kStencil) EIG_LZ(R_, kStencil);                                                           \
    else if (m_ == kSym8) EIG_LZ(R_, kSym8);                                                                 \
    else if (m_ == kSym32) EIG_LZ(R_, kSym32);                                                               \
    else if (m_ == kSymN8) EIG_LZ(R_, kSymN8);                                                               \
    else if (m_ == kSymN32) EIG_LZ(R_, kSymN32);                                                               \
    else EIG_LZ(R_, kMixed);                                                                                 \
  }
  EIG_LZM(1)
#undef EIG_LZM
#undef EIG_LZ
}

void launch_lanczos_fused(const eig_mat_s &A, const double *P, double *Pout, const FusedLaunch &fl,
                          const i32 *slices, i64 first, i64 count, const double *carry, double *out, int ticket,
                          hipStream_t s, ReduceWS red)
{
  EIG_CHECK(A.br == 1 && A.bc == 1, EIG_ERR_BLOCKSIZE, "Lanczos driver: 1x1 blocks only");
  FusedArgs fa{fl.st.nsum, fl.st.alpha, fl.st.beta, fl.st.fred, fl.st.ctl, fl.st.aux, fl.st.mu2, fl.st.pn, fl.L,
               fl.force, 0, Mailbox{}};
  if (fl.xch)
  {
    EIG_CHECK(A.ctx->step_exchange(), EIG_ERR_ARG, "fused step: in-kernel exchange without the mailbox");
    fa.xch = fl.xch & kXchPublish;
    fa.mb = A.ctx->mbox->dev;
  }
  if (!carry)
  {
    const int mode = image_mode(A);
    const MarchPlan mp = launch_plan(A, mode, slices, first, count, true);
    if (mp.nseg > 0)
    {
      const unsigned G = (unsigned)((mp.ncol * (i64)mp.nseg + kWaves - 1) / kWaves);
      EIG_MARCH_LAUNCH(k_lanczos_fused_march, mode, G, s, A.nb_rows, A.own_offset, sell_b1(A), mp,
                       reinterpret_cast<const dpair *>(P), reinterpret_cast<dpair *>(Pout), fa, out, red.partials,
                       red.ticket(ticket));
      return;
    }
  }
#define EIG_LF_(R_, M_, CPF_)                                                                                 \
  hipLaunchKernelGGL((k_lanczos_fused_b1<R_, M_, CPF_>),                                                     \
                     dim3(grid_for_slices(k_lanczos_fused_b1<R_, M_, CPF_>, count, A.ctx->num_cu)),           \
                     dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset, sell_b1(A), slices, first, count,      \
                     reinterpret_cast<const dpair *>(P), reinterpret_cast<dpair *>(Pout), fa, out, carry,        \
                     red.partials, red.ticket(ticket))
#define EIG_LF(R_, M_)                                                                                        \
  do                                                                                                          \
  {                                                                                                           \
    if (sell_cpf(A, true) && (M_ == kExplicit || M_ == kMixed)) EIG_LF_(R_, M_, true);                        \
    else EIG_LF_(R_, M_, false);                                                                              \
  } while (0)
#define EIG_LFM(R_)                                                                                           \
  {                                                                                                           \
    const int m_ = image_mode(A);                                                                             \
    if (m_ == kExplicit) EIG_LF(R_, kExplicit);                                                               \
    else if (m_ == kStencil) EIG_LF(R_, kStencil);                                                            \
    else if (m_ == kSym8) EIG_LF(R_, kSym8);                                                                  \
    else if (m_ == kSym32) EIG_LF(R_, kSym32);                                                                \
    else if (m_ == kSymN8) EIG_LF(R_, kSymN8);                                                                \
    else if (m_ == kSymN32) EIG_LF(R_, kSymN32);                                                              \
    else EIG_LF(R_, kMixed);                                                                                  \
  }
  EIG_LFM(1)
#undef EIG_LFM
#undef EIG_LF
#undef EIG_LF_
}

void launch_lanczos_pipe(const eig_mat_s &A, double *T, double *UZ, const double *S, const FusedLaunch &fl,
                         double *out, hipStream_t s, ReduceWS red)
{
  EIG_CHECK(A.br == 1 && A.bc == 1, EIG_ERR_BLOCKSIZE, "Lanczos driver: 1x1 blocks only");
  const i64 n = A.nb_rows, own = A.own_offset;
  EIG_CHECK((own & 1) == 0 && (((uintptr_t)T | (uintptr_t)UZ | (uintptr_t)S) & 15) == 0, EIG_ERR_ARG,
            "pipelined Lanczos: vectors must be 16-B aligned");
  const FusedArgs fa{fl.st.nsum, fl.st.alpha, fl.st.beta, fl.st.fred, fl.st.ctl, fl.st.aux, fl.st.mu2, fl.st.pn, fl.L,
                     fl.force, 0, Mailbox{}};
  const i64 per = 2LL * kStreamThreads;
  const int G = (int)std::max<i64>(1, std::min<i64>(kStreamBlocks, (n + per - 1) / per));
  hipLaunchKernelGGL(k_lanczos_pipe, dim3(G), dim3(kStreamThreads), 0, s, n, T + own,
                     reinterpret_cast<dpair *>(UZ) + own, S + own, fa, out, red.partials, red.ticket(0));
}

void launch_fused_tail(const LanczosState &st, int L, hipStream_t s)
{
  hipLaunchKernelGGL(k_fused_tail, dim3(1), dim3(64), 0, s, st.nsum, st.beta, st.fred, st.ctl, st.aux, L);
}

// General band geometry for k_spmm8_marchg: carried offset P (widest multiple of 16 with -P stored),
// +-1 stored, every span at most kGSpan offsets.  False when the band does not qualify.
static bool gspans(const eig_mat_s &A, i64 &P, GSpans &sp)
{
  if (!A.sym_val || A.sym_nd < 3) return false;
  const int nd = A.sym_nd;
  auto kof = [&](i64 d) {
    for (int k = 0; k < nd; ++k)
      if (A.sym_off[k] == d) return k;
    return -1;
  };
  if (kof(1) < 0 || kof(-1) < 0) return false;
  int klo = nd, khi = nd;
  for (int k = nd - 1; k >= 0; --k)
  {
    if (A.sym_off[k] >= -1) klo = k;
    if (A.sym_off[k] > 1) khi = k;
  }
  // candidates for P from the widest down; the first whose four spans fit
  for (int kp = nd - 1; kp >= khi; --kp)
  {
    const i64 d = A.sym_off[kp];
    if (d % 16 != 0 || kof(-d) < 0) continue;
    sp.kPm = kof(-d);
    sp.kPp = kp;
    sp.s1b = 0, sp.s1e = sp.kPm;
    sp.s2b = sp.kPm + 1, sp.s2e = klo;
    sp.s3b = khi, sp.s3e = sp.kPp;
    sp.s4b = sp.kPp + 1, sp.s4e = nd;
    if (sp.s1e - sp.s1b <= kGSpan && sp.s2e - sp.s2b <= kGSpan && sp.s3e - sp.s3b <= kGSpan &&
        sp.s4e - sp.s4b <= kGSpan)
    {
      P = d;
      return true;
    }
  }
  return false;
}

// The general-band march (SpMM of non-extreme carried bands, Chebyshev) is a plane march too.
static bool marchg_enabled(const eig_mat_s &A) { return march_enabled(A); }

template <int EPI>
static bool launch_marchg(const eig_mat_s &A, i64 m, const double *X, double *Y, const double *Bv,
                          const double *dinv, double omega, double gamma, hipStream_t s)
{
  if (A.br != 1 || A.bc != 1 || m <= 0 || !marchg_enabled(A)) return false;
  const int mode = image_mode(A);
  if (mode != kSymN8 && mode != kSymN32) return false;
  i64 P;
  GSpans sp;
  if (!gspans(A, P, sp)) return false;
  const i64 nplanes = (A.nb_rows + P - 1) / P;
  if (nplanes < 4) return false;
  const i64 ncol = P / 16;
  const i64 resident = 6LL * 4 * A.ctx->num_cu;  // waves at the kernel's 6 waves / SIMD
  i64 nseg = std::min<i64>(std::max<i64>(1, (resident + ncol - 1) / ncol), nplanes);
  MarchPlan mp{};
  mp.D = P;
  mp.zb = 0;
  mp.nplanes = nplanes;
  mp.mrows = A.nslices * 64;
  mp.ncol = (int)ncol;
  mp.nseg = (int)nseg;
  const dim3 grid((unsigned)((ncol * mp.nseg + kWaves - 1) / kWaves), (unsigned)(m / 8));
  if (mode == kSymN8)
    hipLaunchKernelGGL((k_spmm8_marchg<uint8_t, EPI>), grid, dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset,
                       A.window, sell_b1(A), mp, sp, X, Y, Bv, dinv, omega, gamma);
  else
    hipLaunchKernelGGL((k_spmm8_marchg<uint32_t, EPI>), grid, dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset,
                       A.window, sell_b1(A), mp, sp, X, Y, Bv, dinv, omega, gamma);
  return true;
}

bool launch_cheb_march(const eig_mat_s &M, i64 m, const double *Xk, double *Xold, const double *B, const double *dinv,
                       double omega, double gamma, hipStream_t s)
{
  return launch_marchg<kGCheb>(M, m, Xk, Xold, B, dinv, omega, gamma, s);
}

bool launch_spmm_march(const eig_mat_s &A, i64 m, const double *X, double *Y, hipStream_t s)
{
  if (A.br != 1 || A.bc != 1 || m <= 0) return false;
  const int mode = image_mode(A);
  const MarchPlan mp = march_plan(A, mode, 0, -1, false, 16);
  if (mp.nseg == 0) return launch_marchg<kGStore>(A, m, X, Y, nullptr, nullptr, 0.0, 0.0, s);
  const i64 items = mp.ncol * (i64)mp.nseg;
  const dim3 grid((unsigned)((items + kWaves - 1) / kWaves), (unsigned)(m / 8));
  if (mode == kSymN8)
    hipLaunchKernelGGL((k_spmm8_march<uint8_t>), grid, dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset, A.window,
                       sell_b1(A), mp, X, Y);
  else
    hipLaunchKernelGGL((k_spmm8_march<uint32_t>), grid, dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset, A.window,
                       sell_b1(A), mp, X, Y);
  return true;
}

// Y = A X with the diagonal dots dp (k_spmm8_march<MT, true>) where the band march applies to the
// whole matrix on one rank; false otherwise (the caller runs the product and k_dot_diag_mv8).
bool launch_spmm_march_dot(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, ReduceWS red,
                           hipStream_t s)
{
  if (A.br != 1 || A.bc != 1 || m <= 0 || A.ctx->distributed()) return false;
  const int mode = image_mode(A);
  if (!is_sym_mode(mode)) return false;
  const MarchPlan mp = march_plan(A, mode, 0, -1, false, 16);
  if (mp.nseg == 0) return false;
  const i64 items = mp.ncol * (i64)mp.nseg;
  const dim3 grid((unsigned)((items + kWaves - 1) / kWaves), (unsigned)(m / 8));
  if ((i64)grid.x * 8 * grid.y > (i64)kMaxRedBlocks * kMaxRedVals || grid.y > (unsigned)kNumTickets) return false;
  if (mode == kSymN8)
    hipLaunchKernelGGL((k_spmm8_march<uint8_t, true>), grid, dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset,
                       A.window, sell_b1(A), mp, X, Y, dp, red.partials, red.ticket(0));
  else
    hipLaunchKernelGGL((k_spmm8_march<uint32_t, true>), grid, dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset,
                       A.window, sell_b1(A), mp, X, Y, dp, red.partials, red.ticket(0));
  return true;
}

// The same with the window Gram of Y (k_spmm8_march<MT, 2>), m = 8 only.
bool launch_spmm_march_dot_gram(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, double *gram,
                                ReduceWS red, hipStream_t s, unsigned *zero_word)
{
  if (A.br != 1 || A.bc != 1 || m != 8 || A.ctx->distributed()) return false;
  const int mode = image_mode(A);
  if (!is_sym_mode(mode)) return false;
  const MarchPlan mp = march_plan(A, mode, 0, -1, false, 16);
  if (mp.nseg == 0) return false;
  const i64 items = mp.ncol * (i64)mp.nseg;
  const dim3 grid((unsigned)((items + kWaves - 1) / kWaves), 1u);
  if ((i64)grid.x * 72 + 8 * 72 > (i64)kMaxRedBlocks * kMaxRedVals) return false;
  if (mode == kSymN8)
    hipLaunchKernelGGL((k_spmm8_march<uint8_t, 2>), grid, dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset,
                       A.window, sell_b1(A), mp, X, Y, dp, red.partials, red.ticket(0), gram, zero_word);
  else
    hipLaunchKernelGGL((k_spmm8_march<uint32_t, 2>), grid, dim3(kStreamThreads), 0, s, A.nb_rows, A.own_offset,
                       A.window, sell_b1(A), mp, X, Y, dp, red.partials, red.ticket(0), gram, zero_word);
  return true;
}

void lanczos_kernel_info(const eig_mat_s &A, bool fused, std::string &name, i64 &bytes)
{
  const i64 n = A.nb_rows, vec = fused ? 32 * n : 24 * n;  // fused: (t, u) pairs in + out; K1: x, u_{j-1}, t
  const int mode = A.br == 1 && A.bc == 1 ? image_mode(A) : kExplicit;
  if (is_sym_mode(mode))
  {
    bytes = 8 * (i64)A.sym_nup * n + (i64)A.sym_mask_bytes * n + vec;
    // (distributed launches with a halo take the interior / boundary split, never the march)
    const bool whole = !A.ctx->distributed() || (A.recvs.empty() && A.sends.empty());
    const bool march = whole ? (march_plan(A, mode).nseg > 0)
                             : march_split_active(A);
    // the uniform-band march streams the row mask and the vectors only; the value march (10, 11)
    // the band arrays and the vectors (geometric masks: no mask stream)
    const int mv = march && ((mode == kSymN8 && march_span1(A)) || march_kuhn(A)) ? march_uniform(A, fused) : 0;
    if (mv >= 10)
      bytes = 8 * (mv == 15 || mv == 18 || is_march2l(mv) ? 4 : (i64)A.sym_nup) * n + vec;
    else if (mv)
      bytes = (mv >= 2 ? 0 : (i64)A.sym_mask_bytes * n) + vec;
    name = fused ? (march ? "k_lanczos_fused_march" : "k_lanczos_fused_b1")
                 : (march ? "k_lanczos_spmv_march" : "k_lanczos_spmv_b1");
  }
  else
  {
    bytes = sell_image_bytes(A) + vec;
    name = fused ? "k_lanczos_fused_b1" : "k_lanczos_spmv_b1";
  }
}

// Bytes the SELL-64 slice kernels stream per pass over the image (one row per lane): every padded
// value, the 4-B column index of each explicit-slice entry, per stencil slice its width and 8
// offsets (36 B) and a 1-B mask per row, and the slice pointers -- not SURVEY 8(d)'s CSR count (the
// stencil slices read no column indices).
i64 sell_image_bytes(const eig_mat_s &A)
{
  const i64 bb = (i64)A.br * A.bc, C = 64 * (i64)A.R;
  return 8 * bb * A.nnzb_padded + 4 * A.sell_explicit + 8 * (A.nslices + 1) +
         (A.n_stencil_slices ? 4 * A.nslices + A.n_stencil_slices * (32 + C) : 0);
}

// EIG_LANCZOS_AUTO: the fused step on every 1x1 image.  (Round 3 took the two-kernel step on
// scattered images while k_lanczos_fused_b1 spilled 36-46 VGPRs there -- 634 vs 427 us on the
// scrambled + RCM 256^3 Poisson, the spill write-back being the 3.5x write excess PMC showed; at 6
// waves / SIMD without the spills it runs 408 us, step 415 vs 436 us, PMC 0.97x of the CSR bytes:
// profiles/r03ah_csr*.)
bool fused_step_pays(const eig_mat_s &A) { return A.br == 1 && A.bc == 1; }

std::string kernel_for(const eig_mat_s &A, int op)
{
  const bool b1 = A.br == 1 && A.bc == 1;
  const int mode = b1 ? image_mode(A) : kExplicit;
  const bool whole = !A.ctx->distributed() || (A.recvs.empty() && A.sends.empty());
  std::string name;
  i64 bytes;
  switch (op)
  {
    case 0:
      if (!b1) return "k_spmv_blk";
      return (whole ? march_plan(A, mode).nseg > 0 : march_split_active(A)) ? "k_spmv_march" : "k_spmv_b1";
    case 1:
    case 2:
      lanczos_kernel_info(A, op == 2, name, bytes);
      return name;
    case 3:
    case 4:
      // 3-D box stencils whose rows are class-constant: the row-class kernels for any m % 8 == 0
      if (b1 && box_prepare(A) && A.box_ctab) return op == 3 ? "k_boxc_mv8" : "k_boxc_mv8_cheb";
    {
      if (!b1) return "none";
      i64 P;
      GSpans sp;
      const bool g = marchg_enabled(A) && (mode == kSymN8 || mode == kSymN32) && gspans(A, P, sp) &&
                     (A.nb_rows + P - 1) / P >= 4;
      if (op == 3 && march_plan(A, mode, 0, -1, false, 16).nseg > 0) return "k_spmm8_march";
      if (g) return op == 3 ? "k_spmm8_marchg" : "k_spmm8_marchg_cheb";
      return op == 3 ? (b1 && A.nb_rows > 0 ? "k_sell_mv8g" : "none") : "k_sell_mv8q_cheb";
    }
    case 5:
    case 6:
      if (b1 && box_prepare(A))
      {
        if (A.box_ctab) return op == 5 ? "k_boxc_mv8" : "k_boxc_mv8_cheb";  // row-class image
        if (box_cols(A) == 16) return op == 5 ? "k_box_mv16p" : "k_box_mv16p_cheb";
        return op == 5 ? "k_box_mv32" : "k_box_mv32_cheb";
      }
      return kernel_for(A, op - 2);
    default:
      return "none";
  }
}

}  // namespace eigmi
