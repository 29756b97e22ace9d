// What bounds the plane march at 256^3?  Access-pattern microbenchmark (no matrix, no
// reductions): the fused Lanczos step's HBM streams -- read the (t, u) pair vector once, write one
// pair vector -- issued in the patterns the march kernels use, timed with HIP events.
//
//   hipcc -O3 --offload-arch=gfx950 tools/march_copy.hip -o tools/march_copy && tools/march_copy
//
// One JSON line per (pattern, plane runs): GB/s = 2 * n * 16 B / kernel time.
// `march_copy N values`: the value march's streams instead (k_vmarch; GB/s over 64 B per row).
// `march_copy N kuhn`: the P1 Kuhn march's streams (k_kmarch; GB/s over 96 B per row).
// `march_copy N box`: the C5 Chebyshev step's streams as a plain copy (k_boxcopy; 1152 B per row).
//   linear     grid-stride 16-B copy (the reference rate)
//   march      a wave owns a 64-row column of a plane run: load the +D pair, carry it, store the
//              centre (the march's stream structure, one load in flight per wave)
//   march_g    march + the two +-nx gathers of the same plane (L2 hits when the neighbour column
//              passed first)
//   march_pf   march with the +D pair loaded one plane ahead (two loads in flight per wave)
//   march_2c   two columns per wave (columns c and c + ncol / 2 interleaved: two independent loads)
//   march_t    march with temporal stores
//   *_pp       ping-pong: consecutive launches swap the input and output vectors, as the Lanczos
//              step does (its output pairs are the next step's input)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef double dpair __attribute__((ext_vector_type(2)));
constexpr int kThreads = 256, kW = kThreads / 64;

__device__ __forceinline__ int swz()
{
  const int G = gridDim.x, bid = blockIdx.x;
  if (G < 16) return bid;
  const int q = G >> 3, r = G & 7, x = bid & 7, i = bid >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

__global__ __launch_bounds__(kThreads) void k_linear(int n, const dpair *__restrict__ P, dpair *__restrict__ Q)
{
  const int stride = gridDim.x * kThreads;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
  {
    dpair v = __builtin_nontemporal_load(P + i);
    __builtin_nontemporal_store(v, Q + i);
  }
}

// MODE 0 march, 1 march + gathers, 2 prefetch, 3 temporal stores; 4 / 5: modes 0 / 3 marching the
// planes in descending order (each run from its last plane to its first)
template <int MODE>
__global__ __launch_bounds__(kThreads, 8) void k_march(int n, int D, int nx, int ncol, int nseg, int nplanes,
                                                       const dpair *__restrict__ P, dpair *__restrict__ Q)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int item = swz() * kW + wave;
  if (item >= ncol * nseg) return;
  const int col = item % ncol, seg = item / ncol;
  const int z0 = seg * nplanes / nseg, z1 = (seg + 1) * nplanes / nseg;
  const int last = n - 1;
  auto cl = [&](int g) { return g < 0 ? 0 : (g > last ? last : g); };
  if (MODE >= 4)
  {
    int w = col * 64 + lane + (z1 - 1) * D;
    dpair cur = P[cl(w)];
    for (int z = z1 - 1; z >= z0; --z, w -= D)
    {
      const dpair pd = P[cl(w - D)];
      dpair o = cur;
      o.x += pd.x * 1e-300;
      if (MODE == 5)
        Q[w] = o;
      else
        __builtin_nontemporal_store(o, Q + w);
      cur = pd;
    }
    return;
  }
  int w = col * 64 + lane + z0 * D;
  dpair cur = P[cl(w)];
  dpair nxt;
  if (MODE == 2) nxt = P[cl(w + D)];
  for (int z = z0; z < z1; ++z, w += D)
  {
    dpair pd;
    if (MODE == 2)
    {
      pd = nxt;
      nxt = P[cl(w + 2 * D)];
    }
    else
      pd = P[cl(w + D)];
    dpair o = cur;
    if (MODE == 1)
    {
      const dpair a = P[cl(w - nx)], b = P[cl(w + nx)];
      o.x += a.x + b.x;
      o.y += a.y + b.y;
    }
    o.x += pd.x * 1e-300;
    if (MODE == 3)
      Q[w] = o;
    else
      __builtin_nontemporal_store(o, Q + w);
    cur = pd;
  }
}

// The value march's streams (round 4): per row the (t, u) pair read once (+D carried) and written
// once, plus the value pack's two 16-B pairs ((+D, 0) and (+1, +nx)) read once -- 48 B read + 16 B
// written per row, the fused step's algorithmic bytes.  LIN: grid-stride order (the reference rate
// of this 3 : 1 read : write mix); G: plus the two +-nx pair gathers (L2 hits when the neighbour
// column passed first).
template <bool LIN, bool G>
__global__ __launch_bounds__(kThreads, 8) void k_vmarch(int n, int D, int nx, int ncol, int nseg, int nplanes,
                                                        const dpair *__restrict__ P, const dpair *__restrict__ V,
                                                        dpair *__restrict__ Q)
{
  if (LIN)
  {
    const int stride = gridDim.x * kThreads;
    for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
    {
      const dpair p = __builtin_nontemporal_load(P + i), a = __builtin_nontemporal_load(V + i),
                  b = __builtin_nontemporal_load(V + n + i);
      __builtin_nontemporal_store(dpair{p.x + a.x * b.y, p.y + a.y * b.x}, Q + i);
    }
    return;
  }
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int item = swz() * kW + wave;
  if (item >= ncol * nseg) return;
  const int col = item % ncol, seg = item / ncol;
  const int z0 = seg * nplanes / nseg, z1 = (seg + 1) * nplanes / nseg;
  const int last = n - 1;
  auto cl = [&](int g) { return g < 0 ? 0 : (g > last ? last : g); };
  int w = col * 64 + lane + z0 * D;
  dpair cur = P[cl(w)];
  for (int z = z0; z < z1; ++z, w += D)
  {
    const dpair pd = P[cl(w + D)];
    const dpair a = __builtin_nontemporal_load(V + w), b = __builtin_nontemporal_load(V + n + w);
    dpair o = cur;
    if (G)
    {
      const dpair u = P[cl(w - nx)], v = P[cl(w + nx)];
      o.x += u.x * b.y + v.x;
      o.y += u.y + v.y * b.y;
    }
    o.x += pd.x * a.x * 1e-300;
    o.y += a.y * b.x;
    __builtin_nontemporal_store(o, Q + w);
    cur = pd;
  }
}

// The P1 Kuhn march's streams (round 5, march variants 16 / 20): per row the (t, u) pair read once
// (+D carried) and written once, plus the Kuhn pack's FOUR 16-B value pairs ((0, +1), (+nx, +nx+1),
// (+D, +D+1), (+D+nx, +D+nx+1)) read once -- 80 B read + 16 B written per row, the Kuhn fused
// step's algorithmic bytes.  LIN: grid-stride order; G: plus the y +- 1 line gathers of plane z + 1.
template <bool LIN, bool G>
__global__ __launch_bounds__(kThreads, 8) void k_kmarch(int n, int D, int nx, int ncol, int nseg, int nplanes,
                                                        const dpair *__restrict__ P, const dpair *__restrict__ V,
                                                        dpair *__restrict__ Q)
{
  if (LIN)
  {
    const int stride = gridDim.x * kThreads;
    for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
    {
      const dpair p = __builtin_nontemporal_load(P + i), a = __builtin_nontemporal_load(V + i),
                  b = __builtin_nontemporal_load(V + n + i), c = __builtin_nontemporal_load(V + 2 * (size_t)n + i),
                  d = __builtin_nontemporal_load(V + 3 * (size_t)n + i);
      __builtin_nontemporal_store(dpair{p.x + a.x * b.y + c.x * d.y, p.y + a.y * b.x + c.y * d.x}, Q + i);
    }
    return;
  }
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int item = swz() * kW + wave;
  if (item >= ncol * nseg) return;
  const int col = item % ncol, seg = item / ncol;
  const int z0 = seg * nplanes / nseg, z1 = (seg + 1) * nplanes / nseg;
  const int last = n - 1;
  auto cl = [&](int g) { return g < 0 ? 0 : (g > last ? last : g); };
  int w = col * 64 + lane + z0 * D;
  dpair cur = P[cl(w)];
  for (int z = z0; z < z1; ++z, w += D)
  {
    const dpair pd = P[cl(w + D)];
    const dpair a = V[w], b = V[n + w], c = __builtin_nontemporal_load(V + 2 * (size_t)n + w),
                d = V[3 * (size_t)n + w];
    dpair o = cur;
    if (G)
    {
      const dpair u = P[cl(w + D - nx)], v = P[cl(w + D + nx)];
      o.x += u.x * b.y + v.x;
      o.y += u.y + v.y * d.y;
    }
    o.x += pd.x * a.x * 1e-300 + c.x * d.x;
    o.y += a.y * b.x + c.y;
    __builtin_nontemporal_store(o, Q + w);
    cur = pd;
  }
}

// The C5 Chebyshev step's streams (k_box_mv32_cheb, 32 columns, P1 Kuhn box image): per row X,
// x_{k-1} and B read (3 x 256 B), the 15 box-image values + D^-1 read (128 B), the result written
// (256 B) -- 1152 B per row, no halo, no matrix arithmetic: a plain grid-stride stream of the
// kernel's own bytes (16 lanes per row, one 16-B piece of each 256-B row per lane).
__global__ __launch_bounds__(kThreads) void k_boxcopy(int nrows, const dpair *__restrict__ X, const dpair *__restrict__ Xo,
                                                      const dpair *__restrict__ B, const double *__restrict__ V,
                                                      dpair *__restrict__ Y)
{
  const long total = (long)nrows * 16;
  const long stride = (long)gridDim.x * kThreads;
  for (long t = (long)blockIdx.x * kThreads + threadIdx.x; t < total; t += stride)
  {
    const long r = t >> 4;
    const int q = (int)(t & 15);
    const dpair x = __builtin_nontemporal_load(X + t), xo = __builtin_nontemporal_load(Xo + t),
                b = __builtin_nontemporal_load(B + t);
    (void)r;
    (void)q;
    const double v = __builtin_nontemporal_load(V + t);  // the row's 15 values + D^-1, read coalesced
    __builtin_nontemporal_store(dpair{x.x + v * (b.x - xo.x), x.y + v * (b.y - xo.y)}, Y + t);
  }
}

// Ablation of the value march toward the fused step (round 5): k_vmarch<false, true> (the streams +
// the +-nx gathers) plus, by flag, EDGE = lane 0 / lane 63 load the pair past their end of the
// 64-row line (exec-masked), ARITH = the fused step's per-row arithmetic (u = t - c u for the 7
// operands, the 7 products in order, the t / u epilogue), RED = its three running sums reduced per
// wave and added once per wave; built for W waves per SIMD.
template <bool EDGE, bool ARITH, bool RED, int W, bool MIR = false, int POL = 0, bool TAIL = false>
__global__ __launch_bounds__(kThreads, W) void k_vabl(int n, int D, int nx, int ncol, int nseg, int nplanes,
                                                      const dpair *__restrict__ P, const dpair *__restrict__ V,
                                                      dpair *__restrict__ Q, double *__restrict__ sums, double c)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int item = swz() * kW + wave;
  if (item >= ncol * nseg) return;  // (the grid covers the items exactly: no workgroup leaves early)
  const int col = item % ncol, seg = item / ncol;
  const int z0 = seg * nplanes / nseg, z1 = (seg + 1) * nplanes / nseg;
  const int lastrow = n - 1;
  auto cl = [&](int g) { return g < 0 ? 0 : (g > lastrow ? lastrow : g); };
  int w = col * 64 + lane + z0 * D;
  dpair cur = P[cl(w)];
  dpair prev = P[cl(w - D)];
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (int z = z0; z < z1; ++z, w += D)
  {
    const dpair pd = P[cl(w + D)];
    // POL 1: the (+1, +nx) stream with the default cache policy (its lines stay in L2 for the
    // -nx mirror gather of line y + 1); 2: also no lane-0 -1 value load (DPP only)
    const dpair a = __builtin_nontemporal_load(V + w), b = POL ? V[n + w] : __builtin_nontemporal_load(V + n + w);
    const dpair u = P[cl(w - nx)], v = P[cl(w + nx)];
    dpair e = dpair{0.0, 0.0};
    if (EDGE && (lane == 0 || lane == 63)) e = P[cl(lane == 0 ? w - 1 : w + 1)];
    // MIR: the mirrored lower values -- -nx from the (+1, +nx) pair of row w - nx (an L2 gather),
    // -1 by lane shift of the +1 value with lane 0's own (w - 1) load
    double mnx = 0.0, m1e = 0.0;
    if (MIR)
    {
      mnx = V[n + cl(w - nx)].y;
      if (POL < 2 && lane == 0) m1e = V[n + cl(w - 1)].x;
    }
    dpair o;
    if (ARITH)
    {
      auto uk = [&](dpair p) { return p.x - c * p.y; };
      const double vc = uk(cur);
      const double vl = __shfl_up(vc, 1, 64), vr = __shfl_down(vc, 1, 64);
      double acc = 0.0;
      const double am1 = MIR ? (lane == 0 ? m1e : __shfl_up(b.x, 1, 64)) : b.x;
      acc += b.y * uk(prev);
      acc += (MIR ? mnx : a.y) * uk(u);
      acc += am1 * (lane == 0 ? uk(e) : vl);
      acc += a.x * vc;
      acc += b.x * (lane == 63 ? uk(e) : vr);
      acc += b.y * uk(v);
      acc += a.x * uk(pd);
      const double t = (acc - 0.5 * vc) * 0.25 - 0.125 * cur.y;
      o = dpair{t, vc};
      if (RED)
      {
        s0 += t * vc;
        s1 += t * t;
        s2 += vc * vc;
      }
    }
    else
    {
      o = cur;
      o.x += u.x * b.y + v.x + e.x;
      o.y += u.y + v.y * b.y + e.y;
      o.x += pd.x * a.x * 1e-300;
      o.y += a.y * b.x;
    }
    __builtin_nontemporal_store(o, Q + w);
    prev = cur;
    cur = pd;
  }
  if (RED)
  {
    for (int off = 32; off > 0; off >>= 1)
    {
      s0 += __shfl_down(s0, off, 64);
      s1 += __shfl_down(s1, off, 64);
      s2 += __shfl_down(s2, off, 64);
    }
    if (!TAIL && lane == 0)  // one slot per wave (no contention; the fused step's partials + ticket tail aside)
    {
      sums[3 * item] = s0;
      sums[3 * item + 1] = s1;
      sums[3 * item + 2] = s2;
    }
    if (TAIL)
    {
      // the fused step's tail: workgroup sums -> partials, a ticket, the last workgroup sums them
      __shared__ double ws[kW][3];
      __shared__ int last;
      if (lane == 0)
      {
        ws[wave][0] = s0;
        ws[wave][1] = s1;
        ws[wave][2] = s2;
      }
      __syncthreads();
      double *part = sums + 64;
      unsigned *ticket = reinterpret_cast<unsigned *>(sums);
      if (threadIdx.x < 3)
      {
        double t = 0.0;
        for (int q = 0; q < kW; ++q) t += ws[q][threadIdx.x];
        __hip_atomic_store(reinterpret_cast<unsigned long long *>(part + 3 * blockIdx.x + threadIdx.x),
                           (unsigned long long)__double_as_longlong(t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
      __syncthreads();
      if (last)
      {
        double a0 = 0.0, a1 = 0.0, a2 = 0.0;
        for (unsigned b = threadIdx.x; b < gridDim.x; b += kThreads)
        {
          a0 += __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<unsigned long long *>(part + 3 * b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          a1 += __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<unsigned long long *>(part + 3 * b + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          a2 += __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<unsigned long long *>(part + 3 * b + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
        for (int off = 32; off > 0; off >>= 1)
        {
          a0 += __shfl_down(a0, off, 64);
          a1 += __shfl_down(a1, off, 64);
          a2 += __shfl_down(a2, off, 64);
        }
        if (lane == 0) atomicAdd(sums + 8, a0 + a1 + a2);
        if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// The full ablation step (k_vabl<true, true, true, W, true, 1, true>) with TWO grid lines per wave
// (round 6 probe): lane = x, the wave's lines y0 = 2 ly and y0 + 1, so the +nx operand of line y0 and
// the -nx operand and mirrored -nx value of line y0 + 1 are the other line's registers; only line
// y0 - 1's operand and mirrored value and line y0 + 2's operand are gathered (half the gathers).
template <int W>
__global__ __launch_bounds__(kThreads, W) void k_vabl2(int n, int D, int nx, int ncol, int nseg, int nplanes,
                                                       const dpair *__restrict__ P, const dpair *__restrict__ V,
                                                       dpair *__restrict__ Q, double *__restrict__ sums, double c)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ncol2 = ncol / 2, xc = nx / 64;
  const int item = swz() * kW + wave;
  if (item >= ncol2 * nseg) return;
  const int col2 = item % ncol2, seg = item / ncol2;
  const int z0 = seg * nplanes / nseg, z1 = (seg + 1) * nplanes / nseg;
  const int lastrow = n - 1;
  auto cl = [&](int g) { return g < 0 ? 0 : (g > lastrow ? lastrow : g); };
  const int line0 = 2 * (col2 / xc);
  int w = line0 * nx + (col2 % xc) * 64 + lane + z0 * D;  // row of line y0; line y0 + 1 at w + nx
  dpair cur0 = P[cl(w)], cur1 = P[cl(w + nx)];
  dpair prev0 = P[cl(w - D)], prev1 = P[cl(w + nx - D)];
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  auto uk = [&](dpair p) { return p.x - c * p.y; };
  for (int z = z0; z < z1; ++z, w += D)
  {
    const dpair pd0 = P[cl(w + D)], pd1 = P[cl(w + nx + D)];
    const dpair a0 = __builtin_nontemporal_load(V + w), b0 = V[n + w];
    const dpair a1 = __builtin_nontemporal_load(V + w + nx), b1 = V[n + w + nx];
    const dpair u = P[cl(w - nx)], v = P[cl(w + 2 * nx)];
    dpair e0 = dpair{0.0, 0.0}, e1 = dpair{0.0, 0.0};
    if (lane == 0 || lane == 63)
    {
      e0 = P[cl(lane == 0 ? w - 1 : w + 1)];
      e1 = P[cl(lane == 0 ? w + nx - 1 : w + nx + 1)];
    }
    const double mnx0 = V[n + cl(w - nx)].y;
    double m1e0 = 0.0, m1e1 = 0.0;
    if (lane == 0)
    {
      m1e0 = V[n + cl(w - 1)].x;
      m1e1 = V[n + cl(w + nx - 1)].x;
    }
    const double vc0 = uk(cur0), vc1 = uk(cur1);
    auto row = [&](dpair a, dpair b, dpair prev, double mnx, double vn, double m1e, dpair e, double vc, double vq,
                   dpair pd, dpair cur) {
      const double vl = __shfl_up(vc, 1, 64), vr = __shfl_down(vc, 1, 64);
      const double am1 = lane == 0 ? m1e : __shfl_up(b.x, 1, 64);
      double acc = 0.0;
      acc += b.y * uk(prev);
      acc += mnx * vn;
      acc += am1 * (lane == 0 ? uk(e) : vl);
      acc += a.x * vc;
      acc += b.x * (lane == 63 ? uk(e) : vr);
      acc += b.y * vq;
      acc += a.x * uk(pd);
      const double t = (acc - 0.5 * vc) * 0.25 - 0.125 * cur.y;
      s0 += t * vc;
      s1 += t * t;
      s2 += vc * vc;
      return dpair{t, vc};
    };
    const dpair o0 = row(a0, b0, prev0, mnx0, uk(u), m1e0, e0, vc0, vc1, pd0, cur0);
    const dpair o1 = row(a1, b1, prev1, b0.y, vc0, m1e1, e1, vc1, uk(v), pd1, cur1);
    __builtin_nontemporal_store(o0, Q + w);
    __builtin_nontemporal_store(o1, Q + w + nx);
    prev0 = cur0;
    prev1 = cur1;
    cur0 = pd0;
    cur1 = pd1;
  }
  for (int off = 32; off > 0; off >>= 1)
  {
    s0 += __shfl_down(s0, off, 64);
    s1 += __shfl_down(s1, off, 64);
    s2 += __shfl_down(s2, off, 64);
  }
  __shared__ double ws[kW][3];
  __shared__ int last;
  if (lane == 0)
  {
    ws[wave][0] = s0;
    ws[wave][1] = s1;
    ws[wave][2] = s2;
  }
  __syncthreads();
  double *part = sums + 64;
  unsigned *ticket = reinterpret_cast<unsigned *>(sums);
  if (threadIdx.x < 3)
  {
    double t = 0.0;
    for (int q = 0; q < kW; ++q) t += ws[q][threadIdx.x];
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(part + 3 * blockIdx.x + threadIdx.x),
                       (unsigned long long)__double_as_longlong(t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (last)
  {
    double a0 = 0.0;
    for (unsigned b = threadIdx.x; b < 3 * gridDim.x; b += kThreads)
      a0 += __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<unsigned long long *>(part + b),
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    for (int off = 32; off > 0; off >>= 1) a0 += __shfl_down(a0, off, 64);
    if (lane == 0) atomicAdd(sums + 8, a0);
    if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The same with LN grid lines per wave (LN = 2 reproduces k_vabl2's loads): lines y0 .. y0 + LN - 1,
// only line y0 - 1's operand / mirrored value and line y0 + LN's operand gathered
template <int LN, int W>
__global__ __launch_bounds__(kThreads, W) void k_vablN(int n, int D, int nx, int ncol, int nseg, int nplanes,
                                                       const dpair *__restrict__ P, const dpair *__restrict__ V,
                                                       dpair *__restrict__ Q, double *__restrict__ sums, double c)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ncolN = ncol / LN, xc = nx / 64;
  const int item = swz() * kW + wave;
  if (item >= ncolN * nseg) return;
  const int colN = item % ncolN, seg = item / ncolN;
  const int z0 = seg * nplanes / nseg, z1 = (seg + 1) * nplanes / nseg;
  const int lastrow = n - 1;
  auto cl = [&](int g) { return g < 0 ? 0 : (g > lastrow ? lastrow : g); };
  const int line0 = LN * (colN / xc);
  int w = line0 * nx + (colN % xc) * 64 + lane + z0 * D;
  dpair cur[LN], prev[LN];
#pragma unroll
  for (int l = 0; l < LN; ++l)
  {
    cur[l] = P[cl(w + l * nx)];
    prev[l] = P[cl(w + l * nx - D)];
  }
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  auto uk = [&](dpair p) { return p.x - c * p.y; };
  for (int z = z0; z < z1; ++z, w += D)
  {
    dpair pd[LN], a[LN], b[LN], e[LN];
    double m1e[LN];
#pragma unroll
    for (int l = 0; l < LN; ++l)
    {
      pd[l] = P[cl(w + l * nx + D)];
      a[l] = __builtin_nontemporal_load(V + w + l * nx);
      b[l] = V[n + w + l * nx];
      e[l] = dpair{0.0, 0.0};
      if (lane == 0 || lane == 63) e[l] = P[cl(lane == 0 ? w + l * nx - 1 : w + l * nx + 1)];
      m1e[l] = lane == 0 ? V[n + cl(w + l * nx - 1)].x : 0.0;
    }
    const dpair u = P[cl(w - nx)], v = P[cl(w + LN * nx)];
    const double mnx0 = V[n + cl(w - nx)].y;
    double vc[LN];
#pragma unroll
    for (int l = 0; l < LN; ++l) vc[l] = uk(cur[l]);
#pragma unroll
    for (int l = 0; l < LN; ++l)
    {
      const double vl = __shfl_up(vc[l], 1, 64), vr = __shfl_down(vc[l], 1, 64);
      const double am1 = lane == 0 ? m1e[l] : __shfl_up(b[l].x, 1, 64);
      const double mnx = l == 0 ? mnx0 : b[l > 0 ? l - 1 : 0].y;
      const double vn = l == 0 ? uk(u) : vc[l > 0 ? l - 1 : 0];
      const double vq = l == LN - 1 ? uk(v) : vc[l < LN - 1 ? l + 1 : 0];
      double acc = 0.0;
      acc += b[l].y * uk(prev[l]);
      acc += mnx * vn;
      acc += am1 * (lane == 0 ? uk(e[l]) : vl);
      acc += a[l].x * vc[l];
      acc += b[l].x * (lane == 63 ? uk(e[l]) : vr);
      acc += b[l].y * vq;
      acc += a[l].x * uk(pd[l]);
      const double t = (acc - 0.5 * vc[l]) * 0.25 - 0.125 * cur[l].y;
      s0 += t * vc[l];
      s1 += t * t;
      s2 += vc[l] * vc[l];
      __builtin_nontemporal_store(dpair{t, vc[l]}, Q + w + l * nx);
    }
#pragma unroll
    for (int l = 0; l < LN; ++l)
    {
      prev[l] = cur[l];
      cur[l] = pd[l];
    }
  }
  for (int off = 32; off > 0; off >>= 1)
  {
    s0 += __shfl_down(s0, off, 64);
    s1 += __shfl_down(s1, off, 64);
    s2 += __shfl_down(s2, off, 64);
  }
  if (lane == 0) atomicAdd(sums + 8, s0 + s1 + s2);  // (no tail: compare with abl_full_notail_w6)
}

// two columns per wave: c and c + ncol / 2 (ncol even)
__global__ __launch_bounds__(kThreads, 8) void k_march2(int n, int D, int ncol, int nseg, int nplanes,
                                                        const dpair *__restrict__ P, dpair *__restrict__ Q)
{
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = ncol / 2;
  const int item = swz() * kW + wave;
  if (item >= h * nseg) return;
  const int col = item % h, seg = item / h;
  const int z0 = seg * nplanes / nseg, z1 = (seg + 1) * nplanes / nseg;
  const int last = n - 1;
  auto cl = [&](int g) { return g < 0 ? 0 : (g > last ? last : g); };
  int w = col * 64 + lane + z0 * D;
  const int o2 = h * 64;
  dpair c0 = P[cl(w)], c1 = P[cl(w + o2)];
  for (int z = z0; z < z1; ++z, w += D)
  {
    const dpair p0 = P[cl(w + D)], p1 = P[cl(w + o2 + D)];
    dpair a = c0, b = c1;
    a.x += p0.x * 1e-300;
    b.x += p1.x * 1e-300;
    __builtin_nontemporal_store(a, Q + w);
    __builtin_nontemporal_store(b, Q + w + o2);
    c0 = p0;
    c1 = p1;
  }
}

int main(int argc, char **argv)
{
  const int N = argc > 1 ? std::atoi(argv[1]) : 256;
  // MC_NZ: planes of the grid (default N; 32 = one rank's slab of the 8-GPU split of 256^3)
  const int NZ = std::getenv("MC_NZ") ? std::atoi(std::getenv("MC_NZ")) : N;
  const int n = N * N * NZ, D = N * N, nx = N, ncol = D / 64;
  if (D % 64 != 0 || (ncol & 1)) return 2;
  dpair *P, *Q;
  CK(hipMalloc(&P, (size_t)n * sizeof(dpair)));
  CK(hipMalloc(&Q, (size_t)n * sizeof(dpair)));
  CK(hipMemset(P, 0, (size_t)n * sizeof(dpair)));
  CK(hipMemset(Q, 0, (size_t)n * sizeof(dpair)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 2.0 * n * sizeof(dpair);
  int rep = 0;  // ping-pong launches read P on even reps, Q on odd ones
  auto time = [&](auto launch) {
    for (int i = 0; i < 3; ++i, ++rep) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int i = 0; i < 20; ++i)
    {
      CK(hipEventRecord(e0));
      launch();
      ++rep;
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return (double)t[t.size() / 2] * 1e3;  // median us
  };
  auto out = [&](const char *pat, int nseg, double us) {
    std::printf("{\"pattern\": \"%s\", \"N\": %d, \"runs\": %d, \"us\": %.2f, \"GBs\": %.1f}\n", pat, N, nseg, us,
                bytes / us * 1e-3);
    std::fflush(stdout);
  };
  const char *only = argc > 2 ? argv[2] : "";
  if (std::string(only) == "box")
  {
    // the C5 Chebyshev step's 1152 B per row (GB/s over those bytes)
    dpair *X, *Xo, *B, *Y;
    double *V;
    const size_t nb = (size_t)n * 16 * sizeof(dpair);
    CK(hipMalloc(&X, nb));
    CK(hipMalloc(&Xo, nb));
    CK(hipMalloc(&B, nb));
    CK(hipMalloc(&Y, nb));
    CK(hipMalloc(&V, (size_t)16 * n * sizeof(double)));
    CK(hipMemset(X, 0, nb));
    CK(hipMemset(Xo, 0, nb));
    CK(hipMemset(B, 0, nb));
    CK(hipMemset(V, 0, (size_t)16 * n * sizeof(double)));
    for (int g : {2048, 4096, 8192})
    {
      const double us = time([&] { k_boxcopy<<<g, kThreads>>>(n, rep & 1 ? Y : X, Xo, B, V, rep & 1 ? X : Y); });
      std::printf("{\"pattern\": \"box_cheb_linear_pp\", \"N\": %d, \"grid\": %d, \"us\": %.2f, \"GBs\": %.1f}\n", N, g,
                  us, 1152.0 * n / us * 1e-3);
      std::fflush(stdout);
    }
    CK(hipGetLastError());
    return 0;
  }
  if (std::string(only) == "kuhn")
  {
    // the Kuhn march's streams: 80 B read + 16 B written per row (GB/s over those 96 B)
    dpair *V;
    CK(hipMalloc(&V, (size_t)4 * n * sizeof(dpair)));
    CK(hipMemset(V, 0, (size_t)4 * n * sizeof(dpair)));
    auto src = [&] { return rep & 1 ? Q : P; };
    auto dst = [&] { return rep & 1 ? P : Q; };
    auto outk = [&](const char *pat, int nseg, double us) {
      std::printf("{\"pattern\": \"%s\", \"N\": %d, \"runs\": %d, \"us\": %.2f, \"GBs\": %.1f}\n", pat, N, nseg,
                  us, 6.0 * n * sizeof(dpair) / us * 1e-3);
      std::fflush(stdout);
    };
    for (int g : {2048, 4096, 8192})
      outk("kuhn_linear_pp", g, time([&] { k_kmarch<true, false><<<g, kThreads>>>(n, D, nx, ncol, 1, N, src(), V, dst()); }));
    for (int nseg : {4, 6, 8, 12})
    {
      const int items = ncol * nseg, G = (items + kW - 1) / kW;
      outk("kuhn_march_pp", nseg, time([&] { k_kmarch<false, false><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, src(), V, dst()); }));
      outk("kuhn_march_g_pp", nseg, time([&] { k_kmarch<false, true><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, src(), V, dst()); }));
    }
    CK(hipGetLastError());
    CK(hipFree(V));
    CK(hipFree(P));
    CK(hipFree(Q));
    return 0;
  }
  if (std::string(only) == "values")
  {
    // the value march's streams: 48 B read + 16 B written per row (GB/s over those 64 B)
    dpair *V;
    CK(hipMalloc(&V, (size_t)2 * n * sizeof(dpair)));
    CK(hipMemset(V, 0, (size_t)2 * n * sizeof(dpair)));
    auto src = [&] { return rep & 1 ? Q : P; };
    auto dst = [&] { return rep & 1 ? P : Q; };
    auto outv = [&](const char *pat, int nseg, double us) {
      std::printf("{\"pattern\": \"%s\", \"N\": %d, \"runs\": %d, \"us\": %.2f, \"GBs\": %.1f}\n", pat, N, nseg,
                  us, 4.0 * n * sizeof(dpair) / us * 1e-3);
      std::fflush(stdout);
    };
    for (int g : {2048, 4096, 8192})
      outv("values_linear_pp", g, time([&] { k_vmarch<true, false><<<g, kThreads>>>(n, D, nx, ncol, 1, N, src(), V, dst()); }));
    for (int nseg : {1, 2, 4, 6, 8, 12, 16})
    {
      if (nseg > NZ) continue;
      const int items = ncol * nseg, G = (items + kW - 1) / kW;
      outv("values_march_pp", nseg, time([&] { k_vmarch<false, false><<<G, kThreads>>>(n, D, nx, ncol, nseg, NZ, src(), V, dst()); }));
      outv("values_march_g_pp", nseg, time([&] { k_vmarch<false, true><<<G, kThreads>>>(n, D, nx, ncol, nseg, NZ, src(), V, dst()); }));
    }
    if (argc > 3 && std::string(argv[3]) == "ablation")
    {
      double *sums;
      const int nseg = argc > 4 ? std::atoi(argv[4]) : 8, items = ncol * nseg, G = (items + kW - 1) / kW;
      CK(hipMalloc(&sums, (size_t)(3 * items + 64) * sizeof(double)));
      CK(hipMemset(sums, 0, (size_t)(3 * items + 64) * sizeof(double)));
#define ABL(NAME, E, A, R, W_, ...)                                                                              \
  outv(NAME, nseg, time([&] { k_vabl<E, A, R, W_, ##__VA_ARGS__><<<G, kThreads>>>(n, D, nx, ncol, nseg, NZ, src(), V, dst(), sums, 0.5); }))
      ABL("abl_g_w8", false, false, false, 8);
      ABL("abl_g_edge_w8", true, false, false, 8);
      ABL("abl_g_edge_arith_w8", true, true, false, 8);
      ABL("abl_g_edge_arith_red_w8", true, true, true, 8);
      ABL("abl_g_edge_arith_red_w6", true, true, true, 6);
      ABL("abl_g_w6", false, false, false, 6);
      ABL("abl_g_edge_arith_red_mir_w8", true, true, true, 8, true);
      ABL("abl_g_edge_arith_red_mir_w6", true, true, true, 6, true);
      ABL("abl_g_edge_arith_red_mir_pol1_w8", true, true, true, 8, true, 1);
      ABL("abl_g_edge_arith_red_mir_pol2_w8", true, true, true, 8, true, 2);
      ABL("abl_g_edge_arith_red_pol1_w8", true, true, true, 8, false, 1);
      ABL("abl_full_tail_w6", true, true, true, 6, true, 1, true);
      ABL("abl_full_notail_w6", true, true, true, 6, true, 1, false);
#undef ABL
      // two lines per wave (half the items): W = 4 / 5 / 6 waves per SIMD
      const int G2 = ((ncol / 2) * nseg + kW - 1) / kW;
      outv("abl_full_tail_2lines_w4", nseg, time([&] { k_vabl2<4><<<G2, kThreads>>>(n, D, nx, ncol, nseg, NZ, src(), V, dst(), sums, 0.5); }));
      outv("abl_full_tail_2lines_w5", nseg, time([&] { k_vabl2<5><<<G2, kThreads>>>(n, D, nx, ncol, nseg, NZ, src(), V, dst(), sums, 0.5); }));
      outv("abl_full_tail_2lines_w6", nseg, time([&] { k_vabl2<6><<<G2, kThreads>>>(n, D, nx, ncol, nseg, NZ, src(), V, dst(), sums, 0.5); }));
      for (int ns : {4, 8, 16})
      {
        const int G4 = ((ncol / 4) * ns + kW - 1) / kW, GN2 = ((ncol / 2) * ns + kW - 1) / kW;
        outv("abl_notail_lines2_w5", ns, time([&] { k_vablN<2, 5><<<GN2, kThreads>>>(n, D, nx, ncol, ns, NZ, src(), V, dst(), sums, 0.5); }));
        outv("abl_notail_lines4_w3", ns, time([&] { k_vablN<4, 3><<<G4, kThreads>>>(n, D, nx, ncol, ns, NZ, src(), V, dst(), sums, 0.5); }));
        outv("abl_notail_lines4_w4", ns, time([&] { k_vablN<4, 4><<<G4, kThreads>>>(n, D, nx, ncol, ns, NZ, src(), V, dst(), sums, 0.5); }));
      }
      outv("abl_full_tail_w6_again", nseg, time([&] { k_vabl<true, true, true, 6, true, 1, true><<<G, kThreads>>>(n, D, nx, ncol, nseg, NZ, src(), V, dst(), sums, 0.5); }));
      CK(hipFree(sums));
    }
    CK(hipGetLastError());
    CK(hipFree(V));
    CK(hipFree(P));
    CK(hipFree(Q));
    return 0;
  }
  for (int g : {1024, 2048, 4096, 8192})
    out("linear", g, time([&] { k_linear<<<g, kThreads>>>(n, P, Q); }));
  auto src = [&] { return rep & 1 ? Q : P; };
  auto dst = [&] { return rep & 1 ? P : Q; };
  out("linear_pp", 2048, time([&] { k_linear<<<2048, kThreads>>>(n, src(), dst()); }));
  for (int nseg : {6, 8})
  {
    const int items = ncol * nseg, G = (items + kW - 1) / kW;
    // alternating direction: odd launches march down, so they start on the planes the previous
    // launch wrote last (what a memory-side cache still holds)
    out("march_alt_pp", nseg, time([&] {
      if (rep & 1)
        k_march<4><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, src(), dst());
      else
        k_march<0><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, src(), dst());
    }));
    out("march_alt_t_pp", nseg, time([&] {
      if (rep & 1)
        k_march<5><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, src(), dst());
      else
        k_march<3><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, src(), dst());
    }));
    out("march_pp", nseg, time([&] { k_march<0><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, src(), dst()); }));
    out("march_g_pp", nseg, time([&] { k_march<1><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, src(), dst()); }));
    out("march_t_pp", nseg, time([&] { k_march<3><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, src(), dst()); }));
  }
  for (int nseg : {4, 6, 8, 12, 16, 32})
  {
    const int items = ncol * nseg, G = (items + kW - 1) / kW;
    out("march", nseg, time([&] { k_march<0><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, P, Q); }));
    out("march_g", nseg, time([&] { k_march<1><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, P, Q); }));
    out("march_pf", nseg, time([&] { k_march<2><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, P, Q); }));
    out("march_t", nseg, time([&] { k_march<3><<<G, kThreads>>>(n, D, nx, ncol, nseg, N, P, Q); }));
    const int G2 = (ncol / 2 * nseg + kW - 1) / kW;
    out("march_2c", nseg, time([&] { k_march2<<<G2, kThreads>>>(n, D, ncol, nseg, N, P, Q); }));
  }
  CK(hipGetLastError());
  CK(hipFree(P));
  CK(hipFree(Q));
  return 0;
}
