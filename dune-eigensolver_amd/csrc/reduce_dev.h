// reduce_dev.h -- deterministic grid-wide reductions for gfx950.
//
// Pattern (MI355X_MICROARCH "Valid forms", first row): every workgroup reduces its values
// (wave shuffle tree + LDS, fixed order), ONE wave stores the block partials write-through
// (`sc1`, agent-scope relaxed atomic stores), every wave drains `s_waitcnt vmcnt(0)`, a
// workgroup barrier, then ONE lane takes an agent-scope ticket.  The workgroup whose ticket
// comes last reads all partials with `sc1` loads and sums them in block-index order, so the
// result does not depend on dispatch order or XCD placement and is bitwise reproducible.
// The last workgroup also resets the ticket to zero for the next launch on the stream.
#pragma once
#include <hip/hip_runtime.h>

namespace eigmi {

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;  // valid in lane 0
}

__device__ __forceinline__ void st_sc1(double *p, double v)
{
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p)
{
  unsigned long long b = __hip_atomic_load(reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
  return __longlong_as_double((long long)b);
}

// Sharded arrival ticket (internal.h kTicketStride): workgroup bid adds to shard bid % 8; the
// workgroup that completes a shard adds to the top counter; the one that completes the top is
// the last of all.  Called by ONE lane after the workgroup's partial stores have drained.
// Returns true for exactly one workgroup of the launch.
__device__ __forceinline__ bool ticket_arrive(unsigned *t, unsigned bid, unsigned nblk)
{
  constexpr unsigned L = 32;  // words per 128-B line
  const unsigned shard = bid & 7u;
  const unsigned shard_n = nblk / 8u + ((shard < nblk % 8u) ? 1u : 0u);
  const unsigned nshards = nblk < 8u ? nblk : 8u;
  const unsigned prev = __hip_atomic_fetch_add(t + shard * L, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (prev != shard_n - 1u) return false;
  const unsigned top = __hip_atomic_fetch_add(t + 8u * L, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return top == nshards - 1u;
}

__device__ __forceinline__ void ticket_reset(unsigned *t)
{
  for (unsigned i = 0; i < 9u; ++i) __hip_atomic_store(t + i * 32u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Block-wide sum of NV values per thread, in a fixed order.  Result valid in thread 0's out[].
template <int NV, int NT>
__device__ __forceinline__ void block_sum(double (&v)[NV], double (&out)[NV])
{
  __shared__ double sh[NT / 64][NV];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i)
  {
    double w = wave_sum(v[i]);
    if (lane == 0) sh[wid][i] = w;
  }
  __syncthreads();
  if (threadIdx.x == 0)
  {
#pragma unroll
    for (int i = 0; i < NV; ++i)
    {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) s += sh[w][i];
      out[i] = s;
    }
  }
}

// Grid-wide sum.  Returns true in every thread of the LAST workgroup; there tot[0..NV) (LDS,
// visible to all its threads) holds the grid totals.  partials: >= gridDim.x*NV doubles.
// U: partials per thread and value loaded in one round of the last workgroup's sum (a kernel with
// registers to spare passes 8: the fused march step's 2048 x 3 partials in one round)
template <int NV, int NT, int U = (NV <= 2 ? 8 : 2)>
__device__ bool grid_sum_n(double (&v)[NV], double *partials, unsigned *ticket, double *tot, unsigned bid,
                           unsigned nblk);

template <int NV, int NT, int U = (NV <= 2 ? 8 : 2)>
__device__ __forceinline__ bool grid_sum(double (&v)[NV], double *partials, unsigned *ticket, double *tot)
{
  return grid_sum_n<NV, NT, U>(v, partials, ticket, tot, blockIdx.x, gridDim.x);
}

// Same with an explicit reduction group: `nblk` workgroups with ids `bid` share one ticket and
// partials[0 .. nblk*NV) (used by 2-D grids that run several independent reductions).
template <int NV, int NT, int U>
__device__ bool grid_sum_n(double (&v)[NV], double *partials, unsigned *ticket, double *tot, unsigned bid,
                           unsigned nblk)
{
  __shared__ unsigned s_last;
  double bs[NV];
  block_sum<NV, NT>(v, bs);
  if (threadIdx.x == 0)
  {
#pragma unroll
    for (int i = 0; i < NV; ++i) st_sc1(&partials[(size_t)bid * NV + i], bs[i]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) s_last = ticket_arrive(ticket, bid, nblk) ? 1u : 0u;
  __syncthreads();
  if (!s_last) return false;
  // Last workgroup: thread t sums partials t, t+NT, ... then a fixed-order block tree.  The loads
  // of a round are issued together (independent sc1 loads) before any add, so the tail pays about
  // one memory latency per 8 partials per thread instead of one per partial.
  double acc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) acc[i] = 0.0;
  for (unsigned b0 = threadIdx.x; b0 < nblk; b0 += NT * U)
  {
    double vals[U][NV];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      const unsigned b = b0 + (unsigned)u * NT;
#pragma unroll
      for (int i = 0; i < NV; ++i) vals[u][i] = (b < nblk) ? ld_sc1(&partials[(size_t)b * NV + i]) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < NV; ++i) acc[i] += vals[u][i];
  }
  double r[NV];
  block_sum<NV, NT>(acc, r);
  if (threadIdx.x == 0)
  {
#pragma unroll
    for (int i = 0; i < NV; ++i) tot[i] = r[i];
    ticket_reset(ticket);
  }
  __syncthreads();
  return true;
}

// Two-level grid reduction of E values per workgroup (vals: the workgroup's block sums, in LDS).
// The ticket's shards double as reduction groups: the workgroup completing shard s (members
// bid = s, s + 8, ...) sums the shard's partials in bid order into spart[s]; the workgroup
// completing the top sums the <= 8 shard sums in shard order into out (LDS) and returns true.
// Deterministic like grid_sum_n, but the tail reads nblk / 8 partials per element in 8 workgroups
// at once instead of nblk in one.  part: >= nblk E doubles, spart: >= 8 E doubles.
template <int NT>
__device__ bool grid_sum2(const double *vals, int E, double *part, double *spart, unsigned *t, unsigned bid,
                          unsigned nblk, double *out)
{
  __shared__ unsigned s_flag;
  for (int e = threadIdx.x; e < E; e += NT) st_sc1(&part[(size_t)bid * E + e], vals[e]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr unsigned L = 32;
  const unsigned shard = bid & 7u;
  const unsigned shard_n = nblk / 8u + ((shard < nblk % 8u) ? 1u : 0u);
  const unsigned nshards = nblk < 8u ? nblk : 8u;
  if (threadIdx.x == 0)
    s_flag = __hip_atomic_fetch_add(t + shard * L, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == shard_n - 1u;
  __syncthreads();
  if (!s_flag) return false;
  for (int e = threadIdx.x; e < E; e += NT)
  {
    double acc = 0.0;
    for (unsigned j0 = 0; j0 < shard_n; j0 += 16)
    {
      double v[16];  // 16 independent sc1 loads in flight, then the adds in bid order
#pragma unroll
      for (int u = 0; u < 16; ++u)
        v[u] = (j0 + u < shard_n) ? ld_sc1(&part[(size_t)(shard + 8u * (j0 + u)) * E + e]) : 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[u];
    }
    st_sc1(&spart[(size_t)shard * E + e], acc);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_flag = __hip_atomic_fetch_add(t + 8u * L, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nshards - 1u;
  __syncthreads();
  if (!s_flag) return false;
  for (int e = threadIdx.x; e < E; e += NT)
  {
    double v[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = (unsigned)s < nshards ? ld_sc1(&spart[(size_t)s * E + e]) : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int s = 0; s < 8; ++s) acc += v[s];
    out[e] = acc;
  }
  if (threadIdx.x == 0) ticket_reset(t);
  __syncthreads();
  return true;
}

// ---------------------------------------------------------------------------------------------
// Window Gram of an 8-column MultiVector block held in the SpMM kernels' quad layout: lanes
// 4 r .. 4 r + 3 hold one row, lane cp = lane & 3 its columns 2 cp, 2 cp + 1 (k_spmm8_march,
// k_boxc_mv8).  StandardLargest orthonormalises the block the SpMM writes (eigensolver.hh:78-84), and
// the first read pass of that MGS needs exactly s[w][c] = y_w . y_c (c >= w): summed here while the
// rows are in registers, so the MGS starts from it (k_mgs_la_gram) instead of re-reading the block.
// ---------------------------------------------------------------------------------------------
// DPP quad exchange: the value of lane (lane ^ D) of the same quad (D = 1, 2, 3)
template <int D>
__device__ __forceinline__ double quad_xor(double v)
{
  constexpr int ctrl = D == 1 ? 0xB1 : (D == 2 ? 0x4E : 0x1B);  // quad_perm [1,0,3,2] / [2,3,0,1] / [3,2,1,0]
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, ctrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), ctrl, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// g[w2][2 d + c2] += y_{2 cp + w2} y_{2 (cp ^ d) + c2} for this lane's row (every lane of the wave
// calls it: the quad exchange reads the other lanes; a row that does not exist passes zeros)
__device__ __forceinline__ void quad_gram_add(double (&g)[2][8], double y0, double y1)
{
  const double p[4][2] = {{y0, y1},
                          {quad_xor<1>(y0), quad_xor<1>(y1)},
                          {quad_xor<2>(y0), quad_xor<2>(y1)},
                          {quad_xor<3>(y0), quad_xor<3>(y1)}};
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2)
    {
      g[0][2 * d + c2] += y0 * p[d][c2];
      g[1][2 * d + c2] += y1 * p[d][c2];
    }
}

// Workgroup sums of the quad-layout Gram g and the column dots (d0, d1) of this lane's pair, into
// out[72] (LDS, visible to all threads on return): out[8 w + c] = sum y_w y_c for c >= w (0 below the
// diagonal), out[64 + j] = the dot of column j.  Lanes of one column pair are summed by xor shuffles
// over lane bits 2..5, the waves' totals in wave order: a fixed order.  scratch: NT / 64 x 72
// doubles of LDS.  Every thread calls it.
template <int NT>
__device__ __forceinline__ void quad_gram_block(double (&g)[2][8], double d0, double d1, double *scratch,
                                                double *out)
{
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, cp = lane & 3;
  double v[18];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = g[i / 8][i % 8];
  v[16] = d0;
  v[17] = d1;
#pragma unroll
  for (int m = 4; m < 64; m <<= 1)
#pragma unroll
    for (int i = 0; i < 18; ++i) v[i] += __shfl_xor(v[i], m, 64);
  __syncthreads();  // (scratch may alias storage the caller used before)
  if (lane < 4)
  {
    double *ws = scratch + wave * 72;
#pragma unroll
    for (int w2 = 0; w2 < 2; ++w2)
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2)
        {
          const int w = 2 * cp + w2, c = 2 * (cp ^ d) + c2;
          ws[w * 8 + c] = c >= w ? v[w2 * 8 + 2 * d + c2] : 0.0;
        }
    ws[64 + 2 * cp] = v[16];
    ws[64 + 2 * cp + 1] = v[17];
  }
  __syncthreads();
  if (threadIdx.x < 72)
  {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < NT / 64; ++q) t += scratch[q * 72 + threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();
}

}  // namespace eigmi
