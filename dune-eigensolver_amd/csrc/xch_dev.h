// xch_dev.h -- the fused Lanczos step's allreduce inside the step kernel (gfx950).
//
// EIG_AR_MAILBOX_STEP: the LAST workgroup of fused launch L (the one the grid reduction's ticket
// elects, after every other workgroup has finished) stores the launch's three sums into slot `me`
// of every peer's xGMI mailbox (values, then a release-ordered sequence number), then polls its own
// mailbox until all P slots carry that sequence number and sums them in rank order (bitwise the
// same on every rank) into the launch's result -- so the step's allreduce costs one xGMI store plus
// the arrival of the slowest peer inside the kernel's tail, and no allreduce launch sits between
// two step kernels.  Only that one wave polls (the next launch reads the result from ordinary
// memory): polling in every wave of the next launch's prologue was measured 15-45 us slower per
// step, thousands of waves serialising on the same uncached mailbox lines (profiles/r05b_*).
//
// Step region of a mailbox (u64 words, after the k_comm.hip region): [parity 0..1][slot 0..P-1]
// [kXchWords]; word 0 = sequence number, words 1..3 = (t . u, t . t, u . u).  The sequence number
// lives in device memory (Mailbox::fctr): the exchanging workgroup reads s = fctr + 1, publishes into
// parity s & 1, gathers s, and stores fctr = s.  Parity reuse is safe: rank A publishes s + 2 (into
// the buffer of s) only after it gathered s + 1 from every rank, and rank B publishes s + 1 only
// after it gathered s.
//
// Bounded polling: after kXchTimeout ticks of s_memrealtime (100 MHz) -- or at once when a timeout
// is already recorded (Mailbox::err) -- the sums read NaN and err is set; a rank with err set
// publishes NaN from then on, so every peer's next exchange reads NaN too and all ranks leave the
// recurrence the same way (the host turns NaN sums into EIG_ERR_RCCL, drivers.cpp).  Nothing waits
// unboundedly, so a peer that never arrives cannot hang the GPU.
#pragma once
#include "internal.h"

namespace eigmi {

constexpr unsigned long long kXchTimeout = 200000000ull;  // 2 s of s_memrealtime

__device__ __forceinline__ u64 *xch_slot(u64 *box, const Mailbox &mb, int par, int r)
{
  return box + mb.foff + ((size_t)par * mb.P + r) * kXchWords;
}

// Every lane of the calling wave gets the rank-order sums of sequence seq (wave-uniform).
__device__ __forceinline__ void xch_gather(const Mailbox &mb, u64 seq, unsigned long long timeout, double &d,
                                           double &q, double &m)
{
  const int lane = threadIdx.x & 63;
  const bool mine = lane < mb.P;
  const u64 *src = xch_slot(mb.local, mb, (int)(seq & 1), mine ? lane : 0);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool late = false;
  for (;;)
  {
    const bool ok = !mine || __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == seq;
    if (__all(ok)) break;
    if (__hip_atomic_load(mb.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
        __builtin_amdgcn_s_memrealtime() - t0 > timeout)
    {
      late = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  double a = 0.0, b = 0.0, c = 0.0;
  if (mine)
  {
    a = __longlong_as_double((long long)__hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    b = __longlong_as_double((long long)__hip_atomic_load(src + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    c = __longlong_as_double((long long)__hip_atomic_load(src + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  }
  d = q = m = 0.0;
  for (int r = 0; r < mb.P; ++r)  // rank order: identical on every rank
  {
    d += __shfl(a, r, 64);
    q += __shfl(b, r, 64);
    m += __shfl(c, r, 64);
  }
  if (__any(late))
  {
    if (lane == 0) __hip_atomic_store(mb.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    d = q = m = __builtin_nan("");
  }
}

// The last workgroup of a launch (every thread): v = the launch's three local sums in LDS, replaced
// by the allreduced sums.  Threads 0 .. P-1 publish to the peers, wave 0 gathers, thread 0 then
// advances fctr.
__device__ __forceinline__ void xch_exchange(const Mailbox &mb, double *v)
{
  const int t = threadIdx.x;
  const u64 seq = __hip_atomic_load(mb.fctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  if (t < mb.P)
  {
    const bool poisoned = __hip_atomic_load(mb.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    u64 *dst = xch_slot(mb.peer[t], mb, (int)(seq & 1), mb.me);
    for (int i = 0; i < 3; ++i)
      __hip_atomic_store(dst + 1 + i, (u64)__double_as_longlong(poisoned ? __builtin_nan("") : v[i]),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();  // (every thread has read v and fctr)
  if (t < 64)
  {
    double d, q, m;
    xch_gather(mb, seq, kXchTimeout, d, q, m);
    if (t == 0)
    {
      v[0] = d;
      v[1] = q;
      v[2] = m;
      __hip_atomic_store(mb.fctr, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
}

}  // namespace eigmi
