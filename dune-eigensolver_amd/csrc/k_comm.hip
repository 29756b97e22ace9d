// k_comm.hip -- the xGMI mailbox allreduce for the Lanczos scalars (gfx950).
//
// The step's two global reductions carry one double each; a ring/tree collective spends
// 2(P-1) link latencies on that.  Here every rank owns a small uncached mailbox in its own HBM,
// exported through IPC and mapped by every peer: one launch stores this rank's values straight
// into slot `me` of every peer's mailbox over xGMI (values, then a release-ordered sequence
// number), polls its own mailbox until every slot carries the current sequence number, and sums
// the slots in rank order -- so every rank computes the bitwise identical sum, and the result
// does not depend on which rank arrived first.
//
// Mailbox layout (u64 words): [parity 0..1][slot 0..P-1][1 + kMailboxVals].  Word 0 of a slot is
// the sequence number, words 1.. the values.  Calls alternate parity by sequence number: a rank
// can only reuse a parity buffer after finishing the call in between, which needs every peer's
// values of that call, which every peer writes only after finishing (= having read) the call
// before -- so two buffers are enough and nothing is ever overwritten unread.
//
// The sequence counter lives in device memory and is advanced by the kernel itself, so the
// launch can be captured in a hipGraph and replayed.  Polling is bounded (timeout in
// s_memrealtime ticks, 100 MHz): on timeout the result is NaN and *err is set, instead of a hang.
#include "internal.h"

#include <algorithm>

namespace eigmi {

constexpr unsigned long long kXchTimeoutHalo = 200000000ull;  // 2 s of s_memrealtime

__global__ __launch_bounds__(64) void k_mailbox_allreduce(double *buf, int count, Mailbox mb, unsigned long long timeout)
{
  __shared__ u64 s_seq;
  __shared__ double s_vals[kMaxMailboxRanks][kMailboxVals];
  __shared__ int s_late;
  const int t = threadIdx.x;
  if (t == 0)
  {
    s_seq = *mb.ctr + 1;
    s_late = 0;
  }
  __syncthreads();
  const u64 seq = s_seq;
  const int par = (int)(seq & 1);
  const size_t slot_words = 1 + kMailboxVals;
  if (t < mb.P)
  {
    // push: my values into slot `me` of peer t's mailbox (peer[me] is my own mailbox)
    u64 *dst = mb.peer[t] + ((size_t)par * mb.P + mb.me) * slot_words;
    for (int i = 0; i < count; ++i)
      __hip_atomic_store(dst + 1 + i, __double_as_longlong(buf[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(dst, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    // pull: wait for peer t's values of this call in my own mailbox
    const u64 *src = mb.local + ((size_t)par * mb.P + t) * slot_words;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool late = false;
    // relaxed polling (uncached memory: every load reaches HBM), one acquire fence after it
    while (__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != seq)
    {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout)
      {
        late = true;
        break;
      }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (late) s_late = 1;
    for (int i = 0; i < count; ++i)
      s_vals[t][i] = __longlong_as_double(
          (long long)__hip_atomic_load(src + 1 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  }
  __syncthreads();
  if (t < count)
  {
    double s = 0.0;
    for (int r = 0; r < mb.P; ++r) s += s_vals[r][t];  // rank order: identical on every rank
    buf[t] = s_late ? __builtin_nan("") : s;
  }
  if (t == 0)
  {
    *mb.ctr = seq;
    if (s_late) *mb.err = 1;
  }
}

void launch_mailbox_allreduce(double *buf, int count, const Mailbox &mb, unsigned long long timeout, hipStream_t s)
{
  EIG_CHECK(count >= 1 && count <= kMailboxVals, EIG_ERR_ARG, "mailbox allreduce: bad count");
  EIG_CHECK(mb.P >= 1 && mb.P <= kMaxMailboxRanks, EIG_ERR_ARG, "mailbox allreduce: bad rank count");
  hipLaunchKernelGGL(k_mailbox_allreduce, dim3(1), dim3(64), 0, s, buf, count, mb, timeout);
  EIG_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// The halo exchange of mailbox-only ranks over the same IPC mappings (HaloBox, internal.h): the
// boundary rows a peer needs are stored straight into that peer's uncached staging slot over xGMI,
// and the ghost rows are copied out of my own staging once every peer's sequence line carries the
// exchange's number.  Two launches on the exchange stream:
//   push: every workgroup streams its share of the send ranges into the peers' slots (parity
//         s & 1) and fences at system scope; the last workgroup (ticket) then stores s into slot
//         `me` of the sequence lines of EVERY peer this rank exchanges with (sends and receives);
//   pull: every workgroup's first wave polls my lines of those peers until they read s (bounded,
//         like k_mailbox_allreduce), then the workgroups copy the receive ranges out of my staging
//         into the window; the last workgroup stores s as the completed sequence number.
// Sequence numbers count the exchanges of each PAIR of ranks (seq[peer]): a matrix may connect rank A
// with B but not with C, and C must not see A's count move.  Every exchange of a matrix involves both
// ranks of each pair it connects (the peer relation, sends union receives, is symmetric), so a pair's
// two counters stay equal.  Parity reuse: rank A pushes s + 2 to B (over the slot of s) only after its
// pull of s + 1, which needs B's line of s + 1, which B stores only after its pull of s -- i.e. after
// B read slot s.  The counters live in device memory (captured exchanges replay correctly).  A timed-out pull,
// or any pull or push once the mailbox's error word is set, writes NaN instead of values -- into the
// ghosts and into the peers' slots -- so every rank's recurrence turns NaN the same way.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool halo_last_group(unsigned *ticket)
{
  __shared__ bool s_last;
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  return s_last;
}

__global__ __launch_bounds__(256) void k_halo_push(HaloBox hb, HaloXfer snd, HaloXfer sync, const double *x,
                                                   const double *x2, int w)
{
  const bool poisoned = __hip_atomic_load(hb.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  const double nan = __builtin_nan("");
  const long long g0 = (long long)blockIdx.x * blockDim.x + threadIdx.x, gs = (long long)gridDim.x * blockDim.x;
  for (int k = 0; k < snd.n; ++k)
  {
    const int par = (int)((__hip_atomic_load(hb.seq + snd.peer[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1) & 1);
    double *dst = hb.peer_stage[snd.peer[k]] + ((long long)par * hb.P + hb.me) * hb.cap;
    const long long n = snd.cnt[k] * w;
    const double *a = x + snd.off[k] * w;
    for (long long i = g0; i < n; i += gs) dst[i] = poisoned ? nan : a[i];
    if (x2)
    {
      const double *b = x2 + snd.off[k] * w;
      for (long long i = g0; i < n; i += gs) dst[n + i] = poisoned ? nan : b[i];
    }
  }
  __threadfence_system();  // my slot stores are performed before the ticket
  if (halo_last_group(hb.ticket))
  {
    const int t = threadIdx.x;
    if (t < sync.n)
    {
      const u64 seq = __hip_atomic_load(hb.seq + sync.peer[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
      __hip_atomic_store(hb.peer_flags[sync.peer[t]] + ((long long)(seq & 1) * hb.P + hb.me) * kHaloFlagStride, seq,
                         __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (t == 0) __hip_atomic_store(hb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(256) void k_halo_pull(HaloBox hb, HaloXfer rcv, HaloXfer sync, double *x, double *x2,
                                                   int w, unsigned long long timeout)
{
  __shared__ int s_late;
  const int t = threadIdx.x;
  if (t < 64)
  {
    const bool mine = t < sync.n;
    const int peer = mine ? sync.peer[t] : 0;
    const u64 seq = __hip_atomic_load(hb.seq + peer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    const u64 *line = hb.flags + ((long long)(seq & 1) * hb.P + peer) * kHaloFlagStride;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool late = false;
    for (;;)
    {
      const bool ok = !mine || __hip_atomic_load(line, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == seq;
      if (__all(ok)) break;
      if (__hip_atomic_load(hb.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
          __builtin_amdgcn_s_memrealtime() - t0 > timeout)
      {
        late = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const bool any_late = __any(late) || __hip_atomic_load(hb.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (t == 0)
    {
      s_late = any_late ? 1 : 0;
      if (late) __hip_atomic_store(hb.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // the peers' slot stores are visible after their lines
  const bool bad = s_late != 0;
  const double nan = __builtin_nan("");
  const long long g0 = (long long)blockIdx.x * blockDim.x + t, gs = (long long)gridDim.x * blockDim.x;
  for (int k = 0; k < rcv.n; ++k)
  {
    const int par = (int)((__hip_atomic_load(hb.seq + rcv.peer[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1) & 1);
    const double *src = hb.stage + ((long long)par * hb.P + rcv.peer[k]) * hb.cap;
    const long long n = rcv.cnt[k] * w;
    double *a = x + rcv.off[k] * w;
    for (long long i = g0; i < n; i += gs) a[i] = bad ? nan : src[i];
    if (x2)
    {
      double *b = x2 + rcv.off[k] * w;
      for (long long i = g0; i < n; i += gs) b[i] = bad ? nan : src[n + i];
    }
  }
  if (halo_last_group(hb.ticket + 32))
  {
    // (every workgroup has read the counters: the last one advances them)
    if (t < sync.n)
    {
      u64 *c = hb.seq + sync.peer[t];
      __hip_atomic_store(c, __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0) __hip_atomic_store(hb.ticket + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

void launch_halo_mailbox(const HaloBox &hb, const HaloXfer &snd, const HaloXfer &rcv, const HaloXfer &sync, double *x,
                         double *x2, int w, hipStream_t s)
{
  EIG_CHECK(hb.P >= 2 && hb.P <= kMaxMailboxRanks && w >= 1, EIG_ERR_ARG, "halo mailbox: bad arguments");
  const int m = x2 ? 2 : 1;
  long long most = 0;
  for (int k = 0; k < snd.n; ++k) most = std::max(most, snd.cnt[k]);
  for (int k = 0; k < rcv.n; ++k) most = std::max(most, rcv.cnt[k]);
  EIG_CHECK(most * w * m <= hb.cap, EIG_ERR_ARG, "halo mailbox: exchange larger than the staging slots");
  // about 4 doubles per thread, at most 512 pushing / 256 polling workgroups
  const long long per = std::max(1LL, most * w * m / (kStreamThreads * 4));
  const int gp = (int)std::min<long long>(512, per), gq = (int)std::min<long long>(256, per);
  hipLaunchKernelGGL(k_halo_push, dim3(gp), dim3(kStreamThreads), 0, s, hb, snd, sync, (const double *)x,
                     (const double *)x2, w);
  EIG_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_halo_pull, dim3(gq), dim3(kStreamThreads), 0, s, hb, rcv, sync, x, x2, w, kXchTimeoutHalo);
  EIG_HIP(hipGetLastError());
}

}  // namespace eigmi
