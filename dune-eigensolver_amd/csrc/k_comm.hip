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

namespace eigmi {

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

}  // namespace eigmi
