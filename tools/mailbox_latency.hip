// Intrinsic latency of the mailbox allreduce kernel on ONE device: P "ranks" are P streams of one
// process (kernels of one process run concurrently; separate processes on one GPU may be
// time-sliced, which is what tests/test_mailbox_gpu.py measures).  Each stream runs `calls`
// back-to-back allreduces; prints wall time per call.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/mailbox_latency.hip \
//         dune-eigensolver_amd/csrc/k_comm.hip -o tools/mailbox_latency && tools/mailbox_latency 2 2000
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../dune-eigensolver_amd/csrc/internal.h"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess)                                                       \
    {                                                                          \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));                \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char **argv)
{
  const int P = argc > 1 ? std::atoi(argv[1]) : 2;
  const int calls = argc > 2 ? std::atoi(argv[2]) : 2000;
  if (P < 1 || P > eigmi::kMaxMailboxRanks) return 2;
  const size_t bytes = (size_t)2 * P * (1 + eigmi::kMailboxVals) * sizeof(eigmi::u64);
  std::vector<eigmi::Mailbox> mb(P);
  std::vector<hipStream_t> st(P);
  std::vector<double *> buf(P);
  for (int r = 0; r < P; ++r)
  {
    void *p = nullptr;
    CK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
    CK(hipMemset(p, 0, bytes));
    mb[r].local = static_cast<eigmi::u64 *>(p);
    void *s = nullptr;
    CK(hipMalloc(&s, 256));
    CK(hipMemset(s, 0, 256));
    mb[r].ctr = static_cast<eigmi::u64 *>(s);
    mb[r].err = reinterpret_cast<int *>(static_cast<char *>(s) + 128);
    mb[r].P = P;
    mb[r].me = r;
    CK(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
    CK(hipMalloc(&buf[r], 64 * sizeof(double)));
    CK(hipMemset(buf[r], 0, 64 * sizeof(double)));
  }
  for (int r = 0; r < P; ++r)
    for (int q = 0; q < P; ++q) mb[r].peer[q] = mb[q].local;
  for (int pass = 0; pass < 2; ++pass)
  {
    const int n = pass == 0 ? 50 : calls;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i)
      for (int r = 0; r < P; ++r) eigmi::launch_mailbox_allreduce(buf[r], 1, mb[r], 200000000ull, st[r]);
    for (int r = 0; r < P; ++r) CK(hipStreamSynchronize(st[r]));
    auto t1 = std::chrono::steady_clock::now();
    if (pass == 1)
      std::printf("P=%d streams: %.2f us per allreduce (%d calls)\n", P,
                  std::chrono::duration<double, std::micro>(t1 - t0).count() / n, n);
  }
  int err = 0;
  CK(hipMemcpy(&err, mb[0].err, sizeof(int), hipMemcpyDeviceToHost));
  std::printf("timeouts: %d\n", err);
  return err ? 1 : 0;
}
