// One-GPU rehearsal of the RCCL point-to-point pattern of the halo exchange (api.cpp halo_exchange:
// ncclGroupStart; ncclRecv...; ncclSend...; ncclGroupEnd on a non-blocking stream), with a one-rank
// communicator whose only peer is rank 0 itself: one boundary plane of the 256^3 split (65,536
// doubles = 512 KiB, the classic step) and one plane of (t, u) pairs (1 MiB, the fused step), on the
// library's own stream (eig_ctx_stream), eagerly and inside a hipGraph capture (what bench.py's N > 1
// launch does), plus a grouped allreduce in the same capture.  Any refusal is printed with RCCL's
// own message and the test fails.  SURVEY 8(e); the reference has no distribution
// (src/dune-eigensolver.cc:742-748).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "eigmi.h"

static int fails = 0;
#define HIPC(x)                                                                               \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess)                                                                     \
    {                                                                                         \
      std::printf("HIP FAIL %s: %s\n", #x, hipGetErrorString(e_));                            \
      return 1;                                                                               \
    }                                                                                         \
  } while (0)
#define NCC(x)                                                                                \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    if (r_ != ncclSuccess)                                                                    \
    {                                                                                         \
      std::printf("RCCL FAIL %s: %s (%s)\n", #x, ncclGetErrorString(r_), ncclGetLastError(comm)); \
      return 1;                                                                               \
    }                                                                                         \
  } while (0)

static void expect(bool ok, const char *what)
{
  std::printf("%s %s\n", ok ? "ok  " : "FAIL", what);
  if (!ok) ++fails;
}

// grouped self send/recv of `count` doubles src -> dst on stream s
static ncclResult_t self_exchange(ncclComm_t comm, const double *src, double *dst, size_t count, hipStream_t s)
{
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return r;
  if ((r = ncclRecv(dst, count, ncclDouble, 0, comm, s)) != ncclSuccess) return r;
  if ((r = ncclSend(src, count, ncclDouble, 0, comm, s)) != ncclSuccess) return r;
  return ncclGroupEnd();
}

int main()
{
  eig_ctx_t ctx = nullptr;
  if (eig_ctx_create(0, &ctx) != EIG_OK)
  {
    std::printf("no device: %s\n", eig_last_error(nullptr));
    return 1;
  }
  void *sp = nullptr;
  eig_ctx_stream(ctx, &sp);
  hipStream_t s = (hipStream_t)sp;
  ncclComm_t comm = nullptr;
  ncclUniqueId id;
  NCC(ncclGetUniqueId(&id));
  NCC(ncclCommInitRank(&comm, 1, id, 0));
  int version = 0;
  ncclGetVersion(&version);
  std::printf("RCCL %d, one-rank communicator on device 0, library stream %p\n", version, sp);

  for (size_t count : {size_t(65536), size_t(131072)})
  {
    const size_t bytes = count * sizeof(double);
    std::vector<double> h(count), back(count);
    for (size_t i = 0; i < count; ++i) h[i] = 0.5 * (double)i - 1e-3 * (double)(i % 97);
    double *src = nullptr, *dst = nullptr, *red = nullptr;
    HIPC(hipMalloc(&src, bytes));
    HIPC(hipMalloc(&dst, bytes));
    HIPC(hipMalloc(&red, 3 * sizeof(double)));
    HIPC(hipMemcpy(src, h.data(), bytes, hipMemcpyHostToDevice));

    // eager
    HIPC(hipMemsetAsync(dst, 0, bytes, s));
    NCC(self_exchange(comm, src, dst, count, s));
    HIPC(hipStreamSynchronize(s));
    HIPC(hipMemcpy(back.data(), dst, bytes, hipMemcpyDeviceToHost));
    char what[160];
    std::snprintf(what, sizeof what, "eager grouped self send/recv, %zu KiB", bytes >> 10);
    expect(std::memcmp(back.data(), h.data(), bytes) == 0, what);

    // captured: memset + exchange + allreduce of 3 sums, replayed twice with new source data
    const double sums[3] = {1.25, -2.5, 3.0};
    HIPC(hipMemcpy(red, sums, sizeof(sums), hipMemcpyHostToDevice));
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    HIPC(hipMemsetAsync(dst, 0, bytes, s));
    ncclResult_t rc = self_exchange(comm, src, dst, count, s);
    ncclResult_t ra = ncclAllReduce(red, red, 3, ncclDouble, ncclSum, comm, s);
    hipError_t ec = hipStreamEndCapture(s, &g);
    if (rc != ncclSuccess || ra != ncclSuccess || ec != hipSuccess)
    {
      std::printf("capture refused: send/recv %s, allreduce %s, end capture %s (%s)\n", ncclGetErrorString(rc),
                  ncclGetErrorString(ra), hipGetErrorString(ec), ncclGetLastError(comm));
      ++fails;
      continue;
    }
    HIPC(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 2; ++rep)
    {
      for (size_t i = 0; i < count; ++i) h[i] = (double)(rep + 2) * 0.25 * (double)i + (double)(i % 13);
      HIPC(hipMemcpy(src, h.data(), bytes, hipMemcpyHostToDevice));
      HIPC(hipGraphLaunch(ge, s));
      HIPC(hipStreamSynchronize(s));
      HIPC(hipMemcpy(back.data(), dst, bytes, hipMemcpyDeviceToHost));
      std::snprintf(what, sizeof what, "hipGraph replay %d: grouped self send/recv, %zu KiB", rep, bytes >> 10);
      expect(std::memcmp(back.data(), h.data(), bytes) == 0, what);
    }
    double r3[3];
    HIPC(hipMemcpy(r3, red, sizeof(r3), hipMemcpyDeviceToHost));
    expect(r3[0] == sums[0] && r3[1] == sums[1] && r3[2] == sums[2], "hipGraph replay: one-rank ncclAllReduce is the identity");
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    (void)hipFree(src);
    (void)hipFree(dst);
    (void)hipFree(red);
  }
  ncclCommDestroy(comm);
  eig_ctx_destroy(ctx);
  std::printf(fails ? "FAILED %d\n" : "ALL OK\n", fails);
  return fails ? 1 : 0;
}
