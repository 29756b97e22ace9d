// api.cpp -- the C ABI of libeigmi (include/eigmi.h): contexts, device memory, matrix upload
// into the SELL-64 image, the halo plan of row-partitioned matrices, BlockVector and
// MultiVector operations.  Drivers live in drivers.cpp.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <random>
#include <thread>

#include "internal.h"

using namespace eigmi;

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev)
  {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) EIG_HIP(hipSetDevice(dev));
  }
  ~DeviceGuard()
  {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <class T>
T *dev_alloc(size_t count)
{
  void *p = nullptr;
  if (count == 0) count = 1;
  EIG_HIP(hipMalloc(&p, count * sizeof(T)));
  return static_cast<T *>(p);
}

}  // namespace

// ============================================================================================
// internal helpers shared with drivers.cpp
// ============================================================================================
namespace eigmi {

void *ctx_buffer(eig_ctx_t ctx, int slot, size_t bytes)
{
  if ((int)ctx->pool.size() <= slot) ctx->pool.resize(slot + 1, {nullptr, 0});
  auto &e = ctx->pool[slot];
  if (e.second < bytes)
  {
    if (e.first) EIG_HIP(hipFree(e.first));
    e.first = nullptr;
    e.second = 0;
    EIG_HIP(hipMalloc(&e.first, bytes));
    e.second = bytes;
  }
  return e.first;
}

void allreduce_sum(eig_ctx_t ctx, double *buf, i64 count, hipStream_t s)
{
  if (!ctx->collectives() || count <= 0) return;
  if (ctx->mbox && ctx->mbox->ready && ctx->mbox->on)
  {
    for (i64 off = 0; off < count; off += kMailboxVals)
      launch_mailbox_allreduce(buf + off, (int)std::min<i64>(kMailboxVals, count - off), ctx->mbox->dev,
                               kMailboxTimeout, s);
    return;
  }
  if (ctx->loop)
  {
    // loopback: every virtual rank publishes its values, then sums all ranks in rank order
    LoopHub &h = *ctx->loop;
    std::vector<double> mine((size_t)count);
    EIG_HIP(hipMemcpyAsync(mine.data(), buf, count * sizeof(double), hipMemcpyDeviceToHost, s));
    EIG_HIP(hipStreamSynchronize(s));
    {
      std::lock_guard<std::mutex> lk(h.m);
      h.red[ctx->rank] = mine;
    }
    h.barrier();
    std::vector<double> tot((size_t)count, 0.0);
    for (int r = 0; r < h.P; ++r)
      for (i64 i = 0; i < count; ++i) tot[i] += h.red[r][i];
    h.barrier();
    EIG_HIP(hipMemcpyAsync(buf, tot.data(), count * sizeof(double), hipMemcpyHostToDevice, s));
    EIG_HIP(hipStreamSynchronize(s));
    return;
  }
  EIG_NCCL(ncclAllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, ctx->comm, s));
  ++ctx->n_ar;
}

bool allreduce_overlaps(eig_ctx_t ctx)
{
  const bool ovl = ctx->collectives() && !ctx->loop && ((ctx->mbox && ctx->mbox->ready && ctx->mbox->on) || ctx->comm_red);
  // the reduction stream exists only where it is used (every stream takes a hardware queue)
  if (ovl && !ctx->red_stream) EIG_HIP(hipStreamCreateWithFlags(&ctx->red_stream, hipStreamNonBlocking));
  return ovl;
}

void allreduce_sum_red(eig_ctx_t ctx, double *buf, i64 count, hipStream_t s)
{
  EIG_CHECK(allreduce_overlaps(ctx), EIG_ERR_ARG, "allreduce_sum_red: no concurrent allreduce transport");
  if (ctx->mbox && ctx->mbox->ready && ctx->mbox->on)
  {
    allreduce_sum(ctx, buf, count, s);
    return;
  }
  EIG_NCCL(ncclAllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, ctx->comm_red, s));
  ++ctx->n_ar_red;
}

// ---------------------------------------------------------------------------------------------
// xGMI mailbox (k_comm.hip).  prepare: allocate my uncached mailbox + state and export it;
// open: map every peer's mailbox; validate: one allreduce of rank+1 must give P(P+1)/2 exactly.
// ---------------------------------------------------------------------------------------------
void halobox_free(eig_ctx_t ctx)
{
  HaloBoxHost *h = ctx->hbox;
  if (!h) return;
  for (void *p : h->opened) (void)hipIpcCloseMemHandle(p);
  if (h->alloc) (void)hipFree(h->alloc);
  if (h->state) (void)hipFree(h->state);
  delete h;
  ctx->hbox = nullptr;
}

void mailbox_free(eig_ctx_t ctx)
{
  halobox_free(ctx);  // its error word is the mailbox's
  MailboxHost *m = ctx->mbox;
  if (!m) return;
  for (void *p : m->opened) (void)hipIpcCloseMemHandle(p);
  if (m->local) (void)hipFree(m->local);
  if (m->state) (void)hipFree(m->state);
  delete m;
  ctx->mbox = nullptr;
}

void mailbox_prepare(eig_ctx_t ctx, int nranks, int rank, unsigned char handle[HIP_IPC_HANDLE_SIZE])
{
  EIG_CHECK(nranks >= 1 && nranks <= kMaxMailboxRanks && rank >= 0 && rank < nranks, EIG_ERR_ARG,
            "mailbox: rank count outside 1..16");
  mailbox_free(ctx);
  auto *m = new MailboxHost();
  ctx->mbox = m;
  // k_comm.hip region [2][P][1 + kMailboxVals], then the fused step's region [2][P][kXchWords]
  const size_t foff = (size_t)2 * nranks * (1 + kMailboxVals);
  const size_t bytes = (foff + (size_t)2 * nranks * kXchWords) * sizeof(u64);
  // uncached: a peer's stores over xGMI land in HBM and my polling loads must see them while
  // the kernel runs; fine-grained is the fallback where uncached memory cannot be exported
  void *p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess)
  {
    (void)hipGetLastError();
    EIG_HIP(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained));
  }
  m->local = static_cast<u64 *>(p);
  m->bytes = bytes;
  EIG_HIP(hipMemset(m->local, 0, bytes));
  EIG_HIP(hipMalloc(&m->state, 256));
  EIG_HIP(hipMemset(m->state, 0, 256));
  m->dev.local = m->local;
  m->dev.ctr = static_cast<u64 *>(m->state);
  m->dev.fctr = reinterpret_cast<u64 *>(static_cast<char *>(m->state) + 64);
  m->dev.err = reinterpret_cast<int *>(static_cast<char *>(m->state) + 128);
  m->dev.foff = (long long)foff;
  m->dev.P = nranks;
  m->dev.me = rank;
  hipIpcMemHandle_t h;
  EIG_HIP(hipIpcGetMemHandle(&h, m->local));
  std::memcpy(handle, &h, HIP_IPC_HANDLE_SIZE);
}

void mailbox_open(eig_ctx_t ctx, const unsigned char *handles)
{
  MailboxHost *m = ctx->mbox;
  EIG_CHECK(m && m->local, EIG_ERR_ARG, "mailbox: open before prepare");
  for (int r = 0; r < m->dev.P; ++r)
  {
    if (r == m->dev.me)
    {
      m->dev.peer[r] = m->local;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles + (size_t)r * HIP_IPC_HANDLE_SIZE, HIP_IPC_HANDLE_SIZE);
    void *p = nullptr;
    EIG_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    m->opened.push_back(p);
    m->dev.peer[r] = static_cast<u64 *>(p);
  }
}

bool mailbox_validate(eig_ctx_t ctx)
{
  MailboxHost *m = ctx->mbox;
  double *d = ctx->scratch;
  const int P = m->dev.P;
  double v[3] = {(double)(m->dev.me + 1), 1.0, (double)(m->dev.me + 1) * 0.5};
  EIG_HIP(hipMemcpy(d, v, sizeof(v), hipMemcpyHostToDevice));
  launch_mailbox_allreduce(d, 3, m->dev, 200000000ull /* 2 s */, ctx->stream);
  EIG_HIP(hipStreamSynchronize(ctx->stream));
  int err = 1;
  EIG_HIP(hipMemcpy(v, d, sizeof(v), hipMemcpyDeviceToHost));
  EIG_HIP(hipMemcpy(&err, m->dev.err, sizeof(int), hipMemcpyDeviceToHost));
  const double want = 0.5 * P * (P + 1);
  return err == 0 && v[0] == want && v[1] == (double)P && v[2] == 0.5 * want;
}

// Sum `vals` (count doubles) over the mailbox-only ranks, synchronously on ctx->stream; throws when
// the mailbox timed out.  Also a barrier: no rank returns before every rank has published.
static void mailbox_sum_sync(eig_ctx_t ctx, std::vector<double> &vals, const char *what)
{
  double *d = dev_alloc<double>(vals.size());
  EIG_HIP(hipMemcpy(d, vals.data(), vals.size() * sizeof(double), hipMemcpyHostToDevice));
  for (i64 off = 0; off < (i64)vals.size(); off += kMailboxVals)
    launch_mailbox_allreduce(d + off, (int)std::min<i64>(kMailboxVals, (i64)vals.size() - off), ctx->mbox->dev,
                             kMailboxTimeout, ctx->stream);
  EIG_HIP(hipStreamSynchronize(ctx->stream));
  EIG_HIP(hipMemcpy(vals.data(), d, vals.size() * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(d);
  int err = 0;
  EIG_HIP(hipMemcpy(&err, ctx->mbox->dev.err, sizeof(int), hipMemcpyDeviceToHost));
  EIG_CHECK(err == 0, EIG_ERR_RCCL, std::string(what) + ": mailbox timed out");
}

// (Re)build the halo mailbox with slots of `cap` doubles.  Collective over the mailbox-only ranks,
// which all call it with the same cap (eig_mat_create_bcsr_dist computes it from every rank's plan):
// the old staging is released once every rank is quiet, the new one exported and its IPC handle
// gathered through the mailbox allreduce (each 16-bit chunk one exact double).
void halobox_setup(eig_ctx_t ctx, i64 cap)
{
  MailboxHost *m = ctx->mbox;
  const int P = m->dev.P, me = m->dev.me;
  constexpr int kChunks = HIP_IPC_HANDLE_SIZE / 2;
  EIG_HIP(hipStreamSynchronize(ctx->stream));
  EIG_HIP(hipStreamSynchronize(ctx->comm_stream));
  std::vector<double> bar(1, 0.0);
  mailbox_sum_sync(ctx, bar, "halo mailbox");  // every rank's exchanges have completed
  halobox_free(ctx);
  auto *h = new HaloBoxHost();
  ctx->hbox = h;
  const size_t fbytes = (size_t)2 * P * kHaloFlagStride * sizeof(u64);
  const size_t bytes = fbytes + (size_t)2 * P * (size_t)cap * sizeof(double);
  std::vector<double> g((size_t)P * (kChunks + 1), 0.0);
  bool ok = true;
  try
  {
    void *p = nullptr;
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess)
    {
      (void)hipGetLastError();
      EIG_HIP(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained));
    }
    h->alloc = p;
    EIG_HIP(hipMemset(p, 0, bytes));
    EIG_HIP(hipMalloc(&h->state, 512));  // seq[16] at 0, the push / pull tickets at 128 / 256
    EIG_HIP(hipMemset(h->state, 0, 512));
    hipIpcMemHandle_t ih;
    EIG_HIP(hipIpcGetMemHandle(&ih, p));
    unsigned char raw[HIP_IPC_HANDLE_SIZE];
    std::memcpy(raw, &ih, HIP_IPC_HANDLE_SIZE);
    for (int c = 0; c < kChunks; ++c) g[(size_t)me * (kChunks + 1) + c] = raw[2 * c] + 256.0 * raw[2 * c + 1];
    g[(size_t)me * (kChunks + 1) + kChunks] = 1.0;
  }
  catch (const Error &)
  {
    ok = false;
  }
  mailbox_sum_sync(ctx, g, "halo mailbox");
  for (int r = 0; r < P; ++r) ok = ok && g[(size_t)r * (kChunks + 1) + kChunks] == 1.0;
  HaloBox &d = h->dev;
  if (ok)
  {
    d.flags = static_cast<u64 *>(h->alloc);
    d.stage = reinterpret_cast<double *>(static_cast<char *>(h->alloc) + fbytes);
    d.seq = static_cast<u64 *>(h->state);
    d.ticket = reinterpret_cast<unsigned *>(static_cast<char *>(h->state) + 128);
    d.err = m->dev.err;
    d.cap = cap;
    d.P = P;
    d.me = me;
    try
    {
      for (int r = 0; r < P; ++r)
      {
        char *base = static_cast<char *>(h->alloc);
        if (r != me)
        {
          unsigned char raw[HIP_IPC_HANDLE_SIZE];
          for (int c = 0; c < kChunks; ++c)
          {
            const unsigned v = (unsigned)g[(size_t)r * (kChunks + 1) + c];
            raw[2 * c] = (unsigned char)(v & 255u);
            raw[2 * c + 1] = (unsigned char)(v >> 8);
          }
          hipIpcMemHandle_t ih;
          std::memcpy(&ih, raw, HIP_IPC_HANDLE_SIZE);
          void *p = nullptr;
          EIG_HIP(hipIpcOpenMemHandle(&p, ih, hipIpcMemLazyEnablePeerAccess));
          h->opened.push_back(p);
          base = static_cast<char *>(p);
        }
        d.peer_flags[r] = reinterpret_cast<u64 *>(base);
        d.peer_stage[r] = reinterpret_cast<double *>(base + fbytes);
      }
    }
    catch (const Error &)
    {
      ok = false;
    }
  }
  std::vector<double> agree(1, ok ? 1.0 : 0.0);
  mailbox_sum_sync(ctx, agree, "halo mailbox");
  if (agree[0] != (double)P)
  {
    halobox_free(ctx);
    throw Error(EIG_ERR_RCCL, "halo mailbox: staging setup failed on some rank");
  }
}

// Exchange the ghost entries of the window-layout vector x.  Runs on stream s.
void halo_exchange(const eig_mat_s &A, double *x, hipStream_t s, double *x2, int width)
{
  eig_ctx_t ctx = A.ctx;
  if (!ctx->distributed()) return;
  const i64 w = width;
  if (ctx->loop)
  {
    // loopback: publish (x, window begin), then pull every recv range from the owner's vector
    LoopHub &h = *ctx->loop;
    EIG_HIP(hipStreamSynchronize(s));
    {
      std::lock_guard<std::mutex> lk(h.m);
      h.xptr[ctx->rank] = x;
      h.win_begin[ctx->rank] = A.win_begin;
    }
    h.barrier();
    for (const auto &r : A.recvs)
    {
      const i64 global = A.win_begin + r.offset;
      const double *src = h.xptr[r.peer] + (global - h.win_begin[r.peer]) * w;
      EIG_HIP(hipMemcpyAsync(x + r.offset * w, src, r.count * w * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
    EIG_HIP(hipStreamSynchronize(s));
    h.barrier();
    if (x2) halo_exchange(A, x2, s, nullptr, width);
    return;
  }
  if ((!ctx->comm || ctx->halo_mailbox) && ctx->mbox && ctx->mbox->ready)
  {
    // mailbox-only ranks, or EIG_HALO_MAILBOX: the xGMI halo mailbox (k_comm.hip).  Every rank of the partition takes part
    // in every exchange of the matrix (an empty side still publishes and waits for its lines).
    HaloXfer snd, rcv, syn;
    auto add_sync = [&](int peer) {
      for (int k = 0; k < syn.n; ++k)
        if (syn.peer[k] == peer) return;
      syn.peer[syn.n++] = peer;
    };
    for (const auto &r : A.sends)
    {
      snd.peer[snd.n] = r.peer;
      snd.off[snd.n] = r.offset;
      snd.cnt[snd.n++] = r.count;
      add_sync(r.peer);
    }
    for (const auto &r : A.recvs)
    {
      rcv.peer[rcv.n] = r.peer;
      rcv.off[rcv.n] = r.offset;
      rcv.cnt[rcv.n++] = r.count;
      add_sync(r.peer);
    }
    if (syn.n == 0) return;
    EIG_CHECK(ctx->hbox, EIG_ERR_ARG, "halo exchange: no halo mailbox (matrix created before the mailbox was reopened)");
    launch_halo_mailbox(ctx->hbox->dev, snd, rcv, syn, x, x2, width, s);
    ++ctx->n_halo;
    ctx->n_p2p += (long long)(A.recvs.size() + A.sends.size()) * (x2 ? 2 : 1);
    return;
  }
  if (A.sends.empty() && A.recvs.empty()) return;
  EIG_CHECK(ctx->comm, EIG_ERR_ARG, "halo exchange needs RCCL, the mailbox or the loopback transport");
  EIG_NCCL(ncclGroupStart());
  // per peer, x then x2 on both sides: point-to-point operations match in issue order
  for (const auto &r : A.recvs)
  {
    EIG_NCCL(ncclRecv(x + r.offset * w, (size_t)(r.count * w), ncclDouble, r.peer, ctx->comm, s));
    if (x2) EIG_NCCL(ncclRecv(x2 + r.offset * w, (size_t)(r.count * w), ncclDouble, r.peer, ctx->comm, s));
  }
  for (const auto &r : A.sends)
  {
    EIG_NCCL(ncclSend(x + r.offset * w, (size_t)(r.count * w), ncclDouble, r.peer, ctx->comm, s));
    if (x2) EIG_NCCL(ncclSend(x2 + r.offset * w, (size_t)(r.count * w), ncclDouble, r.peer, ctx->comm, s));
  }
  EIG_NCCL(ncclGroupEnd());
  ++ctx->n_halo;
  ctx->n_p2p += (long long)(A.recvs.size() + A.sends.size()) * (x2 ? 2 : 1);
}

// eigensolver.hh:49-55 generator (libstdc++ mt19937 + normal_distribution, bitwise the
// reference's sequence).
// The reference's start vectors: std::normal_distribution<double>{0, 1} over std::mt19937{seed}
// (eigensolver.hh:50-55), bitwise.  libstdc++ draws them by Marsaglia's polar method on pairs of
// generate_canonical<double, 53> uniforms (random.tcc: two 32-bit words per uniform, the second
// variate of an accepted pair kept for the next call); its generic generate_canonical recomputes
// long-double logarithms on every call, about two thirds of the 45 ns per variate it costs.  The
// same arithmetic with the constants folded (the words are exact in double, the scales powers of
// two) gives the same bits (tests/test_random_host.py against the oracle's std:: draws).
void host_random_normal(i64 count, unsigned seed, double *out)
{
  std::mt19937 urbg{seed};
  auto canonical = [&]() {
    double sum = 0.0;
    sum += double(urbg()) * 1.0;           // mt19937: min() = 0, range 2^32
    sum += double(urbg()) * 4294967296.0;  // x 2^32
    double r = sum / 18446744073709551616.0;  // / 2^64
    if (r >= 1.0) r = std::nextafter(1.0, 0.0);
    return r;
  };
  i64 i = 0;
  while (i < count)
  {
    double x, y, r2;
    do
    {
      x = 2.0 * canonical() - 1.0;
      y = 2.0 * canonical() - 1.0;
      r2 = x * x + y * y;
    } while (r2 > 1.0 || r2 == 0.0);
    const double mult = std::sqrt(-2 * std::log(r2) / r2);
    const double a = y * mult, b = x * mult;  // returned now / cached for the next call
    out[i++] = a * 1.0 + 0.0;                 // (ret * stddev + mean)
    if (i < count) out[i++] = b * 1.0 + 0.0;
  }
}

}  // namespace eigmi

// ============================================================================================
// context
// ============================================================================================
extern "C" int eig_random_normal(int64_t count, unsigned seed, double *out)
{
  return guard(nullptr, [&] {
    EIG_CHECK(count >= 0 && (out || count == 0), EIG_ERR_ARG, "eig_random_normal: bad argument");
    host_random_normal(count, seed, out);
  });
}

extern "C" int eig_device_count(int *count)
{
  return guard(nullptr, [&] {
    EIG_CHECK(count, EIG_ERR_ARG, "eig_device_count: null");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *count = (e == hipSuccess) ? c : 0;
  });
}

extern "C" const char *eig_version(void) { return "eigmi 0.2 gfx950 (band-image plane march SpMV / Lanczos / SpMM, SELL-64, MFMA f64 Gram, RCCL halo)"; }

extern "C" int eig_ctx_create(int device, eig_ctx_t *out)
{
  return guard(nullptr, [&] {
    EIG_CHECK(out, EIG_ERR_ARG, "eig_ctx_create: null output");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || c == 0) throw Error(EIG_ERR_NODEVICE, "no HIP device visible");
    EIG_CHECK(device >= 0 && device < c, EIG_ERR_ARG, "eig_ctx_create: bad device index");
    EIG_HIP(hipSetDevice(device));
    auto *ctx = new eig_ctx_s();
    ctx->device = device;
    try
    {
      EIG_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
      EIG_HIP(hipStreamCreateWithFlags(&ctx->comm_stream, hipStreamNonBlocking));
      hipDeviceProp_t prop;
      EIG_HIP(hipGetDeviceProperties(&prop, device));
      ctx->num_cu = prop.multiProcessorCount;
      ctx->red.partials = dev_alloc<double>((size_t)kMaxRedBlocks * kMaxRedVals);
      ctx->red.tickets = dev_alloc<unsigned>((size_t)kNumTickets * kTicketStride);
      EIG_HIP(hipMemset(ctx->red.tickets, 0, (size_t)kNumTickets * kTicketStride * sizeof(unsigned)));
      ctx->scratch = dev_alloc<double>(4096);
      EIG_HIP(hipMemset(ctx->scratch, 0, 4096 * sizeof(double)));
    }
    catch (...)
    {
      eig_ctx_destroy(ctx);
      throw;
    }
    *out = ctx;
  });
}

extern "C" int eig_ctx_destroy(eig_ctx_t ctx)
{
  if (!ctx) return EIG_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  mailbox_free(ctx);
  if (ctx->mgs_err_host) (void)hipHostFree(ctx->mgs_err_host);
  if (ctx->comm_red) (void)ncclCommDestroy(ctx->comm_red);
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  ctx->loop = nullptr;  // the hub is owned by eig_loopback_create / _destroy
  for (auto &e : ctx->pool)
    if (e.first) (void)hipFree(e.first);
  if (ctx->red.partials) (void)hipFree(ctx->red.partials);
  if (ctx->red.tickets) (void)hipFree(ctx->red.tickets);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->comm_stream) (void)hipStreamDestroy(ctx->comm_stream);
  if (ctx->red_stream) (void)hipStreamDestroy(ctx->red_stream);
  delete ctx;
  return EIG_OK;
}

namespace eigmi {
std::string &tls_error()
{
  thread_local std::string e;
  return e;
}
}  // namespace eigmi

extern "C" const char *eig_last_error(eig_ctx_t ctx) { return ctx ? ctx->last_error.c_str() : tls_error().c_str(); }

extern "C" int eig_ctx_sync(eig_ctx_t ctx)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx, EIG_ERR_ARG, "null context");
    EIG_HIP(hipStreamSynchronize(ctx->stream));
    mgs_lookahead_check(ctx);  // (eig_orthonormalize_mv8 is asynchronous: its barrier error surfaces here)
  });
}

extern "C" int eig_ctx_stream(eig_ctx_t ctx, void **stream)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && stream, EIG_ERR_ARG, "null argument");
    *stream = (void *)ctx->stream;
  });
}

// ============================================================================================
// communicator
// ============================================================================================
extern "C" int eig_comm_unique_id(unsigned char id[128])
{
  return guard(nullptr, [&] {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    EIG_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, 128);
  });
}

namespace {

// RCCL-agreed minimum of a per-rank flag (every rank takes the same branch afterwards).
bool all_ranks(eig_ctx_t ctx, bool mine)
{
  int *d = dev_alloc<int>(1);
  const int v = mine ? 1 : 0;
  EIG_HIP(hipMemcpy(d, &v, sizeof(int), hipMemcpyHostToDevice));
  EIG_NCCL(ncclAllReduce(d, d, 1, ncclInt32, ncclMin, ctx->comm, ctx->stream));
  EIG_HIP(hipStreamSynchronize(ctx->stream));
  int r = 0;
  EIG_HIP(hipMemcpy(&r, d, sizeof(int), hipMemcpyDeviceToHost));
  (void)hipFree(d);
  return r == 1;
}

// Mailbox allreduce next to the RCCL communicator; each stage is agreed by all ranks, so a rank
// whose export, mapping or validation fails makes every rank stay on ncclAllReduce.
void mailbox_setup_rccl(eig_ctx_t ctx)
{
  const int P = ctx->nranks, me = ctx->rank;
  // (one rank with EIG_COMM_ALWAYS: the one-GPU rehearsal of the mailbox transports)
  const bool want = (P > 1 || ctx->comm_always) && P <= kMaxMailboxRanks;
  if (!all_ranks(ctx, want)) return;
  std::vector<unsigned char> h((size_t)P * HIP_IPC_HANDLE_SIZE, 0);
  bool ok = true;
  try
  {
    mailbox_prepare(ctx, P, me, h.data() + (size_t)me * HIP_IPC_HANDLE_SIZE);
  }
  catch (const Error &)
  {
    ok = false;
  }
  if (!all_ranks(ctx, ok)) return mailbox_free(ctx);
  unsigned char *d = dev_alloc<unsigned char>(h.size());
  EIG_HIP(hipMemcpy(d + (size_t)me * HIP_IPC_HANDLE_SIZE, h.data() + (size_t)me * HIP_IPC_HANDLE_SIZE,
                    HIP_IPC_HANDLE_SIZE, hipMemcpyHostToDevice));
  EIG_NCCL(ncclAllGather(d + (size_t)me * HIP_IPC_HANDLE_SIZE, d, HIP_IPC_HANDLE_SIZE, ncclChar, ctx->comm,
                         ctx->stream));
  EIG_HIP(hipStreamSynchronize(ctx->stream));
  EIG_HIP(hipMemcpy(h.data(), d, h.size(), hipMemcpyDeviceToHost));
  (void)hipFree(d);
  try
  {
    mailbox_open(ctx, h.data());
  }
  catch (const Error &)
  {
    ok = false;
  }
  if (!all_ranks(ctx, ok)) return mailbox_free(ctx);
  ok = mailbox_validate(ctx);
  if (!all_ranks(ctx, ok)) return mailbox_free(ctx);
  ctx->mbox->ready = true;
}

}  // namespace

extern "C" int eig_comm_init(eig_ctx_t ctx, int nranks, int rank, const unsigned char id[128])
{
  return eig_comm_init_ex(ctx, nranks, rank, id, 0);
}

extern "C" int eig_comm_init_ex(eig_ctx_t ctx, int nranks, int rank, const unsigned char id[128], int flags)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && id && nranks >= 1 && rank >= 0 && rank < nranks, EIG_ERR_ARG, "eig_comm_init: bad arguments");
    EIG_CHECK((flags & ~(EIG_COMM_MAILBOX | EIG_COMM_ALWAYS)) == 0, EIG_ERR_ARG, "eig_comm_init_ex: unknown flag");
    EIG_CHECK(!ctx->loop && !ctx->mbox, EIG_ERR_ARG, "context already has a transport");
    DeviceGuard dg(ctx->device);
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    EIG_NCCL(ncclCommInitRank(&ctx->comm, nranks, u, rank));
    ctx->nranks = nranks;
    ctx->rank = rank;
    ctx->comm_always = (flags & EIG_COMM_ALWAYS) != 0;
    // second communicator (same ranks, same order) for allreduces that overlap the halo exchange.
    // A rank whose split fails makes every rank drop it (all_ranks), so all ranks agree on
    // allreduce_overlaps() and run the pipelined step's allreduce on the same communicator.
    if (nranks > 1 || ctx->comm_always)
    {
      if (ncclCommSplit(ctx->comm, 0, rank, &ctx->comm_red, nullptr) != ncclSuccess) ctx->comm_red = nullptr;
      if (!all_ranks(ctx, ctx->comm_red != nullptr) && ctx->comm_red)
      {
        (void)ncclCommDestroy(ctx->comm_red);
        ctx->comm_red = nullptr;
      }
    }
    // the mailbox allreduce only on request: set up, validated and agreed by all ranks (else RCCL)
    if (flags & EIG_COMM_MAILBOX) mailbox_setup_rccl(ctx);
  });
}

extern "C" int eig_comm_ipc_handle(eig_ctx_t ctx, int nranks, int rank, unsigned char handle[EIG_IPC_HANDLE_BYTES])
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && handle, EIG_ERR_ARG, "eig_comm_ipc_handle: bad arguments");
    EIG_CHECK(!ctx->comm && !ctx->loop, EIG_ERR_ARG, "context already has a transport");
    DeviceGuard dg(ctx->device);
    mailbox_prepare(ctx, nranks, rank, handle);
  });
}

extern "C" int eig_comm_ipc_open(eig_ctx_t ctx, const unsigned char *handles)
{
  return eig_comm_ipc_open_ex(ctx, handles, 0);
}

extern "C" int eig_comm_ipc_open_ex(eig_ctx_t ctx, const unsigned char *handles, int flags)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && handles && ctx->mbox && !ctx->mbox->ready, EIG_ERR_ARG,
              "eig_comm_ipc_open: call eig_comm_ipc_handle first");
    EIG_CHECK((flags & ~EIG_COMM_ALWAYS) == 0, EIG_ERR_ARG, "eig_comm_ipc_open_ex: unknown flag");
    DeviceGuard dg(ctx->device);
    mailbox_open(ctx, handles);
    ctx->nranks = ctx->mbox->dev.P;
    ctx->rank = ctx->mbox->dev.me;
    ctx->mbox->ready = true;
    ctx->comm_always = (flags & EIG_COMM_ALWAYS) != 0;
  });
}

extern "C" int eig_comm_select_allreduce(eig_ctx_t ctx, int kind)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && (kind == EIG_AR_RCCL || kind == EIG_AR_MAILBOX || kind == EIG_AR_MAILBOX_STEP), EIG_ERR_ARG,
              "eig_comm_select_allreduce: EIG_AR_RCCL, EIG_AR_MAILBOX or EIG_AR_MAILBOX_STEP");
    EIG_CHECK(kind == EIG_AR_RCCL ? ctx->comm != nullptr : (ctx->mbox && ctx->mbox->ready), EIG_ERR_ARG,
              "eig_comm_select_allreduce: that transport is not set up on this context");
    if (ctx->mbox)
    {
      DeviceGuard dg(ctx->device);
      MailboxHost *m = ctx->mbox;
      EIG_HIP(hipStreamSynchronize(ctx->stream));
      if (ctx->comm || ctx->loop)
      {
        // a new selection restarts the mailbox on every rank: after a timed-out call the
        // ranks' sequence words disagree (a lagging rank could match a peer's OLD publication), so
        // with the ranks quiet (barrier over RCCL / the loopback hub), each zeroes its mailbox, its
        // call counters and its error word, and a second barrier keeps any rank from publishing
        // into a mailbox that is not yet zeroed
        m->on = false;
        auto barrier = [&] {
          double *d = ctx->scratch + 4000;
          EIG_HIP(hipMemsetAsync(d, 0, sizeof(double), ctx->stream));
          allreduce_sum(ctx, d, 1, ctx->stream);
          EIG_HIP(hipStreamSynchronize(ctx->stream));
        };
        barrier();
        EIG_HIP(hipMemsetAsync(m->local, 0, m->bytes, ctx->stream));
        EIG_HIP(hipMemsetAsync(m->state, 0, 256, ctx->stream));
        EIG_HIP(hipStreamSynchronize(ctx->stream));
        barrier();
      }
      else
      {
        // mailbox alone (eig_comm_ipc_open, no other transport to agree on a restart): only the
        // error word is cleared; after a timeout re-open the mailbox (eig_comm_ipc_handle / _open)
        EIG_HIP(hipMemset(m->dev.err, 0, sizeof(int)));
      }
      m->on = kind != EIG_AR_RCCL;
      m->step = kind == EIG_AR_MAILBOX_STEP;
    }
  });
}

extern "C" int eig_comm_select_halo(eig_ctx_t ctx, int kind)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && (kind == EIG_HALO_RCCL || kind == EIG_HALO_MAILBOX), EIG_ERR_ARG,
              "eig_comm_select_halo: EIG_HALO_RCCL or EIG_HALO_MAILBOX");
    EIG_CHECK(ctx->comm && ctx->mbox && ctx->mbox->ready, EIG_ERR_ARG,
              "eig_comm_select_halo: needs RCCL and a validated mailbox (eig_comm_init_ex EIG_COMM_MAILBOX)");
    EIG_CHECK(kind == EIG_HALO_RCCL || ctx->hbox || ctx->nranks == 1, EIG_ERR_RCCL,
              "eig_comm_select_halo: no halo mailbox staging (set up by eig_mat_create_bcsr_dist; it failed or no "
              "distributed matrix with a halo exists yet)");
    DeviceGuard dg(ctx->device);
    EIG_HIP(hipStreamSynchronize(ctx->stream));
    EIG_HIP(hipStreamSynchronize(ctx->comm_stream));
    ctx->halo_mailbox = kind == EIG_HALO_MAILBOX;
  });
}

extern "C" int eig_comm_info(eig_ctx_t ctx, int *nranks, int *rank, int *allreduce, int *mailbox_errors)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx, EIG_ERR_ARG, "null context");
    if (nranks) *nranks = ctx->nranks;
    if (rank) *rank = ctx->rank;
    if (allreduce)
      *allreduce = !ctx->collectives()                 ? EIG_AR_NONE
                   : ctx->step_exchange()              ? EIG_AR_MAILBOX_STEP
                   : (ctx->mbox && ctx->mbox->ready && ctx->mbox->on) ? EIG_AR_MAILBOX
                   : ctx->loop                         ? EIG_AR_LOOPBACK
                                                       : EIG_AR_RCCL;
    if (mailbox_errors)
    {
      *mailbox_errors = 0;
      if (ctx->mbox && ctx->mbox->ready)
      {
        DeviceGuard dg(ctx->device);
        EIG_HIP(hipStreamSynchronize(ctx->stream));
        EIG_HIP(hipMemcpy(mailbox_errors, ctx->mbox->dev.err, sizeof(int), hipMemcpyDeviceToHost));
      }
    }
  });
}

extern "C" int eig_fill_normal(eig_ctx_t ctx, int64_t count, unsigned seed, double *x)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && x && count >= 0, EIG_ERR_ARG, "eig_fill_normal: bad argument");
    DeviceGuard dg(ctx->device);
    if (count > 0) launch_fill_normal(count, seed, x, ctx->stream);
  });
}

extern "C" int eig_mat_tune(eig_mat_t A, int key, int value)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && value >= 0, EIG_ERR_ARG, "eig_mat_tune: bad argument");
    EIG_CHECK(key == EIG_TUNE_MARCH_RUNS || key == EIG_TUNE_BOX_SEGS || key == EIG_TUNE_MARCH_PREFETCH ||
                  key == EIG_TUNE_HALO || key == EIG_TUNE_CACHE || key == EIG_TUNE_BOX_COLS ||
                  key == EIG_TUNE_BOX_MAP || key == EIG_TUNE_SELL_CPF || key == EIG_TUNE_MARCH_LINES,
              EIG_ERR_ARG, "eig_mat_tune: unknown key");
    EIG_CHECK(key != EIG_TUNE_HALO || value <= 1, EIG_ERR_ARG, "eig_mat_tune: halo mode 0 / 1");
    EIG_CHECK(key != EIG_TUNE_MARCH_PREFETCH || value <= 18, EIG_ERR_ARG, "eig_mat_tune: march variant 0..18");
    if (key == EIG_TUNE_MARCH_RUNS)
      A->tune_march_runs = value;
    else if (key == EIG_TUNE_MARCH_PREFETCH)
      A->tune_march_prefetch = value;
    else if (key == EIG_TUNE_HALO)
      A->tune_halo_whole = value;
    else if (key == EIG_TUNE_CACHE)
      A->tune_cache = value;
    else if (key == EIG_TUNE_MARCH_LINES)
    {
      EIG_CHECK(value == 0 || value == 4, EIG_ERR_ARG, "eig_mat_tune: march lines 0 / 4");
      A->tune_march_lines = value;
    }
    else if (key == EIG_TUNE_SELL_CPF)
    {
      EIG_CHECK(value <= 2, EIG_ERR_ARG, "eig_mat_tune: column prefetch 0 / 1 / 2");
      A->tune_sell_cpf = value;
    }
    else if (key == EIG_TUNE_BOX_MAP)
    {
      EIG_CHECK(value <= 1, EIG_ERR_ARG, "eig_mat_tune: box map 0 / 1");
      A->tune_box_map = value;
    }
    else if (key == EIG_TUNE_BOX_COLS)
    {
      EIG_CHECK(value == 0 || value == 16 || value == 32, EIG_ERR_ARG, "eig_mat_tune: box columns 0 / 16 / 32");
      A->tune_box_cols = value;
    }
    else
      A->tune_box_segs = value;
  });
}

extern "C" int eig_comm_counters(eig_ctx_t ctx, int64_t out[4])
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && out, EIG_ERR_ARG, "eig_comm_counters: null argument");
    out[0] = ctx->n_ar;
    out[1] = ctx->n_ar_red;
    out[2] = ctx->n_halo;
    out[3] = ctx->n_p2p;
  });
}

extern "C" int eig_loopback_create(int nranks, void **hub)
{
  return guard(nullptr, [&] {
    EIG_CHECK(hub && nranks >= 1, EIG_ERR_ARG, "eig_loopback_create: bad arguments");
    auto *h = new LoopHub();
    h->P = nranks;
    h->xptr.assign(nranks, nullptr);
    h->win_begin.assign(nranks, 0);
    h->red.assign(nranks, {});
    h->gather.assign(4 * (size_t)nranks, 0);
    h->mbox.assign(nranks, nullptr);
    h->flag.assign(nranks, 0);
    *hub = h;
  });
}

extern "C" int eig_loopback_destroy(void *hub)
{
  delete static_cast<LoopHub *>(hub);
  return EIG_OK;
}

extern "C" int eig_comm_init_loopback(eig_ctx_t ctx, void *hub, int rank)
{
  return guard(ctx, [&] {
    auto *h = static_cast<LoopHub *>(hub);
    EIG_CHECK(ctx && h && rank >= 0 && rank < h->P, EIG_ERR_ARG, "eig_comm_init_loopback: bad arguments");
    EIG_CHECK(!ctx->comm && !ctx->mbox, EIG_ERR_ARG, "context already has a transport");
    ctx->loop = h;
    ctx->nranks = h->P;
    ctx->rank = rank;
  });
}

extern "C" int eig_comm_loopback_mailbox(eig_ctx_t ctx)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && ctx->loop && !ctx->mbox, EIG_ERR_ARG, "eig_comm_loopback_mailbox: loopback rank without a mailbox");
    DeviceGuard dg(ctx->device);
    LoopHub &h = *ctx->loop;
    const int P = h.P, me = ctx->rank;
    unsigned char handle[HIP_IPC_HANDLE_SIZE];
    bool ok = true;
    try
    {
      mailbox_prepare(ctx, P, me, handle);
    }
    catch (const Error &)
    {
      ok = false;
    }
    {
      std::lock_guard<std::mutex> lk(h.m);
      h.mbox[me] = ok ? ctx->mbox->local : nullptr;
      h.flag[me] = ok ? 1 : 0;
    }
    h.barrier();
    for (int r = 0; r < P; ++r) ok = ok && h.flag[r] && h.mbox[r];
    // the virtual ranks share one process and device: the peers' mailboxes are plain device pointers
    if (ok)
      for (int r = 0; r < P; ++r) ctx->mbox->dev.peer[r] = h.mbox[r];
    h.barrier();
    if (ok) ok = mailbox_validate(ctx);  // (every rank's kernel runs concurrently: one queue each)
    {
      std::lock_guard<std::mutex> lk(h.m);
      h.flag[me] = ok ? 1 : 0;
    }
    h.barrier();
    for (int r = 0; r < P; ++r) ok = ok && h.flag[r];
    h.barrier();
    if (!ok)
    {
      mailbox_free(ctx);
      throw Error(EIG_ERR_RCCL, "eig_comm_loopback_mailbox: mailbox setup or validation failed on some rank");
    }
    ctx->mbox->ready = true;
  });
}

extern "C" int eig_comm_allreduce_sum(eig_ctx_t ctx, double *buf, int64_t count)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && buf && count >= 0, EIG_ERR_ARG, "eig_comm_allreduce_sum: bad arguments");
    allreduce_sum(ctx, buf, count, ctx->stream);
  });
}

extern "C" int eig_comm_barrier(eig_ctx_t ctx)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx, EIG_ERR_ARG, "null context");
    double *d = ctx->scratch + 4000;
    EIG_HIP(hipMemsetAsync(d, 0, sizeof(double), ctx->stream));
    allreduce_sum(ctx, d, 1, ctx->stream);
    EIG_HIP(hipStreamSynchronize(ctx->stream));
  });
}

// ============================================================================================
// device memory
// ============================================================================================
extern "C" int eig_malloc(eig_ctx_t ctx, size_t bytes, void **ptr)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && ptr, EIG_ERR_ARG, "eig_malloc: null argument");
    DeviceGuard dg(ctx->device);
    EIG_HIP(hipMalloc(ptr, bytes ? bytes : 1));
  });
}
extern "C" int eig_free(eig_ctx_t ctx, void *ptr)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx, EIG_ERR_ARG, "null context");
    if (ptr) EIG_HIP(hipFree(ptr));
  });
}
extern "C" int eig_memcpy_h2d(eig_ctx_t ctx, void *dst, const void *src, size_t bytes)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx, EIG_ERR_ARG, "null context");
    EIG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    EIG_HIP(hipStreamSynchronize(ctx->stream));
  });
}
extern "C" int eig_memcpy_d2h(eig_ctx_t ctx, void *dst, const void *src, size_t bytes)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx, EIG_ERR_ARG, "null context");
    EIG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    EIG_HIP(hipStreamSynchronize(ctx->stream));
  });
}
extern "C" int eig_memcpy_d2d(eig_ctx_t ctx, void *dst, const void *src, size_t bytes)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx, EIG_ERR_ARG, "null context");
    EIG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  });
}
extern "C" int eig_memset(eig_ctx_t ctx, void *dst, int value, size_t bytes)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx, EIG_ERR_ARG, "null context");
    EIG_HIP(hipMemsetAsync(dst, value, bytes, ctx->stream));
  });
}

// ============================================================================================
// matrices
// ============================================================================================
namespace {


template <class F>
void parallel_slices(i64 ns, F &&f)
{
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (ns < 4096) nt = 1;
  if (nt == 1) f(0, ns);
  else
  {
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back([&, t] { f(ns * t / nt, ns * (t + 1) / nt); });
    for (auto &t : th) t.join();
  }
}

// Build the SELL-C image (C = 64 R) of `nb` block rows (rowptr/col/vals on the host; columns are
// shifted by col_shift into window-local block columns; global row = row_begin + r) and upload.
// 1x1 slices whose rows use at most 8 distinct offsets (col - row) become stencil slices: their
// value slots are indexed by offset and a per-row mask marks the stored entries (internal.h).
void build_sell(eig_mat_s &A, i64 nb, const int64_t *rowptr, const int32_t *col, const double *vals, i64 col_shift)
{
  const int bb = A.br * A.bc;
  A.R = 1;  // one row per lane (2 / 4 measured slower for the fused Lanczos kernel)
  const i64 C = 64 * (i64)A.R;
  const i64 ns = (nb + C - 1) / C;
  const bool try_stencil = (bb == 1) && !(A.kflags & EIG_MAT_NO_STENCIL);
  const i64 row0 = A.row_begin;
  std::vector<i32> swidth(ns, -1), sdelta(8 * (size_t)ns, 0);
  std::vector<i64> sp(ns + 1, 0), wdt(ns, 0);
  parallel_slices(ns, [&](i64 s0, i64 s1) {
    std::vector<i64> offs;
    for (i64 s = s0; s < s1; ++s)
    {
      i64 w = 0;
      offs.clear();
      bool ok = try_stencil;
      for (i64 r = s * C; r < std::min(nb, s * C + C); ++r)
      {
        w = std::max<i64>(w, rowptr[r + 1] - rowptr[r]);
        for (i64 p = rowptr[r]; ok && p < rowptr[r + 1]; ++p)
        {
          const i64 d = (i64)col[p] - (row0 + r);
          if (std::find(offs.begin(), offs.end(), d) == offs.end())
          {
            if (offs.size() == 8 || d < INT32_MIN || d > INT32_MAX) ok = false;
            else offs.push_back(d);
          }
        }
      }
      if (ok && !offs.empty())
      {
        std::sort(offs.begin(), offs.end());
        swidth[s] = (i32)offs.size();
        for (size_t k = 0; k < offs.size(); ++k) sdelta[8 * s + k] = (i32)offs[k];
        w = (i64)offs.size();
      }
      wdt[s] = w;
    }
  });
  for (i64 s = 0; s < ns; ++s) sp[s + 1] = sp[s] + C * wdt[s];
  const i64 total = sp[ns];
  std::vector<i32> cimg(std::max<i64>(total, 1));
  std::vector<double> vimg(std::max<i64>(total * bb, 1));
  std::vector<uint8_t> mimg(try_stencil ? (size_t)(ns * C) : 0, 0);
  parallel_slices(ns, [&](i64 s0, i64 s1) {
    for (i64 s = s0; s < s1; ++s)
    {
      const i64 base = sp[s], w = (sp[s + 1] - base) / C;
      for (i64 l = 0; l < C; ++l)
      {
        const i64 r = s * C + l;
        const i64 len = (r < nb) ? rowptr[r + 1] - rowptr[r] : 0;
        for (i64 k = 0; k < w; ++k)
        {
          cimg[base + k * C + l] = -1;
          for (int t = 0; t < bb; ++t) vimg[(base + k * C) * bb + t * C + l] = 0.0;
        }
        for (i64 e = 0; e < len; ++e)
        {
          const i64 p = rowptr[r] + e;
          i64 k = e;
          if (swidth[s] > 0)
          {
            const i64 d = (i64)col[p] - (row0 + r);
            k = std::find(&sdelta[8 * s], &sdelta[8 * s] + swidth[s], (i32)d) - &sdelta[8 * s];
            mimg[s * C + l] |= (uint8_t)(1u << k);
          }
          cimg[base + k * C + l] = (i32)(col[p] - col_shift);
          for (int t = 0; t < bb; ++t) vimg[(base + k * C) * bb + t * C + l] = vals[p * bb + t];
        }
      }
    }
  });
  {
    std::vector<i64> bw(16, 0);
    const i64 nt = std::min<i64>(16, std::max<i64>(1, nb / 65536));
    std::vector<std::thread> th;
    for (i64 t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        i64 m = 0;
        for (i64 r = nb * t / nt; r < nb * (t + 1) / nt; ++r)
          for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p) m = std::max<i64>(m, std::llabs((i64)col[p] - (row0 + r)));
        bw[t] = m;
      });
    for (auto &x : th) x.join();
    A.bandwidth = *std::max_element(bw.begin(), bw.end());
  }
  A.nslices = ns;
  A.nnzb_padded = total;
  A.slice_ptr = dev_alloc<i64>(ns + 1);
  A.col = dev_alloc<i32>(total);
  A.val = dev_alloc<double>(total * bb);
  hipStream_t s = A.ctx->stream;
  EIG_HIP(hipMemcpyAsync(A.slice_ptr, sp.data(), (ns + 1) * sizeof(i64), hipMemcpyHostToDevice, s));
  EIG_HIP(hipMemcpyAsync(A.col, cimg.data(), total * sizeof(i32), hipMemcpyHostToDevice, s));
  EIG_HIP(hipMemcpyAsync(A.val, vimg.data(), total * bb * sizeof(double), hipMemcpyHostToDevice, s));
  A.n_stencil_slices = 0;
  A.sell_explicit = 0;
  for (i64 q = 0; q < ns; ++q)
  {
    A.n_stencil_slices += swidth[q] > 0;
    if (swidth[q] <= 0) A.sell_explicit += sp[q + 1] - sp[q];
  }
  if (A.n_stencil_slices > 0)
  {
    A.st_width = dev_alloc<i32>(ns);
    A.st_delta = dev_alloc<i32>(8 * ns);
    A.st_mask = dev_alloc<uint8_t>(ns * C);
    EIG_HIP(hipMemcpyAsync(A.st_width, swidth.data(), ns * sizeof(i32), hipMemcpyHostToDevice, s));
    EIG_HIP(hipMemcpyAsync(A.st_delta, sdelta.data(), 8 * ns * sizeof(i32), hipMemcpyHostToDevice, s));
    EIG_HIP(hipMemcpyAsync(A.st_mask, mimg.data(), ns * C, hipMemcpyHostToDevice, s));
  }
  EIG_HIP(hipStreamSynchronize(s));
  A.device_bytes = (ns + 1) * 8 + total * 4 + total * bb * 8 + (A.n_stencil_slices ? ns * (36 + C) : 0);
}


// Symmetric band image (internal.h, eig_mat_s::sym_*) next to the SELL image, for square 1x1
// matrices with at most kSymMaxOff distinct offsets whose stored mirror pairs are bitwise equal
// and whose band arrays are smaller than the SELL values.  Pass 1 (rows in parallel) stores each
// row's entries at d >= 0 in slot [j(d)][w]; pass 2 stores the entries at d < 0 in slot
// [j(-d)][w + d], which only the mirror (row w + d, offset -d) of pass 1 can also own -- a set
// slot with different bits rejects the image.  Ghost rows below the owned range (distributed)
// get their slots from the owned rows' lower entries alone.  Silently skipped when not applicable.
void build_sym(eig_mat_s &A, i64 nb, const int64_t *rowptr, const int32_t *col, const double *vals)
{
  if (A.br != 1 || A.bc != 1 || (A.kflags & EIG_MAT_NO_BAND) || nb == 0) return;
  if (A.nb_cols != A.nb_rows_global) return;
  const i64 row0 = A.row_begin;
  // distinct offsets (per thread, then merged)
  std::vector<i64> offs;
  {
    std::mutex mu;
    bool ok = true;
    parallel_slices(nb, [&](i64 r0, i64 r1) {
      std::vector<i64> mine;
      for (i64 r = r0; r < r1 && mine.size() <= (size_t)kSymMaxOff; ++r)
        for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p)
        {
          const i64 d = (i64)col[p] - (row0 + r);
          if (std::find(mine.begin(), mine.end(), d) == mine.end()) mine.push_back(d);
        }
      std::lock_guard<std::mutex> lk(mu);
      if (mine.size() > (size_t)kSymMaxOff) ok = false;
      for (i64 d : mine)
        if (std::find(offs.begin(), offs.end(), d) == offs.end()) offs.push_back(d);
    });
    if (!ok || offs.size() > (size_t)kSymMaxOff || offs.empty()) return;
  }
  std::sort(offs.begin(), offs.end());
  std::vector<i64> ups;
  for (i64 d : offs)
  {
    if (d < INT32_MIN || d > INT32_MAX) return;
    const i64 a = std::llabs(d);
    if (std::find(ups.begin(), ups.end(), a) == ups.end()) ups.push_back(a);
  }
  std::sort(ups.begin(), ups.end());
  const int nd = (int)offs.size(), nup = (int)ups.size();
  const i64 ns = A.nslices, own = A.own_offset;
  const i64 ld = ((std::max<i64>(A.window, own + ns * 64) + 63) / 64) * 64;
  // only worth it when the band arrays are smaller than the SELL values the kernels would stream
  if ((double)nup * (double)ld > 0.9 * (double)A.nnzb_padded) return;
  auto jof = [&](i64 a) { return (int)(std::lower_bound(ups.begin(), ups.end(), a) - ups.begin()); };
  std::vector<int> kj(nd);
  for (int k = 0; k < nd; ++k) kj[k] = jof(std::llabs(offs[k]));
  std::vector<double> U((size_t)nup * ld, 0.0);
  std::vector<uint8_t> set((size_t)nup * ld, 0);
  const int mb = nd <= 8 ? 1 : 4;
  std::vector<uint8_t> m8(mb == 1 ? (size_t)ns * 64 : 0, 0);
  std::vector<uint32_t> m32(mb == 4 ? (size_t)ns * 64 : 0, 0);
  std::atomic<bool> good{true};
  auto kof = [&](i64 d) { return (int)(std::lower_bound(offs.begin(), offs.end(), d) - offs.begin()); };
  parallel_slices(nb, [&](i64 r0, i64 r1) {
    for (i64 r = r0; r < r1; ++r)
    {
      uint32_t m = 0;
      for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p)
      {
        const i64 d = (i64)col[p] - (row0 + r);
        const int k = kof(d);
        m |= 1u << k;
        if (d >= 0)
        {
          const size_t q = (size_t)kj[k] * ld + (size_t)(own + r);
          U[q] = vals[p];
          set[q] = 1;
        }
      }
      if (mb == 1) m8[r] = (uint8_t)m;
      else m32[r] = m;
    }
  });
  parallel_slices(nb, [&](i64 r0, i64 r1) {
    for (i64 r = r0; r < r1 && good.load(std::memory_order_relaxed); ++r)
      for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p)
      {
        const i64 d = (i64)col[p] - (row0 + r);
        if (d >= 0) break;  // ascending columns: the rest are upper entries
        const i64 x = own + r + d;
        if (x < 0 || x >= ld)
        {
          good = false;
          break;
        }
        const size_t q = (size_t)kj[kof(d)] * ld + (size_t)x;
        if (set[q])
        {
          if (std::memcmp(&U[q], &vals[p], sizeof(double)) != 0)
          {
            good = false;
            break;
          }
        }
        else
          U[q] = vals[p];
      }
  });
  if (!good) return;
  // uniform band: one value per array over every stored entry, lower entries included (a lower entry
  // whose mirror is not stored on this rank -- a ghost row's coupling, or a one-sided pattern -- was
  // never compared in the mirror pass, and the uniform march kernels take the array's constant for it)
  {
    std::mutex mu;
    std::vector<double> uc(nup, 0.0);
    std::vector<char> seen(nup, 0);
    bool uni = true;
    parallel_slices(nb, [&](i64 r0, i64 r1) {
      std::vector<double> v(nup, 0.0);
      std::vector<char> sn(nup, 0);
      bool ok = true;
      for (i64 r = r0; r < r1 && ok; ++r)
        for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p)
        {
          const i64 d = (i64)col[p] - (row0 + r);
          const int j = kj[kof(d)];
          if (!sn[j])
          {
            sn[j] = 1;
            v[j] = vals[p];
          }
          else if (std::memcmp(&v[j], &vals[p], sizeof(double)) != 0)
          {
            ok = false;
            break;
          }
        }
      std::lock_guard<std::mutex> lk(mu);
      uni = uni && ok;
      for (int j = 0; j < nup && uni; ++j)
        if (sn[j])
        {
          if (!seen[j])
          {
            seen[j] = 1;
            uc[j] = v[j];
          }
          else if (std::memcmp(&uc[j], &v[j], sizeof(double)) != 0)
            uni = false;
        }
    });
    A.sym_uniform = uni;
    for (int j = 0; j < nup; ++j) A.sym_uc[j] = uni ? uc[j] : 0.0;
  }
  // geometric masks: a grid whose rows store exactly their in-grid neighbours -- the whole grid on
  // one rank, or a rank's slab of whole planes (row0 and nb multiples of the plane size D; z is
  // the global plane, so the slab's first / last planes keep their ghost-plane bits).  A property of
  // the pattern alone: the uniform marches take the values from their arguments, the value march
  // (march variant 10) streams them from the band arrays.
  A.sym_geo = false;
  if (mb == 1 && offs.front() == -offs.back() && (nd == 7 || nd == 5))
  {
    const i64 D = offs.back();
    const i64 nx = nd == 7 ? offs[5] : D;
    bool shape = D > 1 && nx > 1 && D % nx == 0 && nb % D == 0 && row0 % D == 0 && A.nb_rows_global % D == 0 &&
                 (nd == 5 || (offs[4] == 1 && offs[2] == -1 && offs[1] == -nx && nx < D));
    if (nd == 5) shape = shape && offs[1] == -1 && offs[3] == 1;
    if (shape)
    {
      const i64 ny = D / nx, nz = A.nb_rows_global / D;
      std::atomic<bool> same{true};
      parallel_slices(nb, [&](i64 r0, i64 r1) {
        for (i64 r = r0; r < r1 && same.load(std::memory_order_relaxed); ++r)
        {
          const i64 g = row0 + r;
          const i64 x = g % nx, y = (g / nx) % ny, z = g / D;
          unsigned e = 0;
          int k = 0;
          e |= (z > 0 ? 1u : 0u) << k++;
          if (nd == 7) e |= (y > 0 ? 1u : 0u) << k++;
          e |= (x > 0 ? 1u : 0u) << k++;
          e |= 1u << k++;
          e |= (x < nx - 1 ? 1u : 0u) << k++;
          if (nd == 7) e |= (y < ny - 1 ? 1u : 0u) << k++;
          e |= (z < nz - 1 ? 1u : 0u) << k++;
          if (e != m8[r]) same = false;
        }
      });
      if (same && nx <= INT32_MAX && ny <= INT32_MAX && nz <= INT32_MAX)
      {
        A.sym_geo = true;
        A.sym_gx = (int)nx;
        A.sym_gy = (int)ny;
        A.sym_gz = (int)nz;
        A.sym_gz0 = (int)(row0 / D);
      }
    }
  }
  // box-geometric masks (general 27-point box subsets, e.g. the P1 Kuhn 15-point stencil): decompose the
  // offsets as a D + b nx + c -- nx the smallest offset > 1 (or that + 1 when (0, 1, -1) is stored), D
  // the smallest offset past nx + 1 (or that + 1, + nx - 1, + nx, + nx + 1) -- then check row by row
  A.sym_box27 = 0;
  if (!A.sym_geo && nd >= 3 && nd <= 27 && offs.front() == -offs.back())
  {
    i64 s1 = 0;
    for (i64 d : offs)
      if (d > 1 && (s1 == 0 || d < s1)) s1 = d;
    std::vector<int> bx(nd), by(nd), bz(nd);
    auto decompose = [&](i64 nxc, i64 Dc) {
      for (int k = 0; k < nd; ++k)
      {
        bool found = false;
        for (int a = -1; a <= 1 && !found; ++a)
          for (int b2 = -1; b2 <= 1 && !found; ++b2)
            for (int c = -1; c <= 1 && !found; ++c)
              if (a * Dc + b2 * nxc + c == offs[k]) bz[k] = a, by[k] = b2, bx[k] = c, found = true;
        if (!found) return false;
      }
      return true;
    };
    i64 gnx = 0, gD = 0;
    for (i64 nxc : {s1, s1 + 1})
    {
      if (nxc < 3 || gD) continue;
      i64 t = 0;
      for (i64 d : offs)
        if (d > nxc + 1 && (t == 0 || d < t)) t = d;
      if (t == 0) continue;
      for (i64 Dc : {t, t + 1, t + nxc - 1, t + nxc, t + nxc + 1})
        if (!gD && Dc % nxc == 0 && Dc / nxc >= 3 && A.nb_rows_global % Dc == 0 && nb % Dc == 0 && row0 % Dc == 0 &&
            decompose(nxc, Dc))
          gnx = nxc, gD = Dc;
    }
    if (gD && A.nb_rows_global / gD >= 3 && gnx <= INT32_MAX && gD / gnx <= INT32_MAX &&
        A.nb_rows_global / gD <= INT32_MAX)
    {
      decompose(gnx, gD);
      const i64 gny = gD / gnx, gnz = A.nb_rows_global / gD;
      std::atomic<bool> same{true};
      parallel_slices(nb, [&](i64 r0, i64 r1) {
        for (i64 r = r0; r < r1 && same.load(std::memory_order_relaxed); ++r)
        {
          const i64 g = row0 + r;
          const i64 x = g % gnx, y = (g / gnx) % gny, z = g / gD;
          uint32_t e = 0;
          for (int k = 0; k < nd; ++k)
          {
            const i64 xx = x + bx[k], yy = y + by[k], zz = z + bz[k];
            if (xx >= 0 && xx < gnx && yy >= 0 && yy < gny && zz >= 0 && zz < gnz) e |= 1u << k;
          }
          if (e != (mb == 1 ? (uint32_t)m8[r] : m32[r])) same = false;
        }
      });
      if (same)
      {
        for (int k = 0; k < nd; ++k) A.sym_box27 |= 1u << ((bz[k] + 1) * 9 + (by[k] + 1) * 3 + (bx[k] + 1));
        A.sym_gx = (int)gnx;
        A.sym_gy = (int)gny;
        A.sym_gz = (int)gnz;
        A.sym_gz0 = (int)(row0 / gD);
      }
    }
  }
  hipStream_t s = A.ctx->stream;
  A.sym_val = dev_alloc<double>((size_t)nup * ld);
  A.sym_mask = mb == 1 ? (void *)dev_alloc<uint8_t>(ns * 64) : (void *)dev_alloc<uint32_t>(ns * 64);
  EIG_HIP(hipMemcpyAsync(A.sym_val, U.data(), (size_t)nup * ld * sizeof(double), hipMemcpyHostToDevice, s));
  EIG_HIP(hipMemcpyAsync(A.sym_mask, mb == 1 ? (const void *)m8.data() : (const void *)m32.data(), ns * 64 * mb,
                         hipMemcpyHostToDevice, s));
  EIG_HIP(hipStreamSynchronize(s));
  A.sym_mask_bytes = mb;
  A.sym_nd = nd;
  A.sym_nup = nup;
  A.sym_ld = ld;
  for (int k = 0; k < nd; ++k)
  {
    A.sym_off[k] = (i32)offs[k];
    A.sym_dj[k] = kj[k];
  }
  A.device_bytes += (i64)nup * ld * 8 + ns * 64 * mb;
}

void validate_csr(i64 nb, i64 ncols, const int64_t *rowptr, const int32_t *col)
{
  EIG_CHECK(rowptr[0] == 0, EIG_ERR_ARG, "rowptr[0] must be 0");
  for (i64 r = 0; r < nb; ++r)
  {
    EIG_CHECK(rowptr[r + 1] >= rowptr[r], EIG_ERR_ARG, "rowptr must be non-decreasing");
    for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p)
    {
      EIG_CHECK(col[p] >= 0 && col[p] < ncols, EIG_ERR_SHAPE, "column index out of range");
      if (p > rowptr[r]) EIG_CHECK(col[p] > col[p - 1], EIG_ERR_ARG, "columns must be strictly ascending per row");
    }
  }
}

// Diagonal share of the owned rows (global row = row_begin + r): sum of the stored diagonal
// entries of the diagonal blocks and the number of scalar rows that store one.
void diag_share(eig_mat_s &A, i64 nb, i64 row_begin, const int64_t *rowptr, const int32_t *col, const double *vals)
{
  const int br = A.br, bc = A.bc;
  double s = 0.0;
  i64 cnt = 0;
  for (i64 r = 0; r < nb; ++r)
    for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p)
      if (col[p] == row_begin + r)
        for (int i = 0; i < std::min(br, bc); ++i)
        {
          s += vals[p * br * bc + (i64)i * bc + i];
          ++cnt;
        }
  A.diag_sum = s;
  A.diag_count = cnt;
}

void destroy_mat(eig_mat_s *A)
{
  if (!A) return;
  if (A->slice_ptr) (void)hipFree(A->slice_ptr);
  if (A->col) (void)hipFree(A->col);
  if (A->val) (void)hipFree(A->val);
  if (A->st_width) (void)hipFree(A->st_width);
  if (A->st_delta) (void)hipFree(A->st_delta);
  if (A->st_mask) (void)hipFree(A->st_mask);
  if (A->slice_list) (void)hipFree(A->slice_list);
  if (A->march_bnd) (void)hipFree(A->march_bnd);
  if (A->sym_val) (void)hipFree(A->sym_val);
  if (A->sym_pack) (void)hipFree(A->sym_pack);
  if (A->sym_mask) (void)hipFree(A->sym_mask);
  if (A->box_val) (void)hipFree(A->box_val);
  if (A->box_ctab) (void)hipFree(A->box_ctab);
  if (A->box_cmask) (void)hipFree(A->box_cmask);
  delete A;
}

}  // namespace

extern "C" int eig_mat_create_bcsr(eig_ctx_t ctx, int64_t nb_rows, int64_t nb_cols, int br, int bc,
                                   const int64_t *rowptr, const int32_t *col, const double *vals, eig_mat_t *out)
{
  return eig_mat_create_bcsr_ex(ctx, nb_rows, nb_cols, br, bc, rowptr, col, vals, 0, out);
}

extern "C" int eig_mat_create_bcsr_ex(eig_ctx_t ctx, int64_t nb_rows, int64_t nb_cols, int br, int bc,
                                      const int64_t *rowptr, const int32_t *col, const double *vals, int flags,
                                      eig_mat_t *out)
{
  return guard(ctx, [&] {
    EIG_CHECK((flags & ~EIG_MAT_FLAGS_ALL) == 0, EIG_ERR_ARG, "eig_mat_create_bcsr_ex: unknown flag");
    EIG_CHECK(ctx && out && rowptr && (rowptr[nb_rows] == 0 || (col && vals)), EIG_ERR_ARG,
              "eig_mat_create_bcsr: null argument");
    EIG_CHECK(nb_rows >= 0 && nb_cols >= 0, EIG_ERR_ARG, "eig_mat_create_bcsr: negative size");
    EIG_CHECK(br >= 1 && br <= 4 && bc >= 1 && bc <= 4, EIG_ERR_BLOCKSIZE, "block size must be in 1..4");
    EIG_CHECK(nb_cols * bc < (int64_t)INT32_MAX, EIG_ERR_SHAPE, "matrix too large for int32 column indices");
    DeviceGuard dg(ctx->device);
    validate_csr(nb_rows, nb_cols, rowptr, col);
    auto *A = new eig_mat_s();
    A->ctx = ctx;
    A->kflags = flags;
    A->br = br;
    A->bc = bc;
    A->nb_rows = A->nb_rows_global = nb_rows;
    A->nb_cols = nb_cols;
    A->row_begin = 0;
    A->win_begin = 0;
    A->window = nb_cols * bc;
    A->own_offset = 0;
    A->nnzb = rowptr[nb_rows];
    try
    {
      build_sell(*A, nb_rows, rowptr, col, vals, 0);
      build_sym(*A, nb_rows, rowptr, col, vals);
      diag_share(*A, nb_rows, 0, rowptr, col, vals);
    }
    catch (...)
    {
      destroy_mat(A);
      throw;
    }
    *out = A;
  });
}

extern "C" int eig_mat_create_bcsr_dist(eig_ctx_t ctx, int64_t nb_rows_global, int64_t row_begin,
                                        int64_t nb_local, int br, int bc, const int64_t *rowptr, const int32_t *col,
                                        const double *vals, eig_mat_t *out)
{
  return eig_mat_create_bcsr_dist_ex(ctx, nb_rows_global, row_begin, nb_local, br, bc, rowptr, col, vals, 0, out);
}

extern "C" int eig_mat_create_bcsr_dist_ex(eig_ctx_t ctx, int64_t nb_rows_global, int64_t row_begin,
                                           int64_t nb_local, int br, int bc, const int64_t *rowptr,
                                           const int32_t *col, const double *vals, int flags, eig_mat_t *out)
{
  return guard(ctx, [&] {
    EIG_CHECK((flags & ~EIG_MAT_FLAGS_ALL) == 0, EIG_ERR_ARG, "eig_mat_create_bcsr_dist_ex: unknown flag");
    EIG_CHECK(ctx && out && rowptr, EIG_ERR_ARG, "eig_mat_create_bcsr_dist: null argument");
    EIG_CHECK(br == bc && br >= 1 && br <= 4, EIG_ERR_BLOCKSIZE, "distributed matrices need square blocks 1..4");
    EIG_CHECK(row_begin >= 0 && nb_local >= 0 && row_begin + nb_local <= nb_rows_global, EIG_ERR_SHAPE,
              "eig_mat_create_bcsr_dist: row range outside the matrix");
    EIG_CHECK(nb_rows_global * bc < (int64_t)INT32_MAX, EIG_ERR_SHAPE, "matrix too large for int32 column indices");
    DeviceGuard dg(ctx->device);
    validate_csr(nb_local, nb_rows_global, rowptr, col);
    const int P = ctx->nranks, me = ctx->rank;
    int64_t plan[5];
    {
      int rc = eig_plan_window(row_begin, nb_local, bc, rowptr, col, plan);
      EIG_CHECK(rc == EIG_OK, rc, "eig_plan_window failed");
    }
    const i64 wb_blk = plan[0], cmin = plan[3], cmax = plan[4];
    auto *A = new eig_mat_s();
    A->ctx = ctx;
    A->kflags = flags;
    A->br = br;
    A->bc = bc;
    A->nb_rows = nb_local;
    A->nb_rows_global = nb_rows_global;
    A->nb_cols = nb_rows_global;
    A->row_begin = row_begin;
    A->win_begin = wb_blk * bc;
    A->window = plan[1];
    A->own_offset = plan[2];
    A->nnzb = rowptr[nb_local];
    try
    {
      build_sell(*A, nb_local, rowptr, col, vals, wb_blk);
      build_sym(*A, nb_local, rowptr, col, vals);
      diag_share(*A, nb_local, row_begin, rowptr, col, vals);
      // --- halo plan: allgather (row_begin, nb_local, cmin, cmax) of every rank ---
      std::vector<i64> mine = {row_begin, nb_local, cmin, cmax};
      std::vector<i64> all(4 * (size_t)P, 0);
      if (ctx->loop && P > 1)
      {
        LoopHub &h = *ctx->loop;
        {
          std::lock_guard<std::mutex> lk(h.m);
          for (int t = 0; t < 4; ++t) h.gather[4 * me + t] = mine[t];
        }
        h.barrier();
        all = h.gather;
        h.barrier();
      }
      else if (!ctx->comm && P > 1 && ctx->mbox && ctx->mbox->ready)
      {
        // mailbox-only ranks (eig_comm_ipc_open): an allgather as an allreduce of zero-padded rows
        // (integers below 2^53: the double sums are exact)
        std::vector<double> g(4 * (size_t)P, 0.0);
        for (int t = 0; t < 4; ++t) g[4 * me + t] = (double)mine[t];
        double *d = dev_alloc<double>(g.size());
        EIG_HIP(hipMemcpy(d, g.data(), g.size() * sizeof(double), hipMemcpyHostToDevice));
        for (i64 off = 0; off < (i64)g.size(); off += kMailboxVals)
          launch_mailbox_allreduce(d + off, (int)std::min<i64>(kMailboxVals, (i64)g.size() - off), ctx->mbox->dev,
                                   kMailboxTimeout, ctx->stream);
        EIG_HIP(hipStreamSynchronize(ctx->stream));
        EIG_HIP(hipMemcpy(g.data(), d, g.size() * sizeof(double), hipMemcpyDeviceToHost));
        (void)hipFree(d);
        int err = 0;
        EIG_HIP(hipMemcpy(&err, ctx->mbox->dev.err, sizeof(int), hipMemcpyDeviceToHost));
        EIG_CHECK(err == 0, EIG_ERR_RCCL, "eig_mat_create_bcsr_dist: mailbox allgather timed out");
        for (size_t t = 0; t < g.size(); ++t) all[t] = (i64)g[t];
      }
      else if (ctx->comm && P > 1)
      {
        i64 *d = dev_alloc<i64>(4 * (size_t)P);
        EIG_HIP(hipMemcpy(d + 4 * me, mine.data(), 4 * sizeof(i64), hipMemcpyHostToDevice));
        EIG_NCCL(ncclAllGather(d + 4 * me, d, 4 * sizeof(i64), ncclChar, ctx->comm, ctx->stream));
        EIG_HIP(hipStreamSynchronize(ctx->stream));
        EIG_HIP(hipMemcpy(all.data(), d, 4 * P * sizeof(i64), hipMemcpyDeviceToHost));
        (void)hipFree(d);
      }
      else
      {
        all = mine;
      }
      const int nr = ctx->distributed() ? P : 1;
      std::vector<int64_t> rv(3 * (size_t)nr), sd(3 * (size_t)nr);
      int nrecv = 0, nsend = 0;
      {
        int rc = eig_plan_halo(nr, nr > 1 ? me : 0, all.data(), bc, wb_blk, rv.data(), &nrecv, sd.data(), &nsend);
        EIG_CHECK(rc == EIG_OK, rc, "eig_plan_halo failed");
      }
      if (!ctx->loop && P > 1 && ctx->mbox && ctx->mbox->ready)
      {
        // the halo mailbox's slots hold the largest range of any rank's plan, 8 columns wide
        // (blanczos.cpp exchanges blocks of 8); grown collectively when a matrix needs more
        i64 most = 0;
        std::vector<int64_t> qr(3 * (size_t)P), qs(3 * (size_t)P);
        for (int q = 0; q < P; ++q)
        {
          int nq = 0, ns = 0;
          int rc = eig_plan_halo(P, q, all.data(), bc, 0, qr.data(), &nq, qs.data(), &ns);
          EIG_CHECK(rc == EIG_OK, rc, "eig_plan_halo failed");
          for (int k = 0; k < nq; ++k) most = std::max<i64>(most, qr[3 * k + 2]);
        }
        const i64 cap = 8 * most;
        if (cap > 0 && (!ctx->hbox || ctx->hbox->dev.cap < cap))
        {
          if (!ctx->comm)
            halobox_setup(ctx, cap);  // mailbox-only ranks: their only halo transport
          else
          {
            // beside RCCL the halo mailbox is an option (eig_comm_select_halo): a rank set that could
            // not build it keeps ncclSend / ncclRecv (the failure is agreed inside halobox_setup)
            try
            {
              halobox_setup(ctx, cap);
            }
            catch (const Error &)
            {
              halobox_free(ctx);
              ctx->halo_mailbox = false;
            }
          }
        }
      }
      for (int k = 0; k < nrecv; ++k) A->recvs.push_back({(int)rv[3 * k], rv[3 * k + 1], rv[3 * k + 2]});
      for (int k = 0; k < nsend; ++k) A->sends.push_back({(int)sd[3 * k], sd[3 * k + 1], sd[3 * k + 2]});
      for (auto &r : A->recvs) A->halo_recv += r.count;
      for (auto &r : A->sends) A->halo_send += r.count;
      // interior / boundary slices: a slice is interior when every column is owned
      std::vector<i32> inter, bound;
      const i64 own_lo = row_begin, own_hi = row_begin + nb_local;
      for (i64 s = 0; s < A->nslices; ++s)
      {
        bool in = true;
        const i64 C = 64 * (i64)A->R;
        for (i64 r = s * C; r < std::min(nb_local, s * C + C) && in; ++r)
          for (i64 p = rowptr[r]; p < rowptr[r + 1]; ++p)
            if (col[p] < own_lo || col[p] >= own_hi)
            {
              in = false;
              break;
            }
        (in ? inter : bound).push_back((i32)s);
      }
      A->n_interior = (i64)inter.size();
      A->n_boundary = (i64)bound.size();
      std::vector<i32> lst(inter);
      lst.insert(lst.end(), bound.begin(), bound.end());
      A->slice_list = dev_alloc<i32>(std::max<size_t>(lst.size(), 1));
      if (!lst.empty()) EIG_HIP(hipMemcpy(A->slice_list, lst.data(), lst.size() * sizeof(i32), hipMemcpyHostToDevice));
      // plane-march split: the longest run of planes whose slices are all interior (>= 2 planes)
      i64 D;
      if (march_geometry(*A, D))
      {
        const i64 spp = D / 64, np = (nb_local + D - 1) / D;
        std::vector<char> is_in(A->nslices, 0);
        for (i32 q : inter) is_in[q] = 1;
        i64 best0 = 0, best1 = 0;
        for (i64 z = 0; z < np;)
        {
          auto plane_in = [&](i64 zz) {
            for (i64 q = zz * spp; q < std::min(A->nslices, (zz + 1) * spp); ++q)
              if (!is_in[q]) return false;
            return true;
          };
          if (!plane_in(z))
          {
            ++z;
            continue;
          }
          i64 e = z;
          while (e < np && plane_in(e)) ++e;
          if (e - z > best1 - best0) best0 = z, best1 = e;
          z = e;
        }
        if (best1 - best0 >= 2)
        {
          std::vector<i32> bnd;
          for (i64 q = 0; q < A->nslices; ++q)
            if (q < best0 * spp || q >= best1 * spp) bnd.push_back((i32)q);
          A->mz0 = best0;
          A->mz1 = best1;
          A->n_march_bnd = (i64)bnd.size();
          A->march_bnd = dev_alloc<i32>(std::max<size_t>(bnd.size(), 1));
          if (!bnd.empty())
            EIG_HIP(hipMemcpy(A->march_bnd, bnd.data(), bnd.size() * sizeof(i32), hipMemcpyHostToDevice));
        }
      }
    }
    catch (...)
    {
      destroy_mat(A);
      throw;
    }
    *out = A;
  });
}

namespace eigmi {
void mat_download_bcsr(const eig_mat_s &A, std::vector<i64> &rowptr, std::vector<i32> &col, std::vector<double> &vals)
{
  EIG_CHECK(!A.ctx->distributed() || A.nb_rows == A.nb_rows_global, EIG_ERR_ARG, "download: single-rank matrix only");
  const i64 C = 64 * (i64)A.R, ns = A.nslices, bb = (i64)A.br * A.bc;
  std::vector<i64> sp(ns + 1);
  std::vector<i32> ci(std::max<i64>(A.nnzb_padded, 1));
  std::vector<double> vi(std::max<i64>(A.nnzb_padded * bb, 1));
  EIG_HIP(hipMemcpy(sp.data(), A.slice_ptr, (ns + 1) * sizeof(i64), hipMemcpyDeviceToHost));
  if (A.nnzb_padded)
  {
    EIG_HIP(hipMemcpy(ci.data(), A.col, A.nnzb_padded * sizeof(i32), hipMemcpyDeviceToHost));
    EIG_HIP(hipMemcpy(vi.data(), A.val, A.nnzb_padded * bb * sizeof(double), hipMemcpyDeviceToHost));
  }
  rowptr.assign(A.nb_rows + 1, 0);
  col.clear();
  vals.clear();
  for (i64 r = 0; r < A.nb_rows; ++r)
  {
    const i64 s = r / C, l = r % C, base = sp[s], w = (sp[s + 1] - base) / C;
    for (i64 k = 0; k < w; ++k)
    {
      const i32 c = ci[base + k * C + l];
      if (c < 0) continue;
      col.push_back(c + (i32)(A.win_begin / A.bc));
      for (i64 t = 0; t < bb; ++t) vals.push_back(vi[(base + k * C) * bb + t * C + l]);
    }
    rowptr[r + 1] = (i64)col.size();
  }
}
}  // namespace eigmi

extern "C" int eig_mat_destroy(eig_mat_t A)
{
  if (!A) return EIG_OK;
  (void)hipSetDevice(A->ctx->device);
  (void)hipStreamSynchronize(A->ctx->stream);
  destroy_mat(A);
  return EIG_OK;
}

extern "C" int eig_mat_get_info(eig_mat_t A, eig_mat_info *info)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && info, EIG_ERR_ARG, "null argument");
    info->n = A->nb_rows * A->br;
    info->n_global = A->nb_rows_global * A->br;
    info->ncols = A->nb_cols * A->bc;
    info->row_begin = A->row_begin * A->br;
    info->window = A->window;
    info->own_offset = A->own_offset;
    info->nnzb = A->nnzb;
    info->nnzb_padded = A->nnzb_padded;
    info->nslices = A->nslices;
    info->br = A->br;
    info->bc = A->bc;
    info->halo_recv = A->halo_recv;
    info->halo_send = A->halo_send;
    info->device_bytes = A->device_bytes;
    info->stencil_slices = A->n_stencil_slices;
    info->rows_per_lane = A->R;
    info->sym_offsets = A->sym_val ? A->sym_nd : 0;
    info->sym_arrays = A->sym_val ? A->sym_nup : 0;
    info->sym_mask_bytes = A->sym_val ? A->sym_mask_bytes : 0;
    info->sym_uniform = (A->sym_val && A->sym_uniform && !(A->kflags & EIG_MAT_NO_UNIFORM))
                            ? (A->sym_geo ? 2 : 1)
                            : 0;
    info->sym_geo = A->sym_val && A->sym_geo ? 1 : 0;
    info->march_variant = march_variant(*A, true);
    info->march_variant_mv = march_variant(*A, false);
  });
}

extern "C" int eig_lanczos_kernel_info(eig_mat_t A, int fused, char *name, int name_len, int64_t *bytes)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && bytes && (name || name_len == 0), EIG_ERR_ARG, "eig_lanczos_kernel_info: null argument");
    std::string nm;
    i64 b = 0;
    lanczos_kernel_info(*A, fused != 0, nm, b);
    *bytes = b;
    if (name_len > 0)
    {
      const size_t k = std::min<size_t>(nm.size(), (size_t)name_len - 1);
      std::memcpy(name, nm.data(), k);
      name[k] = 0;
    }
  });
}

extern "C" int eig_mat_kernel_info(eig_mat_t A, int op, char *name, int name_len)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && name && name_len > 0, EIG_ERR_ARG, "eig_mat_kernel_info: null argument");
    EIG_CHECK(op >= EIG_OP_SPMV && op <= EIG_OP_CHEB32, EIG_ERR_ARG, "eig_mat_kernel_info: bad op");
    const std::string nm = kernel_for(*A, op);
    const size_t k = std::min<size_t>(nm.size(), (size_t)name_len - 1);
    std::memcpy(name, nm.data(), k);
    name[k] = 0;
  });
}

extern "C" int eig_mat_shift_diag(eig_mat_t A, double shift)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A, EIG_ERR_ARG, "null matrix");
    EIG_CHECK(A->br == A->bc, EIG_ERR_BLOCKSIZE, "StandardLargest: blocks of input matrix must be square");
    DeviceGuard dg(A->ctx->device);
    launch_shift_diag(*A, shift, A->ctx->stream);
  });
}

namespace eigmi {
// y = A x with halo exchange overlapped with the interior slices when distributed.
void mv_device(eig_mat_s &A, double *x, double *y)
{
  eig_ctx_t ctx = A.ctx;
  if (!ctx->distributed() || (A.recvs.empty() && A.sends.empty()))
  {
    launch_spmv(A, x, y, nullptr, 0, A.nslices, ctx->stream);
    return;
  }
  // interior / boundary split: the interior planes on the plane march when it applies, else the
  // interior slices
  const bool mz = march_split_active(A);
  auto interior = [&](hipStream_t s) {
    if (mz) launch_spmv(A, x, y, &kMarchInteriorTag, 0, 0, s);
    else launch_spmv(A, x, y, A.slice_list, 0, A.n_interior, s);
  };
  auto boundary = [&](hipStream_t s) {
    if (mz) launch_spmv(A, x, y, A.march_bnd, 0, A.n_march_bnd, s);
    else launch_spmv(A, x, y, A.slice_list, A.n_interior, A.n_boundary, s);
  };
  if (ctx->loop)
  {
    // synchronous exchange, then the same interior / boundary launches as the RCCL path
    halo_exchange(A, x, ctx->stream);
    interior(ctx->stream);
    boundary(ctx->stream);
    return;
  }
  hipEvent_t e0, e1;
  EIG_HIP(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
  EIG_HIP(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  EIG_HIP(hipEventRecord(e0, ctx->stream));
  EIG_HIP(hipStreamWaitEvent(ctx->comm_stream, e0, 0));
  halo_exchange(A, x, ctx->comm_stream);
  EIG_HIP(hipEventRecord(e1, ctx->comm_stream));
  interior(ctx->stream);
  EIG_HIP(hipStreamWaitEvent(ctx->stream, e1, 0));
  boundary(ctx->stream);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}
}  // namespace eigmi

extern "C" int eig_mv(eig_mat_t A, const double *x, double *y)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && x && y, EIG_ERR_ARG, "eig_mv: null argument");
    DeviceGuard dg(A->ctx->device);
    mv_device(*A, const_cast<double *>(x), y);
  });
}

extern "C" int eig_mv_timed(eig_mat_t A, const double *x, double *y, int reps, double *avg_ms)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && x && y && avg_ms && reps > 0, EIG_ERR_ARG, "eig_mv_timed: bad argument");
    DeviceGuard dg(A->ctx->device);
    hipStream_t s = A->ctx->stream;
    hipEvent_t e0, e1;
    EIG_HIP(hipEventCreate(&e0));
    EIG_HIP(hipEventCreate(&e1));
    EIG_HIP(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) mv_device(*A, const_cast<double *>(x), y);
    EIG_HIP(hipEventRecord(e1, s));
    EIG_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    EIG_HIP(hipEventElapsedTime(&ms, e0, e1));
    *avg_ms = ms / reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  });
}

extern "C" int eig_mv_host(eig_mat_t A, const double *xh, double *yh)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && xh && yh, EIG_ERR_ARG, "eig_mv_host: null argument");
    DeviceGuard dg(A->ctx->device);
    eig_ctx_t ctx = A->ctx;
    const size_t wb = (size_t)A->window * sizeof(double);
    double *x = (double *)ctx_buffer(ctx, 0, wb);
    double *y = (double *)ctx_buffer(ctx, 1, wb);
    const i64 n = A->nb_rows * A->br;
    if (A->nb_rows_global == A->nb_rows && !ctx->distributed())
    {
      // square or rectangular single-rank operator: x has ncols entries
      EIG_HIP(hipMemcpyAsync(x, xh, (size_t)A->nb_cols * A->bc * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    }
    else
    {
      EIG_HIP(hipMemsetAsync(x, 0, wb, ctx->stream));
      EIG_HIP(hipMemcpyAsync(x + A->own_offset, xh, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    }
    mv_device(*A, x, y);
    EIG_HIP(hipMemcpyAsync(yh, y + A->own_offset, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    EIG_HIP(hipStreamSynchronize(ctx->stream));
  });
}

// ============================================================================================
// BlockVector ops
// ============================================================================================
extern "C" int eig_dot(eig_ctx_t ctx, int64_t n, const double *x, const double *y, double *result)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && x && y && result && n >= 0, EIG_ERR_ARG, "eig_dot: bad argument");
    DeviceGuard dg(ctx->device);
    launch_dot(n, x, y, result, 0, ctx->stream, ctx->red);
    allreduce_sum(ctx, result, 1, ctx->stream);
  });
}
extern "C" int eig_nrm2(eig_ctx_t ctx, int64_t n, const double *x, double *result)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && x && result && n >= 0, EIG_ERR_ARG, "eig_nrm2: bad argument");
    DeviceGuard dg(ctx->device);
    launch_nrm2sq(n, x, result, 0, ctx->stream, ctx->red);
    allreduce_sum(ctx, result, 1, ctx->stream);
    launch_sqrt_inplace(result, 1, ctx->stream);
  });
}
extern "C" int eig_lanczos_update(eig_ctx_t ctx, int64_t n, const double *alpha, const double *beta,
                                  const double *v, const double *vprev, double *w, double *result)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && alpha && v && w && result && n >= 0 && (!vprev || beta), EIG_ERR_ARG,
              "eig_lanczos_update: bad argument");
    DeviceGuard dg(ctx->device);
    launch_lanczos_update_ext(n, alpha, beta, v, vprev, w, result, 0, ctx->stream, ctx->red);
    allreduce_sum(ctx, result, 2, ctx->stream);  // ||w||^2 and v.w in ONE allreduce
    launch_sqrt_inplace(result, 1, ctx->stream);
  });
}
extern "C" int eig_axpy(eig_ctx_t ctx, int64_t n, double a, const double *x, double *y)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && x && y && n >= 0, EIG_ERR_ARG, "eig_axpy: bad argument");
    DeviceGuard dg(ctx->device);
    launch_axpy(n, a, x, y, ctx->stream);
  });
}
extern "C" int eig_scal(eig_ctx_t ctx, int64_t n, double a, double *x)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && x && n >= 0, EIG_ERR_ARG, "eig_scal: bad argument");
    DeviceGuard dg(ctx->device);
    launch_scal(n, a, x, ctx->stream);
  });
}
extern "C" int eig_copy(eig_ctx_t ctx, int64_t n, const double *x, double *y)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && x && y && n >= 0, EIG_ERR_ARG, "eig_copy: bad argument");
    DeviceGuard dg(ctx->device);
    EIG_HIP(hipMemcpyAsync(y, x, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
  });
}

extern "C" int eig_stream_copy_timed(eig_ctx_t ctx, int64_t n, const double *x, double *y, int reps, int mode,
                                     double *avg_ms)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && x && y && n >= 0 && reps >= 1 && avg_ms, EIG_ERR_ARG, "eig_stream_copy_timed: bad argument");
    DeviceGuard dg(ctx->device);
    hipStream_t s = ctx->stream;
    hipEvent_t e0, e1;
    EIG_HIP(hipEventCreate(&e0));
    EIG_HIP(hipEventCreate(&e1));
    launch_stream_copy(n, x, y, ctx->num_cu, s, mode);  // warm-up
    EIG_HIP(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch_stream_copy(n, x, y, ctx->num_cu, s, mode);
    EIG_HIP(hipEventRecord(e1, s));
    EIG_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    EIG_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *avg_ms = ms / reps;
  });
}

// ============================================================================================
// MultiVector<double,8>
// ============================================================================================
#define EIG_MV8_CHECK(m)                                                                             \
  EIG_CHECK((m) % 8 == 0, EIG_ERR_SHAPE, "number of cols must be a multiple of block size");       \
  EIG_CHECK((m) >= 0, EIG_ERR_ARG, "negative column count")

extern "C" int eig_spmm_mv8(eig_mat_t A, int64_t m, const double *Qin, double *Qout)
{
  return guard(A ? A->ctx : nullptr, [&] {
    EIG_CHECK(A && Qin && Qout, EIG_ERR_ARG, "eig_spmm_mv8: null argument");
    EIG_MV8_CHECK(m);
    EIG_CHECK(A->nb_rows == A->nb_cols && !A->ctx->distributed(), EIG_ERR_SHAPE,
              "eig_spmm_mv8: square single-rank matrix required");
    DeviceGuard dg(A->ctx->device);
    if (m > 0) launch_spmm_mv8(*A, m, Qin, Qout, A->ctx->stream);
  });
}

extern "C" int eig_dot_diag_mv8(eig_ctx_t ctx, int64_t n, int64_t m, const double *Q1, const double *Q2, double *dp)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && Q1 && Q2 && dp && n >= 0, EIG_ERR_ARG, "eig_dot_diag_mv8: bad argument");
    EIG_MV8_CHECK(m);
    DeviceGuard dg(ctx->device);
    for (i64 b = 0; b < m; b += 8 * 32)
    {
      const i64 mm = std::min<i64>(m - b, 8 * 32);
      launch_dot_diag_mv8(n, mm, Q1 + b * n, Q2 + b * n, dp + b, 0, ctx->stream, ctx->red);
    }
    allreduce_sum(ctx, dp, m, ctx->stream);
  });
}

namespace eigmi {
// G (m1 x m2 row-major) = Q1^T Q2, tiled so that one launch stays within the ticket pool.
void gram_device(eig_ctx_t ctx, i64 n, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G)
{
  if (gram_mv8_chunks(m1, m2) <= 48)
  {
    launch_gram_mv8(n, m1, m2, Q1, Q2, G, 0, ctx->stream, ctx->red);
  }
  else
  {
    // row panels of Q1 (32 columns each) against all of Q2; write into a temp then scatter
    EIG_CHECK(gram_mv8_chunks(32, m2) <= 48, EIG_ERR_ARG, "gram: Q2 too wide (> 1536 columns)");
    double *tmp = (double *)ctx_buffer(ctx, 2, (size_t)32 * m2 * sizeof(double));
    for (i64 r = 0; r < m1; r += 32)
    {
      const i64 mr = std::min<i64>(32, m1 - r);
      launch_gram_mv8(n, mr, m2, Q1 + r * n, Q2, tmp, 0, ctx->stream, ctx->red);
      EIG_HIP(hipMemcpyAsync(G + r * m2, tmp, mr * m2 * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    }
  }
  allreduce_sum(ctx, G, m1 * m2, ctx->stream);
}


void spmm_dot_gram_device(const eig_mat_s &A, const double *X, double *Y, double *dp, double *gram)
{
  eig_ctx_t ctx = A.ctx;
  if (launch_spmm_dot_gram_mv8(A, 8, X, Y, dp, gram, ctx->stream, ctx->red)) return;
  // no fused kernel on this image: the product with its dots, then the panel Gram of the block
  launch_spmm_dot_mv8(A, 8, X, Y, dp, ctx->stream, ctx->red);
  gram_device(ctx, A.nb_rows, 8, 8, Y, Y, gram);
}

void orthonormalize_device(eig_ctx_t ctx, i64 n, i64 m, double *Q, int variant, const double *gram0)
{
  const int flags = variant & (EIG_ORTHO_GRID | EIG_ORTHO_NO_COOP | EIG_ORTHO_ONE_WG);
  const int la = (variant >> EIG_ORTHO_LOOKAHEAD_SHIFT) & 15;  // EIG_ORTHO_LOOKAHEAD(L); 0: the default
  const int L = la ? std::min(la, 8) : mgs_lookahead_default();
  variant &= 0xff;
  hipStream_t s = ctx->stream;
  double *S = (double *)ctx_buffer(ctx, 3, 64 * sizeof(double));
  double *U = S + 0;  // reused: Ssum for MGS, Gram for CholQR
  double *U2 = (double *)ctx_buffer(ctx, 4, 64 * sizeof(double));
  double *Sg = nullptr;
  if (m > 8) Sg = (double *)ctx_buffer(ctx, 5, (size_t)8 * m * sizeof(double));
  for (i64 bk = 0; bk < m; bk += 8)
  {
    double *Qb = Q + bk * n;
    if (bk == 0 && gram0 && variant == EIG_ORTHO_MGS && !ctx->distributed() && L == 8 &&
        launch_mgs_lookahead_gram(ctx, n, Qb, gram0, s))
    {
      // (the block's first read pass replaced by the Gram the caller's product summed)
    }
    else if (variant == EIG_ORTHO_MGS && !ctx->distributed() && (flags & EIG_ORTHO_ONE_WG) && !(flags & EIG_ORTHO_GRID) &&
        launch_mgs_small(n, Qb, s))
    {
    }
    else if (variant == EIG_ORTHO_MGS && !ctx->distributed() && !(flags & EIG_ORTHO_GRID) &&
             launch_mgs_coop(ctx, n, Qb, S, s))
    {
    }
    else if (variant == EIG_ORTHO_MGS && !ctx->distributed() && launch_mgs_lookahead(ctx, n, Qb, L, !(flags & EIG_ORTHO_NO_COOP), s))
    {
    }
    else if (variant == EIG_ORTHO_MGS)
    {
      for (int k = 0; k <= 8; ++k)
      {
        launch_mgs_pass(n, Qb, k, S, 0, s, ctx->red);
        if (k < 8) allreduce_sum(ctx, S + 8 * k, 8, s);
      }
    }
    else
    {
      gram_device(ctx, n, 8, 8, Qb, Qb, U);
      launch_cholqr_factor(U, U2, nullptr, 0, s);
      launch_apply_upper(n, Qb, U2, s);
    }
    const i64 mrest = m - bk - 8;
    if (mrest > 0 && variant == EIG_ORTHO_CHOLQR_SPLIT)
    {
      // orthonormalize_avx2_b8 (kernels_avx2.hh:255-381): columns 0-3 of Q_bk first, then 4-7
      // against the updated later blocks.  Each half is the full 8 x mrest Gram with the other
      // half's rows zeroed: those add 0 * q_k, which leaves every entry exactly as it was.
      for (int h = 0; h < 2; ++h)
      {
        gram_device(ctx, n, 8, mrest, Qb, Qb + 8 * n, Sg);
        EIG_HIP(hipMemsetAsync(Sg + (h ? 0 : 4 * mrest), 0, (size_t)4 * mrest * sizeof(double), s));
        launch_project(n, mrest, Qb, Qb + 8 * n, Sg, s);
      }
    }
    else if (mrest > 0)
    {
      gram_device(ctx, n, 8, mrest, Qb, Qb + 8 * n, Sg);
      launch_project(n, mrest, Qb, Qb + 8 * n, Sg, s);
    }
  }
}
}  // namespace eigmi

extern "C" int eig_gram_mv8(eig_ctx_t ctx, int64_t n, int64_t m1, int64_t m2, const double *Q1, const double *Q2,
                            double *G)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && Q1 && Q2 && G && n >= 0, EIG_ERR_ARG, "eig_gram_mv8: bad argument");
    EIG_MV8_CHECK(m1);
    EIG_MV8_CHECK(m2);
    DeviceGuard dg(ctx->device);
    if (m1 > 0 && m2 > 0) gram_device(ctx, n, m1, m2, Q1, Q2, G);
  });
}

extern "C" int eig_orthonormalize_mv8(eig_ctx_t ctx, int64_t n, int64_t m, double *Q, int variant)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && Q && n >= 0, EIG_ERR_ARG, "eig_orthonormalize_mv8: bad argument");
    const int v = variant & 0xff;
    EIG_CHECK(v == EIG_ORTHO_MGS || v == EIG_ORTHO_CHOLQR || v == EIG_ORTHO_CHOLQR_SPLIT, EIG_ERR_ARG,
              "unknown variant");
    EIG_CHECK((variant & ~(0xff | EIG_ORTHO_GRID | EIG_ORTHO_NO_COOP | EIG_ORTHO_ONE_WG | (15 << EIG_ORTHO_LOOKAHEAD_SHIFT))) == 0 &&
                  ((variant >> EIG_ORTHO_LOOKAHEAD_SHIFT) & 15) <= 8,
              EIG_ERR_ARG, "unknown variant flags");
    EIG_MV8_CHECK(m);
    DeviceGuard dg(ctx->device);
    orthonormalize_device(ctx, n, m, Q, variant);
  });
}

extern "C" int eig_orthonormalize_gram_mv8(eig_ctx_t ctx, int64_t n, int64_t m, double *Q, const double *gram)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && Q && gram && n >= 0, EIG_ERR_ARG, "eig_orthonormalize_gram_mv8: bad argument");
    EIG_MV8_CHECK(m);
    DeviceGuard dg(ctx->device);
    orthonormalize_device(ctx, n, m, Q, EIG_ORTHO_MGS, gram);
  });
}

extern "C" int eig_spmm_dot_gram_mv8(eig_mat_t mat, int64_t m, const double *Qin, double *Qout, double *dp,
                                     double *gram)
{
  return guard(mat ? mat->ctx : nullptr, [&] {
    EIG_CHECK(mat && Qin && Qout && dp && gram, EIG_ERR_ARG, "eig_spmm_dot_gram_mv8: bad argument");
    EIG_CHECK(m == 8, EIG_ERR_SHAPE, "eig_spmm_dot_gram_mv8: one 8-column block (m = 8)");
    EIG_CHECK(mat->br == 1 && mat->bc == 1, EIG_ERR_BLOCKSIZE,
              "matmul_sparse_tallskinny_blocked: only implemented for FieldMatrix<..,1,1>");
    DeviceGuard dg(mat->ctx->device);
    spmm_dot_gram_device(*mat, Qin, Qout, dp, gram);
  });
}

extern "C" int eig_orthonormalize_passes(eig_ctx_t ctx, int *passes)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && passes, EIG_ERR_ARG, "eig_orthonormalize_passes: null argument");
    DeviceGuard dg(ctx->device);
    *passes = mgs_lookahead_passes(ctx);
  });
}

extern "C" int eig_orthonormalize_naive(eig_ctx_t ctx, int64_t n, int64_t m, double *Q)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && Q && n >= 0 && m >= 0, EIG_ERR_ARG, "eig_orthonormalize_naive: bad argument");
    EIG_CHECK(m <= 512, EIG_ERR_ARG, "eig_orthonormalize_naive: at most 512 columns");
    DeviceGuard dg(ctx->device);
    hipStream_t s = ctx->stream;
    double *d = (double *)ctx_buffer(ctx, 6, (size_t)(m + 1) * sizeof(double));
    // kernels_cpp.hh:128-154: normalise q_k, then q_j -= (q_k . q_j) q_k for every j > k.
    for (i64 k = 0; k < m; ++k)
    {
      double *qk = Q + k * n;
      launch_nrm2sq(n, qk, d + m, 0, s, ctx->red);
      allreduce_sum(ctx, d + m, 1, s);
      launch_scal_dev(n, d + m, true, qk, s);
      const i64 rest = m - k - 1;
      for (i64 j0 = 0; j0 < rest; j0 += 8 * 48)
      {
        const int kk = (int)std::min<i64>(rest - j0, 8 * 48);
        launch_gemv_t(n, kk, Q + (k + 1 + j0) * n, n, qk, d + j0, 0, s, ctx->red);
      }
      allreduce_sum(ctx, d, rest, s);
      // q_j -= d_j q_k : rank-1 update, one axpy per column (same rounding as the reference)
      for (i64 j = 0; j < rest; ++j) launch_axpy_dev(n, d + j, -1.0, qk, Q + (k + 1 + j) * n, s);
    }
  });
}

namespace eigmi {
// B_orthonormalize_blocked (kernels_cpp.hh:356-591) on the device; *norm (device) receives the
// max off-diagonal R coefficient.
void b_orthonormalize_device(eig_mat_s &B, i64 m, double *Q, double *norm)
{
  eig_ctx_t ctx = B.ctx;
  hipStream_t s = ctx->stream;
  const i64 n = B.nb_rows;
  double *P = (double *)ctx_buffer(ctx, 7, (size_t)n * 8 * sizeof(double));
  double *G = (double *)ctx_buffer(ctx, 3, 64 * sizeof(double));
  double *U = (double *)ctx_buffer(ctx, 4, 64 * sizeof(double));
  double *Sg = m > 8 ? (double *)ctx_buffer(ctx, 5, (size_t)8 * m * sizeof(double)) : nullptr;
  EIG_HIP(hipMemsetAsync(norm, 0, sizeof(double), s));
  for (i64 bk = 0; bk < m; bk += 8)
  {
    double *Qb = Q + bk * n;
    launch_spmm_mv8(B, 8, Qb, P, s);                   // P = B Q_bk          (:378-395)
    gram_device(ctx, n, 8, 8, P, Qb, G);               // s = P^T Q_bk        (:450-456)
    launch_cholqr_factor(G, U, norm, 1, s);            // mirror upper, norm, U (:457-526)
    launch_apply_upper(n, Qb, U, s);                   // Q_bk := Q_bk U      (:528-539)
    launch_apply_upper(n, P, U, s);                    // P := P U            (:540-552)
    const i64 mrest = m - bk - 8;
    if (mrest > 0)
    {
      gram_device(ctx, n, 8, mrest, P, Qb + 8 * n, Sg);  // S = P^T Q_bj     (:559-565)
      launch_max_offdiag(Sg, 8, mrest, false, norm, s);  // norm (:566-568)
      launch_project(n, mrest, Qb, Qb + 8 * n, Sg, s);   // Q_bj -= Q_bk S   (:570-584)
    }
  }
}
}  // namespace eigmi

extern "C" int eig_b_orthonormalize_mv8(eig_mat_t B, int64_t m, double *Q, double *norm)
{
  return guard(B ? B->ctx : nullptr, [&] {
    EIG_CHECK(B && Q && norm, EIG_ERR_ARG, "eig_b_orthonormalize_mv8: null argument");
    EIG_CHECK(B->br == 1 && B->bc == 1, EIG_ERR_BLOCKSIZE,
              "B_orthonormalize_blocked: only implemented for FieldMatrix<..,1,1>");
    EIG_MV8_CHECK(m);
    EIG_CHECK(!B->ctx->distributed(), EIG_ERR_ARG, "eig_b_orthonormalize_mv8: single rank only");
    DeviceGuard dg(B->ctx->device);
    b_orthonormalize_device(*B, m, Q, norm);
  });
}

extern "C" int eig_random_mv8(eig_ctx_t ctx, int64_t n, int64_t m, unsigned seed, double *Q)
{
  return guard(ctx, [&] {
    EIG_CHECK(ctx && Q && n >= 0, EIG_ERR_ARG, "eig_random_mv8: bad argument");
    EIG_MV8_CHECK(m);
    DeviceGuard dg(ctx->device);
    std::vector<double> h((size_t)(n * m));
    // (block, row, col) fill order == the flat block-column-major order
    host_random_normal(n * m, seed, h.data());
    EIG_HIP(hipMemcpyAsync(Q, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    EIG_HIP(hipStreamSynchronize(ctx->stream));
  });
}

extern "C" double eig_flops_orthonormalize(int64_t n, int64_t m)
{
  // kernels_cpp.hh:98-106
  double f = 0.0;
  for (i64 k = m; k > 0; k--) f += 2.0 * n + n + (k - 1) * 4.0 * n;
  return f;
}

extern "C" double eig_bytes_orthonormalize_blocked(int64_t n, int64_t m, int b)
{
  // kernels_cpp.hh:157-175
  double c = 0.0;
  for (i64 bk = 0; bk < m; bk += b)
  {
    for (int k = b; k > 0; k--) c += (double)n * k + (double)n * (1 + (k - 1) + 1);
    for (i64 bj = bk + b; bj < m; bj += b) c += 5.0 * b * n;
  }
  return c * 8;
}

// ============================================================================================
// partition planning (host only)
// ============================================================================================
extern "C" int eig_plan_window(int64_t row_begin, int64_t nb_local, int bc, const int64_t *rowptr,
                               const int32_t *col, int64_t out[5])
{
  if (!rowptr || !out || nb_local < 0 || row_begin < 0 || bc < 1) return EIG_ERR_ARG;
  if (rowptr[nb_local] > 0 && !col) return EIG_ERR_ARG;
  i64 cmin = row_begin, cmax = row_begin + nb_local;  // [cmin, cmax) in block columns
  for (i64 p = 0; p < rowptr[nb_local]; ++p)
  {
    cmin = std::min<i64>(cmin, col[p]);
    cmax = std::max<i64>(cmax, (i64)col[p] + 1);
  }
  const i64 lo = row_begin - cmin;
  const i64 pad = (8 - lo % 8) % 8;  // (lo + pad) * bc is a multiple of 8 scalar entries
  const i64 wb = cmin - pad;
  i64 wlen = (cmax - wb) * bc;
  wlen = (wlen + 7) / 8 * 8;
  out[0] = wb;
  out[1] = wlen;
  out[2] = (row_begin - wb) * bc;
  out[3] = cmin;
  out[4] = cmax;
  return EIG_OK;
}

extern "C" int eig_plan_halo(int nranks, int me, const int64_t *ranks, int bc, int64_t wb_blk, int64_t *recv,
                             int *nrecv, int64_t *send, int *nsend)
{
  if (!ranks || !recv || !send || !nrecv || !nsend || nranks < 1 || me < 0 || me >= nranks) return EIG_ERR_ARG;
  const i64 rb0 = ranks[4 * me], nl = ranks[4 * me + 1], cmin = ranks[4 * me + 2], cmax = ranks[4 * me + 3];
  int nr = 0, ns = 0;
  for (int q = 0; q < nranks; ++q)
  {
    if (q == me) continue;
    const i64 qb = ranks[4 * q], qe = ranks[4 * q] + ranks[4 * q + 1];
    // receive from q: q's rows inside my window
    const i64 rb = std::max(qb, cmin), re = std::min(qe, cmax);
    if (re > rb)
    {
      recv[3 * nr] = q;
      recv[3 * nr + 1] = (rb - wb_blk) * bc;
      recv[3 * nr + 2] = (re - rb) * bc;
      ++nr;
    }
    // send to q: my rows inside q's referenced range
    const i64 qwb = ranks[4 * q + 2], qwe = ranks[4 * q + 3];
    const i64 sb = std::max(rb0, qwb), se = std::min(rb0 + nl, qwe);
    if (se > sb)
    {
      send[3 * ns] = q;
      send[3 * ns + 1] = (sb - wb_blk) * bc;
      send[3 * ns + 2] = (se - sb) * bc;
      ++ns;
    }
  }
  *nrecv = nr;
  *nsend = ns;
  return EIG_OK;
}
