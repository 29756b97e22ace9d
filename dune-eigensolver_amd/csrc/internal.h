// internal.h -- shared host-side structures of libeigmi (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <complex>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <memory>
#include <vector>

#include "../../include/eigmi.h"

namespace eigmi {

typedef int64_t i64;
typedef int32_t i32;
typedef uint64_t u64;

// Status-carrying exception used inside the library; every C entry point catches it and turns
// it into the int status + eig_last_error message.
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define EIG_HIP(call)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (call);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      throw ::eigmi::Error(EIG_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));     \
  } while (0)

#define EIG_NCCL(call)                                                                         \
  do {                                                                                         \
    ncclResult_t r_ = (call);                                                                  \
    if (r_ != ncclSuccess)                                                                     \
      throw ::eigmi::Error(EIG_ERR_RCCL, std::string(#call) + ": " + ncclGetErrorString(r_));  \
  } while (0)

#define EIG_CHECK(cond, code, msg)                                                             \
  do {                                                                                         \
    if (!(cond)) throw ::eigmi::Error((code), (msg));                                          \
  } while (0)

// Streaming kernels use this many workgroups (8 per CU x 256 CUs) and grid-stride inside.
constexpr int kStreamBlocks = 2048;
constexpr int kStreamThreads = 256;
// Reduction workspace: per-block partials (sc1 stores) + one ticket per concurrent reduction.
constexpr int kMaxRedBlocks = 2048;
constexpr int kMaxRedVals = 256;   // values reduced by one launch (e.g. a 16x16 Gram tile)
constexpr int kNumTickets = 64;
constexpr int kSymMaxOff = 32;   // offsets of the symmetric band image (eig_mat_s::sym_*)
// One logical ticket = 8 shard counters (workgroup id mod 8, i.e. one per XCD group) + 1 top
// counter, each on its own 128-B line: a single contended word serialises at ~88 agent atomics
// per microsecond (MI355X_MICROARCH price list, row "dequeue"), i.e. ~23 us for 2048 workgroups.
constexpr int kTicketLine = 32;                 // unsigned words per 128-B line
constexpr int kTicketStride = 9 * kTicketLine;  // words per logical ticket

struct ReduceWS {
  double *partials = nullptr;  // kMaxRedBlocks * kMaxRedVals
  unsigned *tickets = nullptr; // kNumTickets * kTicketStride, zero between launches (last block resets)
  unsigned *ticket(int t) const { return tickets + (size_t)t * kTicketStride; }
};

// In-process loopback transport: P virtual ranks (one host thread + context each, usually on the
// same device) exchange through this hub instead of RCCL.  Test-only path for the distributed
// code on a single GPU; every operation is synchronous.
struct LoopHub {
  int P = 1;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  unsigned long gen = 0;
  std::vector<double *> xptr;      // per rank: vector being exchanged
  std::vector<i64> win_begin;      // per rank: window begin (scalar)
  std::vector<std::vector<double>> red;
  std::vector<i64> gather;
  std::vector<u64 *> mbox;                 // per rank: its mailbox (eig_comm_loopback_mailbox)
  std::vector<int> flag;                   // per rank: a flag agreed through the hub
  void barrier()
  {
    std::unique_lock<std::mutex> lk(m);
    const unsigned long g = gen;
    if (++arrived == P)
    {
      arrived = 0;
      ++gen;
      cv.notify_all();
    }
    else
      cv.wait(lk, [&] { return gen != g; });
  }
};

// xGMI mailbox allreduce (k_comm.hip): each rank's uncached mailbox, IPC-mapped by every peer.
constexpr int kMaxMailboxRanks = 16;
constexpr int kMailboxVals = 63;  // values per call (slot = 1 sequence word + 63 values = 512 B)
constexpr int kXchWords = 4;       // step region slot (xch_dev.h): sequence number + 3 sums
struct Mailbox {
  u64 *local = nullptr;                  // my mailbox: [2][P][1 + kMailboxVals], then the step region
  u64 *peer[kMaxMailboxRanks] = {};      // peer[r] = rank r's mailbox mapped here (peer[me] = local)
  u64 *ctr = nullptr;                    // device: sequence number of the last completed call
  u64 *fctr = nullptr;                   // device: sequence number of the last fused-step exchange
  int *err = nullptr;                    // device: set when a call timed out
  long long foff = 0;                    // word offset of the step region [2][P][kXchWords] (xch_dev.h)
  int P = 1, me = 0;
};
// Host-side ownership of the mailbox resources of a context.
struct MailboxHost {
  Mailbox dev;
  u64 *local = nullptr;          // hipExtMallocWithFlags allocation (exported)
  size_t bytes = 0;              // its size
  void *state = nullptr;         // ctr + fctr + err (hipMalloc, 256 B)
  std::vector<void *> opened;    // IPC-opened peer mappings (closed on destroy)
  bool ready = false;            // peers opened and validated: allreduce_sum uses it
  bool on = true;                // eig_comm_select_allreduce: false = ncclAllReduce although ready
  bool step = false;             // EIG_AR_MAILBOX_STEP: the fused step exchanges its sums in-kernel
};
constexpr unsigned long long kMailboxTimeout = 1000000000ull;  // 10 s of s_memrealtime (100 MHz)
void launch_mailbox_allreduce(double *buf, int count, const Mailbox &mb, unsigned long long timeout, hipStream_t s);

// xGMI halo mailbox (k_comm.hip) of mailbox-only ranks (eig_comm_ipc_open, no RCCL): every rank's
// uncached staging area, IPC-mapped by every peer.  Layout: [2][P] sequence lines (one 128-B line
// per word), then [2][P][cap] doubles; parity = sequence & 1, slot = the sending rank.
constexpr int kHaloFlagStride = 16;  // u64 words per sequence line
struct HaloBox {
  u64 *flags = nullptr;                         // mine: [2][P] lines
  u64 *peer_flags[kMaxMailboxRanks] = {};       // rank r's lines mapped here (peer_flags[me] = flags)
  double *stage = nullptr;                      // mine: [2][P][cap]
  double *peer_stage[kMaxMailboxRanks] = {};
  u64 *seq = nullptr;                           // device: [P] exchanges completed with each peer
  unsigned *ticket = nullptr;                   // device: push / pull last-workgroup tickets (128 B apart)
  int *err = nullptr;                           // the mailbox's error word (Mailbox::err)
  long long cap = 0;                            // doubles per slot
  int P = 1, me = 0;
};
struct HaloBoxHost {
  HaloBox dev;
  void *alloc = nullptr;         // hipExtMallocWithFlags allocation (exported)
  void *state = nullptr;         // seq + tickets (hipMalloc, 512 B)
  std::vector<void *> opened;    // IPC-opened peer mappings
};
// One side of an exchange: n ranges (peer, window offset, count) in scalar units.
struct HaloXfer {
  int n = 0;
  int peer[kMaxMailboxRanks] = {};
  long long off[kMaxMailboxRanks] = {};
  long long cnt[kMaxMailboxRanks] = {};
};
void launch_halo_mailbox(const HaloBox &hb, const HaloXfer &snd, const HaloXfer &rcv, const HaloXfer &sync, double *x,
                         double *x2, int width, hipStream_t s);

}  // namespace eigmi

struct eig_mg_s;  // mg.cpp

struct eig_ctx_s {
  int device = 0;
  hipStream_t stream = nullptr;      // compute stream
  hipStream_t comm_stream = nullptr; // halo exchange stream
  hipStream_t red_stream = nullptr;  // allreduce stream of the pipelined Lanczos step (drivers.cpp)
  std::string last_error;
  eigmi::ReduceWS red;
  double *scratch = nullptr;         // small device scalars (reduction results)
  int num_cu = 256;
  // RCCL
  ncclComm_t comm = nullptr;
  // split of `comm` for the pipelined step's allreduce on red_stream, concurrent with the halo
  // exchange on comm_stream (two streams never share a communicator); nullptr: no overlap
  ncclComm_t comm_red = nullptr;
  eigmi::LoopHub *loop = nullptr;    // in-process loopback transport (tests), exclusive with comm
  eigmi::MailboxHost *mbox = nullptr; // xGMI mailbox allreduce (with RCCL, or alone for tests)
  eigmi::HaloBoxHost *hbox = nullptr; // xGMI halo mailbox of mailbox-only ranks (grown by eig_mat_create_bcsr_dist)
  int nranks = 1, rank = 0;
  long long n_ar = 0, n_ar_red = 0, n_halo = 0, n_p2p = 0;  // eig_comm_counters
  bool comm_always = false;          // EIG_COMM_ALWAYS: collectives through `comm` even at one rank
  bool halo_mailbox = false;         // eig_comm_select_halo(EIG_HALO_MAILBOX) beside RCCL
  bool distributed() const { return nranks > 1 && (comm || loop || (mbox && mbox->ready)); }
  // whether allreduces go through a transport (distributed, or a forced one-rank RCCL communicator)
  bool collectives() const { return distributed() || (comm_always && (comm || (mbox && mbox->ready))); }
  // the fused Lanczos step exchanges its three sums inside the step kernel (EIG_AR_MAILBOX_STEP)
  bool step_exchange() const { return collectives() && mbox && mbox->ready && mbox->on && mbox->step; }
  // reusable device buffers for drivers (grown on demand)
  std::vector<std::pair<void *, size_t>> pool;
  // a look-ahead MGS last launch (grid barriers without a cooperative launch) has been enqueued
  // since the last mgs_lookahead_check: its sticky error word must be read at the next sync point
  bool mgs_la_armed = false;
  // its sticky error word in page-locked, device-mapped host memory: the kernel stores into it, the
  // host reads it after any stream synchronisation without a copy (allocated at first use)
  int *mgs_err_host = nullptr, *mgs_err_dev = nullptr;
  // the window Gram whose product also zeroed the look-ahead MGS's barrier word (launch_spmm_dot_gram_mv8);
  // consumed by the next launch_mgs_lookahead_gram of that Gram
  const double *mgs_bar_clean = nullptr;
};

namespace eigmi {

// Halo plan of a row-partitioned matrix (scalar units): the window covers global scalar
// columns [win_begin, win_begin + window); owned rows sit at own_offset.  For every peer,
// `sends` lists owned ranges it needs and `recvs` the window ranges it fills.
struct HaloRange {
  int peer;
  i64 offset;  // scalar offset inside the window (recv) or inside the window (send: own rows)
  i64 count;   // scalar entries
};

}  // namespace eigmi

struct eig_mat_s {
  eig_ctx_t ctx = nullptr;
  int br = 1, bc = 1;
  eigmi::i64 nb_rows = 0;         // owned block rows
  eigmi::i64 nb_rows_global = 0;
  eigmi::i64 nb_cols = 0;         // global block columns
  eigmi::i64 row_begin = 0;       // first owned global block row
  eigmi::i64 win_begin = 0;       // first global scalar column in the window
  eigmi::i64 window = 0;          // window length (scalar)
  eigmi::i64 own_offset = 0;      // owned rows' offset in the window (scalar)
  eigmi::i64 nnzb = 0, nnzb_padded = 0;
  eigmi::i64 nslices = 0;
  // SELL-C device image, C = 64 R: slice s covers block rows [C s, C s + C); entry k of slice row
  // r sits at slice_ptr[s] + k*C + r (cols) and (slice_ptr[s] + k*C)*br*bc + t*C + r (values,
  // t < br*bc).  Lane l of the slice's wavefront owns rows l R .. l R + R - 1.  R = 1 for blocks.
  int R = 1;
  // kernel-image policy fixed at creation (eig_mat_create_bcsr_ex flags: EIG_MAT_NO_BAND,
  // EIG_MAT_BAND_GATHER, EIG_MAT_NO_STENCIL, EIG_MAT_NO_MARCH)
  int kflags = 0;
  // Stencil slices (1x1 blocks only): when every row of slice s draws its columns from one set of
  // at most 8 offsets delta = global col - global row (structured-grid / banded matrices), the
  // slice is read through st_delta[8 s + k] (ascending) and a per-row bit mask st_mask[r] (bit k
  // = row r stores the entry at delta_k) instead of the per-entry columns: 1 B per row instead of
  // 4 B per entry.  st_width[s] = number of offsets, or -1 for an explicit-column slice.  Entries
  // keep their ascending-column order, so results stay bitwise identical.
  eigmi::i32 *st_width = nullptr;   // nslices
  eigmi::i32 *st_delta = nullptr;   // 8 * nslices
  uint8_t *st_mask = nullptr;       // nslices * C
  eigmi::i64 n_stencil_slices = 0;
  // Symmetric band image (1x1 blocks, R = 1; api.cpp build_sym): when every row draws its columns
  // from one global set of at most kSymMaxOff offsets d = col - row and every stored pair
  // (r, r+d) / (r+d, r) is bitwise equal, the values live once, in nup = |{|d|}| window-indexed
  // arrays: sym_val[j * sym_ld + x] = a(x, x + p_j) = a(x + p_j, x) for the j-th non-negative
  // offset p_j.  Row w reads offset d >= 0 at [j(d)][w] and d < 0 at [j(-d)][w + d] (the mirrored
  // upper entry); the per-row mask (bit k = row stores off[k], u8 when nd <= 8, else u32) gates
  // the accumulation, so each row still sums exactly its own entries in ascending-column order.
  // The SELL image above stays (SpMM, block and download paths use it).
  double *sym_val = nullptr;
  void *sym_mask = nullptr;         // nslices * 64 entries of sym_mask_bytes
  int sym_mask_bytes = 0;
  int sym_nd = 0, sym_nup = 0;
  eigmi::i64 sym_ld = 0;
  eigmi::i32 sym_off[eigmi::kSymMaxOff] = {};      // ascending offsets (ISTL column order)
  eigmi::i32 sym_dj[eigmi::kSymMaxOff] = {};       // array index of |sym_off[k]|
  // Uniform band (constant-coefficient stencils): every stored entry of band array j has the value
  // sym_uc[j] bit for bit, so the plane-march kernels take the values from their arguments and
  // stream the row mask and the vectors only (the arrays stay for the other kernels)
  bool sym_uniform = false;
  double sym_uc[eigmi::kSymMaxOff] = {};
  // Geometric row masks (a property of the pattern; one rank's whole grid or a slab of whole
  // planes): the rows form an nx x ny x nz grid (offsets -D, -nx, -1, 0, 1, nx, D with D = nx ny, or
  // the 2-D -D, -1, 0, 1, D with D = nx) and every row stores exactly its in-grid neighbours; the
  // march derives the masks from the coordinates (uniform bands: values from the arguments; other
  // bands: the value march streams the band arrays, k_spmv.hip march variant 10)
  bool sym_geo = false;
  int sym_gx = 0, sym_gy = 0, sym_gz = 0, sym_gz0 = 0;  // grid (global planes) and this rank's first plane
  // Box-geometric masks (api.cpp build_sym): offsets inside the 27-point box a D + b nx + c (a, b, c in
  // {-1, 0, 1}) of an nx x ny x nz grid, every row storing exactly its in-grid neighbours among them
  // (sym_geo's 5 / 7-point grids excluded); sym_box27 = bit (a + 1) 9 + (b + 1) 3 + (c + 1) per stored
  // offset; grid in sym_gx / gy / gz / gz0.  The box marches (k_spmv.hip, e.g. the P1 Kuhn 15-point
  // stencil of config C5) derive the masks from the coordinates
  unsigned sym_box27 = 0;
  // packed copy of the 4 value arrays of a 7-point band ({+D, 0, +1, +nx} per row, 32 B; the P1 Kuhn
  // band: 8 arrays, 64 B) for the value marches 15 / 16 / 18 / 19 (k_spmv.hip sym_pack_prepare: built
  // at the first launch that marches on it, never by a query; refilled in place by a shift)
  double *sym_pack = nullptr;
  eigmi::i64 sym_pack_bytes = 0;
  // SELL image: padded entries of the explicit-column slices (their 4-B column indices are streamed)
  eigmi::i64 sell_explicit = 0;
  // Plane-march split of a distributed slab (k_spmv.hip march_plan): planes [mz0, mz1) have no
  // ghost columns and are marched while the halo is in flight; march_bnd lists every slice outside
  // them (the boundary launch after the exchange).  mz1 <= mz0: no split.
  eigmi::i64 mz0 = 0, mz1 = 0;
  int tune_march_runs = 0;  // eig_mat_tune(EIG_TUNE_MARCH_RUNS): plane runs per column, 0 = automatic
  int tune_halo_whole = 0;      // eig_mat_tune(EIG_TUNE_HALO): 1 = exchange first, then one whole launch
  int tune_march_prefetch = 0;  // eig_mat_tune(EIG_TUNE_MARCH_PREFETCH): geometric march variant, 0 = automatic
  int tune_cache = 0;           // eig_mat_tune(EIG_TUNE_CACHE): cache-policy bits of the march streams (measurement)
  int tune_box_cols = 0;    // eig_mat_tune(EIG_TUNE_BOX_COLS): columns per box-image workgroup (16 / 32), 0 = automatic
  int tune_box_map = 0;     // eig_mat_tune(EIG_TUNE_BOX_MAP): 1 = XCD-contiguous tile map of k_box_mv32 (measurement)
  int tune_sell_cpf = 2;    // eig_mat_tune(EIG_TUNE_SELL_CPF): explicit slices' column prefetch, 2 = automatic
  int tune_march_lines = 0; // eig_mat_tune(EIG_TUNE_MARCH_LINES): 4 = line-group mapping of the value march
  int tune_box_segs = 0;    // eig_mat_tune(EIG_TUNE_BOX_SEGS): z segments per box tile column, 0 = automatic
  // Box-stencil image for the 32-column SpMM / Chebyshev kernel (k_box.hip): box_state 0 = not
  // examined yet, 1 = built, -1 = the band is not a 3-D box stencil; box_val[k n + r] = the entry of
  // row r at sym_off[k]; grid nx x ny x nz; per offset its plane step and halo-tile row shift
  int box_state = 0;
  double *box_val = nullptr;
  int box_nx = 0, box_ny = 0, box_nz = 0;
  // a rank's slab of whole planes (distributed contexts): ghost planes below / above the owned ones
  // in the window (0 or 1 each; the owned rows start at own_offset = box_glo planes)
  int box_glo = 0, box_ghi = 0;
  int box_dz[27] = {}, box_dxy[27] = {}, box_dx[27] = {}, box_dy[27] = {};
  // Row classes (k_box.hip k_boxc_mv8): when every row's stored entries equal those of its
  // geometric class representative (27 classes: first / interior / last position in x, y and z),
  // box_ctab holds per class the nd values and 1 / a_rr (slot 15), box_cmask the row mask, and the
  // class kernels read no matrix stream at all (box_val is then freed)
  double *box_ctab = nullptr;
  unsigned *box_cmask = nullptr;
  // every offset a row does not store points out of the grid (its halo row is 0): the kernels with
  // a compile-time stencil then sum all offsets with the zero image / class entries, no masks
  bool box_geomask = false;
  eigmi::i32 *march_bnd = nullptr;
  eigmi::i64 n_march_bnd = 0;
  eigmi::i64 *slice_ptr = nullptr;  // nslices + 1
  eigmi::i32 *col = nullptr;        // nnzb_padded, window-local block columns, -1 = padding
  double *val = nullptr;            // nnzb_padded * br * bc
  // Interior / boundary slice split for halo overlap (distributed only).
  eigmi::i32 *slice_list = nullptr; // [interior..., boundary...]
  eigmi::i64 n_interior = 0, n_boundary = 0;
  std::vector<eigmi::HaloRange> sends, recvs;
  eigmi::i64 halo_send = 0, halo_recv = 0;
  eigmi::i64 device_bytes = 0;
  // max |global col - global row| over the stored blocks (block units): the far-neighbour distance
  // the XCD-aware gather kernels size their grid by (k_block.hip)
  eigmi::i64 bandwidth = 0;
  // sum of the stored diagonal entries of the owned rows (trace share; shift_diag keeps it current)
  // and how many rows store one: the fused Lanczos step's shift mu = trace / n
  double diag_sum = 0.0;
  eigmi::i64 diag_count = 0;
};

namespace eigmi {

// ---- kernel launchers (k_*.hip) -------------------------------------------------------------
// Scalar results land in `out` (device); reductions use ctx->red.

// SpMV over the SELL image: y[own_offset + r] = (A x)[r] for the slices [first, first+count) of
// `slices` (or all slices when slices == nullptr).
void launch_spmv(const eig_mat_s &A, const double *x, double *y, const i32 *slices, i64 first, i64 count,
                 hipStream_t s, bool keep = false);

// Lanczos fused kernels (see DESIGN.md "Lanczos step").  Device scalar arrays live in `st`.
struct LanczosState {
  double *dsum;   // dsum[j]  = t . u_j (local, then allreduced)
  double *nsum;   // nsum[j]  = ||u_j||^2 (local, then allreduced); nsum[0] from the start vector
  double *alpha;  // alpha[j]
  double *beta;   // beta[j]  = sqrt(nsum[j])
  // fused step (k_spmv.hip "Fused one-reduction Lanczos step"), indexed by LAUNCH L (a repair is a
  // launch that is not a step):
  double *fred;   // fred[3L..3L+2] = (t . u, t . t, u . u) of launch L (local, then allreduced)
  int *ctl;       // ctl[2L], ctl[2L+1] = logical step and mode at the start of launch L
  double *aux;    // aux[2L], aux[2L+1] = (rn, rm) a repair hands to launch L
  double *mu2;    // (sum of the diagonal, rows), allreduced: the step's shift mu = mu2[0] / mu2[1]
  double *pn;     // pn[L] = nsum[j - 1] for launch L at step j (written by launch L - 1), so a launch's
                  // prologue loads are independent of each other (one memory round trip)
};
enum { kFusedModeStep = 0, kFusedModePost = 1, kFusedModeHalt = 2 };  // ctl[2L + 1]
struct FusedLaunch {
  LanczosState st;
  int L;        // launch index
  int force;    // repair regardless of the prediction (exact final beta, eig_lanczos_tridiag)
  int xch = 0;  // kXchPublish: the sums allreduced inside the kernel (EIG_AR_MAILBOX_STEP, xch_dev.h)
};
enum { kXchPublish = 2 };
// P, Pout: interleaved (t, u) pair vectors in window layout (2 doubles per row).
void launch_lanczos_fused(const eig_mat_s &A, const double *P, double *Pout, const FusedLaunch &fl,
                          const i32 *slices, i64 first, i64 count, const double *carry, double *out, int ticket,
                          hipStream_t s, ReduceWS red);
// Pipelined step, row half (k_lanczos_pipe): T = t (window layout, updated in place), UZ = (u, z)
// pairs (window layout, 2 doubles per row), S = A t of this launch (window layout); the three sums
// of launch fl.L to `out`.
void launch_lanczos_pipe(const eig_mat_s &A, double *T, double *UZ, const double *S, const FusedLaunch &fl,
                         double *out, hipStream_t s, ReduceWS red);
// beta / nsum of the current logical step after a repair launch (L = the next launch index)
void launch_fused_tail(const LanczosState &st, int L, hipStream_t s);
// Plane march (k_spmv.hip): band geometry (widest offset D) and whether the interior-plane split
// launch applies now (split built at upload, image and EIGMI_* switches allow it).  Passing
// slices == &kMarchInteriorTag to launch_spmv / launch_lanczos_spmv / launch_lanczos_fused marches
// planes [A.mz0, A.mz1).
bool march_geometry(const eig_mat_s &A, i64 &D, int chunk = 64);
bool march_split_active(const eig_mat_s &A);
int march_variant(const eig_mat_s &A, bool fused);
extern const i32 kMarchInteriorTag;
// a2 SpMM (kernels_cpp.hh:626-657) on the band-image plane march for 1x1 matrices whose band
// qualifies; false (nothing launched) otherwise.  X, Y: window-layout multivectors, m % 8 == 0.
bool box_prepare(const eig_mat_s &A);
// launch_box_spmm would take this product (row-class image, or the box image at m % 32 == 0)
inline bool box_spmm_applies(const eig_mat_s &A, i64 m)
{
  return m > 0 && m % 8 == 0 && box_prepare(A) && (A.box_ctab != nullptr || m % 32 == 0);
}
int box_cols(const eig_mat_s &A);  // columns per box-image workgroup (k_box_mv32: 32, k_box_mv16p: 16)
bool launch_box_spmm(const eig_mat_s &A, i64 m, const double *X, double *Y, hipStream_t s);
bool launch_box_spmm_dot(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, ReduceWS red,
                         hipStream_t s);
bool launch_box_spmm_dot_gram(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, double *gram,
                              ReduceWS red, hipStream_t s, unsigned *zero_word = nullptr);
bool launch_spmm_march_dot_gram(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, double *gram,
                                ReduceWS red, hipStream_t s, unsigned *zero_word = nullptr);
// the look-ahead MGS state's barrier word of this context (allocated and zeroed on first use)
unsigned *mgs_lookahead_barrier(eig_ctx_t ctx);
// StandardLargest's product: Y = A X, dp = diag(X^T Y) and (gram != null, m = 8) the window Gram of Y
// for the next iteration's MGS; false when no fused kernel applies (then gram is not written).
bool launch_spmm_dot_gram_mv8(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, double *gram,
                              hipStream_t s, ReduceWS red);
bool launch_spmm_march_dot(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, ReduceWS red,
                           hipStream_t s);
// Xnew: x_{k+1} into a third buffer (nullptr: in place over Xold); Xold nullptr (with Xnew): x_{k-1} = 0
bool launch_box_cheb(const eig_mat_s &M, i64 m, const double *Xk, double *Xold, const double *B, const double *dinv,
                     double omega, double gamma, hipStream_t s, double *Xnew = nullptr);
void box_invalidate(eig_mat_s &A);
bool launch_box_resid(const eig_mat_s &A, i64 m, const double *X, const double *B, double *R, hipStream_t s);
bool launch_box_resid_acc(const eig_mat_s &A, i64 m, const double *E, const double *B, double *R, double *Xacc,
                          bool copy, hipStream_t s);
bool launch_box_cheb_first(const eig_mat_s &M, i64 m, const double *B, double omega, double gamma, double *Y,
                           hipStream_t s);
bool launch_box_cheb_first_add(const eig_mat_s &M, i64 m, const double *B, double omega, double gamma, double *Y,
                               hipStream_t s);
bool launch_box_cheb_second(const eig_mat_s &M, i64 m, const double *X2, const double *B, double omega, double gamma,
                            double *Y, hipStream_t s);
// R = B - A X for window-layout multivectors (m % 8 == 0); R may alias B, not X.
void launch_resid_mv8(const eig_mat_s &A, i64 m, const double *X, const double *B, double *R, hipStream_t s);
bool launch_spmm_march(const eig_mat_s &A, i64 m, const double *X, double *Y, hipStream_t s);
// Chebyshev step (k_block.hip kCheb semantics) on the general band march; false when not applicable.
bool launch_cheb_march(const eig_mat_s &M, i64 m, const double *Xk, double *Xold, const double *B, const double *dinv,
                       double omega, double gamma, hipStream_t s);
// Kernel a whole-matrix Lanczos step launch picks on this image, and its algorithmic bytes per launch.
void lanczos_kernel_info(const eig_mat_s &A, bool fused, std::string &name, i64 &bytes);
i64 sell_image_bytes(const eig_mat_s &A);
// Build what a march launch on A streams beside the band arrays (the value pack), ahead of a capture
void march_prepare(const eig_mat_s &A);
// whether the P1 Kuhn value pack (64 B per row) fits the 32-bit buffer descriptor march 16 / 19 read it by
bool kuhn_pack_fits(const eig_mat_s &A);
// The P1 Kuhn march variant of a matrix the Kuhn march applies to (k_spmv.hip march_uniform): 16 / 19
// on the value pack, 12 on the band arrays
int kuhn_variant(const eig_mat_s &A);
// Whether EIG_LANCZOS_AUTO takes the fused step on this image: every 1x1 image (round 3: without
// register spills the fused step beats the two-kernel step on scattered images too).
bool fused_step_pays(const eig_mat_s &A);
// Kernel family a whole-matrix launch of `op` (eig_mat_kernel_info's EIG_OP_*) picks on this image.
std::string kernel_for(const eig_mat_s &A, int op);
void launch_lanczos_spmv(const eig_mat_s &A, const double *u, const double *up, double *t, int j,
                         const LanczosState &st, const i32 *slices, i64 first, i64 count, double *dot_out,
                         double *beta_out, const double *carry, int ticket, hipStream_t s, ReduceWS red);
void launch_lanczos_update(i64 n, const double *u, double *t, int j, const LanczosState &st, int ticket,
                           hipStream_t s, ReduceWS red);
void launch_beta_tail(const LanczosState &st, int j, hipStream_t s);

// BLAS-1 (results to device memory).
void launch_dot(i64 n, const double *x, const double *y, double *out, int ticket, hipStream_t s, ReduceWS red);
void launch_nrm2sq(i64 n, const double *x, double *out, int ticket, hipStream_t s, ReduceWS red);
void launch_lanczos_update_ext(i64 n, const double *alpha, const double *beta, const double *v, const double *p,
                               double *w, double *out, int ticket, hipStream_t s, ReduceWS red);
void launch_axpy(i64 n, double a, const double *x, double *y, hipStream_t s);
void launch_axpy_dev(i64 n, const double *a, double scale, const double *x, double *y, hipStream_t s);
void launch_scal(i64 n, double a, double *x, hipStream_t s);
void launch_fill_normal(i64 n, unsigned seed, double *x, hipStream_t s);  // counter-based N(0, 1)
void launch_stream_copy(i64 n, const double *x, double *y, int num_cu, hipStream_t s, int mode);
void launch_scal_dev(i64 n, const double *a, bool reciprocal_sqrt, double *x, hipStream_t s);
void launch_sqrt_inplace(double *v, int count, hipStream_t s);
void launch_shift_diag(eig_mat_s &A, double shift, hipStream_t s);
// (Re)fill the packed value image sym_pack from the band arrays on stream s (k_spmv.hip)
void sym_pack_fill(eig_mat_s &A, hipStream_t s);

// MultiVector<double,8> kernels.
void launch_spmm_mv8(const eig_mat_s &A, i64 m, const double *Qin, double *Qout, hipStream_t s);
// Y = A X and dp = the diagonal dots X_j . Y_j (StandardLargest's :84-85): one fused launch on the
// row-class image, else the product and k_dot_diag_mv8 (tickets 0 .. m / 8 - 1 of red)
void launch_spmm_dot_mv8(const eig_mat_s &A, i64 m, const double *X, double *Y, double *dp, hipStream_t s,
                         ReduceWS red);
void launch_dot_diag_mv8(i64 n, i64 m, const double *Q1, const double *Q2, double *dp, int ticket,
                         hipStream_t s, ReduceWS red);
void launch_gram_mv8(i64 n, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G, int ticket,
                     hipStream_t s, ReduceWS red);
int gram_mv8_chunks(i64 m1, i64 m2);  // tickets one launch_gram_mv8 takes
// The same Gram on window-layout panels (column blocks ld rows apart, pointers at owned row 0).
void launch_gram_panel(eig_ctx_t ctx, i64 n, i64 ld, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G,
                       hipStream_t s);
// Block Gram-Schmidt building blocks, see k_mv8.hip.
void launch_mgs_pass(i64 n, double *Qb, int k, double *S, int ticket, hipStream_t s, ReduceWS red);
// MGS with Gram look-ahead (k_mv8.hip): L steps per read pass, gated; false when L <= 1 or n <= 0
constexpr int kMgsLookaheadDefault = 8;
int mgs_lookahead_default();  // EIGMI_MGS_LOOKAHEAD or kMgsLookaheadDefault
bool launch_mgs_lookahead(eig_ctx_t ctx, i64 n, double *Qb, int L, bool coop, hipStream_t s);
// The look-ahead MGS of one 8-column block whose window Gram G (8 x 8 row-major, device) is already
// known: the first read pass is replaced by G (k_mgs_la_gram), then the last launch as usual.
bool launch_mgs_lookahead_gram(eig_ctx_t ctx, i64 n, double *Qb, const double *G, hipStream_t s);
int mgs_lookahead_passes(eig_ctx_t ctx);  // read passes of the last call (-1: none finished)
// After the stream is synchronised: throw EIG_ERR_HIP (and clear the sticky flag) when a look-ahead
// MGS last launch since the previous check timed out in its grid barrier (its rows are NaN)
void mgs_lookahead_check(eig_ctx_t ctx);
// Whole column MGS of one 8-column block in one workgroup (n <= 4096, one rank); false = not taken.
bool launch_mgs_small(i64 n, double *Qb, hipStream_t s);
// The 9 read-only MGS passes in one cooperative launch with grid barriers (k_mv8.hip k_mgs_coop; one
// rank); false = refused or timed out (nothing written): run the per-pass launches instead
bool launch_mgs_coop(eig_ctx_t ctx, i64 n, double *Qb, double *Ssum, hipStream_t s);
void launch_apply_upper(i64 n, double *Qb, const double *U, hipStream_t s);
void launch_cholqr_factor(const double *G, double *U, double *normmax, int flags, hipStream_t s);
void launch_project(i64 n, i64 mrest, const double *Qk, double *Qrest, const double *S, hipStream_t s);
void launch_max_offdiag(const double *S, i64 rows, i64 cols, bool upper_only, double *normmax, hipStream_t s);

// Column-major (b = 1) GEMV-type helpers for the Lanczos re-orthogonalisation:
// c = V^T w (V: k columns of length ld, owned slice at off), w -= V c.
// gate (device, nullable): {r, w} squared norms; the launch does nothing unless
// r <= 0.717^2 w -- ARPACK's DGKS test for a second Gram-Schmidt pass (dsaitr: rnorm > 0.717 wnorm
// means the first pass sufficed), evaluated on the device so no step synchronises with the host.
void launch_gemv_t(i64 n, int k, const double *V, i64 ldv, const double *w, double *c, int ticket,
                   hipStream_t s, ReduceWS red, const double *gate = nullptr);
// w -= sum_q V_q * c[q] / (scale2 ? scale2[q] : 1)
void launch_gemv_n_sub(i64 n, int k, const double *V, i64 ldv, const double *c, const double *scale2, double *w,
                       hipStream_t s, const double *gate = nullptr);
// y = sum_q V_q * c[q] / sqrt(nsum[q])   (Ritz vector assembly from an unnormalised basis)
void launch_zero_gated(i64 n, double *w, const double *gate, hipStream_t s);
void launch_gemv_n_set(i64 n, int k, const double *V, i64 ldv, const double *c, const double *nsum, double *y,
                       hipStream_t s);
// r = ||A y - theta y|| helper: out = ||x - theta*y||^2
void launch_resid_sq(i64 n, const double *x, const double *y, double theta, double *out, int ticket,
                     hipStream_t s, ReduceWS red);

// Window-layout multivector kernels (k_block.hip).  m columns (multiple of 8), leading dimension
// = the matrix window, owned rows at own_offset.
void launch_sell_mv8(const eig_mat_s &A, i64 m, const double *X, double *Y, hipStream_t s);
int sell_mv8_launches(i64 m);  // kernel launches per launch_sell_mv8 / launch_cheb_step call
void launch_cheb_step(const eig_mat_s &M, i64 m, const double *Xk, double *Xold, const double *B, const double *dinv,
                      double omega, double gamma, hipStream_t s);
void launch_diag_inv(const eig_mat_s &A, double *dinv, hipStream_t s);
void launch_cheb_init(i64 n, i64 ld, i64 own, i64 m, const double *B, const double *dinv, double gamma, double *X,
                      hipStream_t s);
// G (m1 x m2, row-major, device) = Q1^T Q2 over n rows; Q1, Q2 address owned row 0 (pointer + 8 own).
void launch_panel_gram(eig_ctx_t ctx, i64 n, i64 ld, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G,
                       hipStream_t s);
void launch_panel_gram_2stage(eig_ctx_t ctx, i64 n, i64 ld, i64 m1, i64 m2, const double *Q1, const double *Q2,
                              double *G, hipStream_t s);
// Chebyshev-Jacobi semi-iteration for M X = Bv (degree steps on the spectrum bounds [lmin, lmax]
// of diag(M)^-1 M, from X = 0; blanczos.cpp): returns the buffer (Xa, Xb or Xc) holding x_degree.
double *cheb_solve(eig_mat_s &M, i64 m, int degree, double lmin, double lmax, const double *Bv, const double *dinv,
                   double *Xa, double *Xb, double *Xc, hipStream_t s);
// Geometric multigrid inner solve (mg.cpp): X = S_cycles B on the level-0 matrix's window layout.
void mg_apply(eig_mg_s &mg, i64 m, const double *B, double *X, int cycles);
eig_mat_s *mg_matrix(const eig_mg_s &mg);
int mg_max_cols(const eig_mg_s &mg);
// CholQR2's middle step, b = 32: Z <- Z S, G = (Z S)^T (MZ S) (k_block.hip; partials in context slot 8)
void launch_cholqr_fold(eig_ctx_t ctx, i64 n, i64 ld, double *Z, const double *MZ, const double *S, double *G,
                        hipStream_t s);
void launch_chol_small(int b, int pass, const double *G, double *R, double *Ri, double *Rtot, int *flag,
                       hipStream_t s);
// Y = beta Y + alpha Q S over n rows (owned-row pointers), m2 <= 32.
void launch_panel_update(i64 n, i64 ldq, i64 ldy, i64 m1, i64 m2, const double *Q, const double *S, double alpha,
                         double beta, double *Y, hipStream_t s);

// Exported-LU-factor solves (k_trsv.hip, lu.cpp): device image of the factors.
struct TrsvImage {
  i64 n = 0;
  i64 *lrp = nullptr, *lsplit = nullptr;  // L rows (no unit diagonal), ascending columns
  i32 *lc = nullptr;
  double *lv = nullptr;
  i64 *urp = nullptr, *usplit = nullptr;  // U rows (no diagonal), descending columns
  i32 *uc = nullptr;
  double *uv = nullptr, *ud = nullptr;
  i32 *P = nullptr, *Q = nullptr;
  double *scale = nullptr;                // Rs[P[k]] (do_recip) or 1 / Rs[P[k]]
  void *arena = nullptr;                  // the one allocation holding P, Q, scale
  void *arena_rows = nullptr;             // the one allocation holding lrp .. ud (when `rows`)
  bool rows = false;                      // the row-CSR factors are on the device
  hipStream_t stream = nullptr;           // the owning context's stream (uploads)
  // Block-staged image (k_tsolve_staged, k_trsv.hip), per factor (0 = L, 1 = U) and 64-row block b:
  // the entries outside the block as an ELL slab [k][r] (off1[b] .. + w1[b] * 64; column -1 =
  // padding), the entries inside it as a dense 64 x 64 tile [t][r] (tile + b * 4096) + row masks.
  i64 *off1[2] = {nullptr, nullptr};
  i32 *w1[2] = {nullptr, nullptr};
  double *v1[2] = {nullptr, nullptr};
  i32 *c1[2] = {nullptr, nullptr};
  double *tile[2] = {nullptr, nullptr};
  unsigned long long *tmask[2] = {nullptr, nullptr};
  bool staged = false;  // the factors fit k_tsolve_staged (k_trsv.hip)
  int solver = 0;       // eig_lu_set_solver: EIG_TRSV_AUTO / _BLOCKINV / _STAGED / _CSR
  // the staged image is built on first use (EIG_TRSV_STAGED, or factors without the
  // block-inverse image): host copies of the split factor rows until then
  bool staged_built = false;
  std::shared_ptr<struct TrsvHostRows> host;
  // Block-inverse image (k_binv_z / k_binv_chain, k_trsv.hip), per factor: the inverse of every
  // 64 x 64 diagonal block, dinv + b * 4096 as [t][r], and G(b, d) = inv(D_b) T(b, d) for the
  // coupling T(b, d) of block b to the block d before it (L) / after it (U), g + (b * gd + d - 1) * 4096
  double *dinv[2] = {nullptr, nullptr};
  double *g[2] = {nullptr, nullptr};
  int gd[2] = {0, 0};
  bool binv = false;
};
void trsv_upload_rows(TrsvImage &img, const std::vector<i64> &lrp, const std::vector<i32> &lc,
                      const std::vector<double> &lv, const std::vector<i64> &urp, const std::vector<i32> &uc,
                      const std::vector<double> &uv, const std::vector<double> &ud);
void trsv_upload(eig_ctx_t ctx, i64 n, const std::vector<i64> &lrp, const std::vector<i32> &lc,
                 const std::vector<double> &lv, const std::vector<i64> &urp, const std::vector<i32> &uc,
                 const std::vector<double> &uv, const std::vector<double> &ud, const std::vector<i64> &P,
                 const std::vector<i64> &Q, const std::vector<double> &scale, TrsvImage &img);
void trsv_free(TrsvImage &img);
void trsv_attach_perm(eig_ctx_t ctx, i64 n, const std::vector<i64> &P, const std::vector<i64> &Q,
                      const std::vector<double> &scale, TrsvImage &img);
// Device band LU of B = (R^-1 A)[perm, perm] (k_band.hip) + its block-inverse image in img; the
// band ([b][d + gd] 64 x 64 column-major tiles) is returned in *band_out.  false: a diagonal tile
// failed the conditioning test (img untouched, the band still returned).
bool band_lu_device(eig_ctx_t ctx, i64 n, int gd, const std::vector<i64> &rp, const std::vector<i32> &cj,
                    const std::vector<double> &cv, const std::vector<i32> &inv, const std::vector<double> &rs,
                    TrsvImage &img, double **band_out);
void launch_inverse_mv8(TrsvImage &img, i64 m, double *Qin, double *Qout, hipStream_t s);
void lu_inverse_device(eig_lu_t lu, i64 m, double *Qin, double *Qout, hipStream_t s);
i64 lu_size(eig_lu_t lu);

// ---- dense host linear algebra (dense.cpp) ---------------------------------------------------
void tridiag_eig(int k, std::vector<double> &d, std::vector<double> e, std::vector<double> &Z, bool z_identity = true);
void householder_tridiag(int n, std::vector<double> A, std::vector<double> &d, std::vector<double> &e,
                         std::vector<double> &Q);
void sym_eig(int n, const std::vector<double> &A, std::vector<double> &w, std::vector<double> &Z);
bool chol_upper(int n, const double *G, double *R);
void tri_upper_inv(int n, const double *R, double *Rinv);
// General real n x n matrix g (row-major): eigenvalues w and unit eigenvectors Y (column j of the
// row-major n x n Y belongs to w[j]; conjugate pairs adjacent).  False when the QR iteration
// did not converge.
bool gen_eig(int n, const std::vector<double> &g, std::vector<std::complex<double>> &w,
             std::vector<std::complex<double>> &Y);

// ---- helpers in api.cpp --------------------------------------------------------------------
// Ghost entries of window vector x (and x2 when given) from their owners.
// width: doubles per row of x (2 for the fused step's interleaved pair vectors).
void halo_exchange(const eig_mat_s &A, double *x, hipStream_t s, double *x2 = nullptr, int width = 1);
void mv_device(eig_mat_s &A, double *x, double *y);
void gram_device(eig_ctx_t ctx, i64 n, i64 m1, i64 m2, const double *Q1, const double *Q2, double *G);
// gram0 (or null): the window Gram of the first 8-column block, already summed by the caller's
// product (eig_orthonormalize_gram_mv8; MGS look-ahead on one rank only, else ignored)
void orthonormalize_device(eig_ctx_t ctx, i64 n, i64 m, double *Q, int variant, const double *gram0 = nullptr);
// Y = A X (one 8-column block), dp = diag(X^T Y), gram = Y^T Y (8 x 8): fused into the product where a
// kernel has the epilogue (launch_spmm_dot_gram_mv8), else product + panel Gram
void spmm_dot_gram_device(const eig_mat_s &A, const double *X, double *Y, double *dp, double *gram);
void b_orthonormalize_device(eig_mat_s &B, i64 m, double *Q, double *norm);
// Host CSR copy of a single-rank matrix's device image (rows in ISTL order, padding dropped).
void mat_download_bcsr(const eig_mat_s &A, std::vector<i64> &rowptr, std::vector<i32> &col, std::vector<double> &vals);
void allreduce_sum(eig_ctx_t ctx, double *buf, i64 count, hipStream_t s);
// Whether allreduce_sum_red can run on ctx->red_stream concurrently with the compute and halo
// streams (RCCL with the split communicator, or the mailbox); false for one rank / loopback.
bool allreduce_overlaps(eig_ctx_t ctx);
// allreduce_sum on the split communicator (or the mailbox), for ctx->red_stream.
void allreduce_sum_red(eig_ctx_t ctx, double *buf, i64 count, hipStream_t s);
void *ctx_buffer(eig_ctx_t ctx, int slot, size_t bytes);
void host_random_normal(i64 count, unsigned seed, double *out);

}  // namespace eigmi

namespace eigmi {

// C-ABI entry guard: runs f, maps exceptions to the int status and stores the message in the
// context (or the thread's error slot when there is no context; eig_last_error(NULL) reads it).
std::string &tls_error();
template <class F>
int guard(eig_ctx_t ctx, F &&f)
{
  try
  {
    f();
    return EIG_OK;
  }
  catch (const Error &e)
  {
    (ctx ? ctx->last_error : tls_error()) = e.what();
    return e.code;
  }
  catch (const std::bad_alloc &)
  {
    (ctx ? ctx->last_error : tls_error()) = "host allocation failed";
    return EIG_ERR_ARG;
  }
  catch (const std::exception &e)
  {
    (ctx ? ctx->last_error : tls_error()) = e.what();
    return EIG_ERR_ARG;
  }
}

// Owning device buffer for driver workspaces.
struct DevBuf {
  void *p = nullptr;
  size_t n = 0;
  explicit DevBuf(size_t bytes) : n(bytes) { EIG_HIP(hipMalloc(&p, bytes ? bytes : 1)); }
  size_t bytes() const { return n; }
  ~DevBuf()
  {
    if (p) (void)hipFree(p);
  }
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  double *d() const { return static_cast<double *>(p); }
};

}  // namespace eigmi
