/* eigmi.h -- C ABI of the MI355X-native eigensolver inner loop (libeigmi.so).
 *
 * Drop-in boundary for the dune-eigensolver hot path.  Plain C: opaque
 * handles, raw pointers, sizes, int status codes.  No HIP / torch / ISTL types appear here;
 * the header-only C++ facade (eigmi.hh) maps these calls onto the reference's ISTL-style API.
 *
 * Conventions
 *  - Every `double*` vector / multivector argument is a DEVICE pointer unless the name ends in
 *    `_host`.  Small results (dot products, Gram matrices, norms) are written to DEVICE memory
 *    so that iterations never synchronise with the host; eigmi.hh copies them back.
 *  - Calls are stream-ordered on the context's stream; eig_ctx_sync() waits.  Calls that return
 *    host results (suffix _host, the drivers) are synchronous at return, like the reference.
 *  - MultiVector<double,8> buffers use the reference's block-column-major layout
 *    ((j/8)*n + i)*8 + j%8 (multivector.hh:130-139), so a host MultiVector mirrors with one copy.
 *  - Distributed vectors (a context with a communicator) use the matrix's WINDOW layout:
 *    length info.window, owned rows at offset info.own_offset; ghost rows are filled by the
 *    halo exchange inside eig_mv / the drivers.  On one rank window == n, own_offset == 0.
 *  - Errors: 0 = EIG_OK; otherwise an EIG_ERR_* code and eig_last_error(ctx) holds the message.
 *    The C++ facade rethrows SHAPE / BLOCKSIZE as std::invalid_argument, like the reference
 *    (kernels_cpp.hh:29-32, :632-633; multivector.hh:48-49).
 */
#ifndef EIGMI_H
#define EIGMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EIGMI_VERSION_MAJOR 0
#define EIGMI_VERSION_MINOR 1

enum eig_status {
  EIG_OK = 0,
  EIG_ERR_SHAPE = 1,      /* size mismatch (reference: std::invalid_argument "... does not match") */
  EIG_ERR_BLOCKSIZE = 2,  /* unsupported block size (reference: "only implemented for FieldMatrix<..,1,1>") */
  EIG_ERR_HIP = 3,        /* HIP runtime failure */
  EIG_ERR_RCCL = 4,       /* RCCL failure, or an xGMI mailbox exchange that timed out */
  EIG_ERR_BREAKDOWN = 5,  /* Krylov breakdown (beta == 0) or non-positive pivot in (B-)Gram-Schmidt */
  EIG_ERR_ARG = 6,        /* invalid argument (null handle, negative size, bad enum) */
  EIG_ERR_NODEVICE = 7    /* no HIP device visible */
};

typedef struct eig_ctx_s *eig_ctx_t;
typedef struct eig_mat_s *eig_mat_t;

/* ---------------------------------------------------------------- context ------------------ */
/* One context = one GPU + one HIP stream (+ optional RCCL communicator).  One per host thread. */
int eig_ctx_create(int device, eig_ctx_t *ctx);
int eig_ctx_destroy(eig_ctx_t ctx);
const char *eig_last_error(eig_ctx_t ctx);
int eig_ctx_sync(eig_ctx_t ctx);
/* The hipStream_t the context enqueues on, as an opaque pointer. */
int eig_ctx_stream(eig_ctx_t ctx, void **stream);
int eig_device_count(int *count);
/* Library version string, e.g. "eigmi 0.1 gfx950". */
const char *eig_version(void);

/* ---------------------------------------------------------------- communicator ------------- */
/* RCCL bootstrap in the ncclGetUniqueId / ncclCommInitRank pattern: rank 0 calls
 * eig_comm_unique_id, the 128 bytes travel by any side channel (MPI_Bcast, a TCP store),
 * then every rank calls eig_comm_init.  Afterwards dots / norms are global (allreduce over
 * xGMI) and matrices created with eig_mat_create_bcsr_dist exchange halos. */
int eig_comm_unique_id(unsigned char id[128]);
int eig_comm_init(eig_ctx_t ctx, int nranks, int rank, const unsigned char id[128]);
/* flags: EIG_COMM_MAILBOX = also set up the xGMI mailbox allreduce (below); default (0, and
 * eig_comm_init): ncclAllReduce.  EIG_COMM_ALWAYS = route every collective of the drivers through
 * the communicator even at nranks == 1 (ncclAllReduce on the main and on the split communicator,
 * inside hipGraph captures too) instead of skipping it: a one-GPU rehearsal of the transport whose
 * results must be bitwise those of the run without a communicator.  Kernel choices stay those of a
 * single rank. */
enum { EIG_COMM_MAILBOX = 1, EIG_COMM_ALWAYS = 2 };
int eig_comm_init_ex(eig_ctx_t ctx, int nranks, int rank, const unsigned char id[128], int flags);
int eig_comm_allreduce_sum(eig_ctx_t ctx, double *buf, int64_t count);
/* In-process loopback transport for testing the distributed path on ONE device: create a hub for
 * nranks virtual ranks, give each rank its own host thread + context and attach it with
 * eig_comm_init_loopback.  Halo exchange and allreduce then go through device copies and a host
 * barrier instead of RCCL (synchronous; not a performance path). */
int eig_loopback_create(int nranks, void **hub);
int eig_loopback_destroy(void *hub);
int eig_comm_init_loopback(eig_ctx_t ctx, void *hub, int rank);
/* Collective over a loopback hub (every virtual rank calls it after eig_comm_init_loopback): the
 * xGMI mailbox allreduce between the virtual ranks (their mailboxes are device pointers of the same
 * process), validated by all ranks; then eig_comm_select_allreduce may pick EIG_AR_MAILBOX /
 * EIG_AR_MAILBOX_STEP while the halo keeps the loopback copies.  The ranks' kernels wait for each
 * other, so each rank's stream needs a hardware queue of its own (GPU_MAX_HW_QUEUES >= 3 x ranks). */
int eig_comm_loopback_mailbox(eig_ctx_t ctx);
int eig_comm_barrier(eig_ctx_t ctx);
/* Allreduce transport.  With RCCL and EIG_COMM_MAILBOX, eig_comm_init_ex also sets up the xGMI
 * mailbox allreduce (every rank exports a small uncached mailbox through IPC; one launch stores
 * this rank's values into every peer's mailbox and sums all slots in rank order) for up to 16
 * ranks, validated and agreed by all ranks, else ncclAllReduce stays in use.
 * eig_comm_ipc_handle / eig_comm_ipc_open attach the mailbox alone (no RCCL): every rank exports
 * its handle, the nranks x 64 bytes travel by any side channel (rank order), then every rank opens
 * them.  Allreduces and dots go through the mailbox; the halo of distributed matrices through the
 * halo mailbox: each rank's uncached staging area (two parities x nranks slots of 8 x the largest
 * halo range of any rank), set up -- and grown -- collectively by eig_mat_create_bcsr_dist, its
 * handle gathered through the mailbox.  An exchange is two launches on the halo stream: the boundary
 * rows stored straight into the peers' slots over xGMI, then, once every peer's sequence word has
 * arrived (bounded: 2 s, then NaN ghosts and a recorded timeout), the ghosts copied out of the own
 * slots.  Sequence numbers live on the device: exchanges captured into a hipGraph replay correctly. */
#define EIG_IPC_HANDLE_BYTES 64
/* EIG_AR_MAILBOX_STEP: the mailbox for every allreduce, and the fused Lanczos step
 * (EIG_LANCZOS_FUSED) exchanges its three sums INSIDE the step kernel: the last workgroup of launch L
 * stores them into every peer's mailbox and, before launch L ends, polls its own mailbox until every
 * peer's sums of launch L have arrived (bounded: a peer that does not arrive within 2 s makes the
 * sums NaN on every rank and the step call -- or eig_lanczos_tridiag's final repair launch -- returns
 * EIG_ERR_RCCL) -- no allreduce launch between two steps. */
enum eig_allreduce_kind { EIG_AR_NONE = 0, EIG_AR_RCCL = 1, EIG_AR_MAILBOX = 2, EIG_AR_LOOPBACK = 3,
                          EIG_AR_MAILBOX_STEP = 4 };
/* Collectives the library has enqueued on its RCCL communicators since eig_comm_init (a captured
 * hipGraph counts once, at capture): out[0] = ncclAllReduce on the main communicator, out[1] =
 * ncclAllReduce on the split one (the pipelined step's overlapped allreduce), out[2] = halo groups
 * (ncclGroupStart .. End), out[3] = ncclSend + ncclRecv calls inside them. */
int eig_comm_counters(eig_ctx_t ctx, int64_t out[4]);
int eig_comm_ipc_handle(eig_ctx_t ctx, int nranks, int rank, unsigned char handle[EIG_IPC_HANDLE_BYTES]);
int eig_comm_ipc_open(eig_ctx_t ctx, const unsigned char *handles);
/* flags: EIG_COMM_ALWAYS = route the collectives through the mailbox even at nranks == 1 (a one-rank
 * mailbox: the one-GPU rehearsal of the transport, as eig_comm_init_ex's flag for RCCL). */
int eig_comm_ipc_open_ex(eig_ctx_t ctx, const unsigned char *handles, int flags);
/* nranks / rank / the allreduce in use (eig_allreduce_kind) / mailbox timeouts so far (syncs). */
int eig_comm_info(eig_ctx_t ctx, int *nranks, int *rank, int *allreduce, int *mailbox_errors);
/* Switch the allreduce transport of a communicator that has both (RCCL + a validated mailbox):
 * EIG_AR_RCCL, EIG_AR_MAILBOX or EIG_AR_MAILBOX_STEP (the mailbox alone: EIG_AR_MAILBOX or _STEP).
 * A collective: every rank selects the same one.  Synchronises the stream; with RCCL (or loopback)
 * beside the mailbox it restarts the mailbox on every rank between two barriers (mailbox, call
 * counters and recorded timeouts zeroed), so a transport that timed out can be selected again with
 * consistent sequence words.  A mailbox alone (eig_comm_ipc_open) only clears the recorded timeouts:
 * after a timeout, re-open it. */
int eig_comm_select_allreduce(eig_ctx_t ctx, int kind);
/* Halo transport of the distributed matrices of a context that has RCCL and a validated mailbox
 * (eig_comm_init_ex with EIG_COMM_MAILBOX): EIG_HALO_RCCL (grouped ncclSend / ncclRecv, the
 * default) or EIG_HALO_MAILBOX (the halo mailbox, as on mailbox-only ranks; its staging is set up
 * by eig_mat_create_bcsr_dist whenever the mailbox is).  A collective: every rank selects the same
 * one; synchronises the context's streams. */
enum eig_halo_kind { EIG_HALO_RCCL = 1, EIG_HALO_MAILBOX = 2 };
int eig_comm_select_halo(eig_ctx_t ctx, int kind);

/* ---------------------------------------------------------------- device memory ------------ */
int eig_malloc(eig_ctx_t ctx, size_t bytes, void **ptr);
int eig_free(eig_ctx_t ctx, void *ptr);
int eig_memcpy_h2d(eig_ctx_t ctx, void *dst, const void *src_host, size_t bytes);
int eig_memcpy_d2h(eig_ctx_t ctx, void *dst_host, const void *src, size_t bytes);
int eig_memcpy_d2d(eig_ctx_t ctx, void *dst, const void *src, size_t bytes);
int eig_memset(eig_ctx_t ctx, void *dst, int value, size_t bytes);

/* ---------------------------------------------------------------- matrices ----------------- */
/* Replaces Dune::BCRSMatrix<FieldMatrix<double,br,bc>> on the device.  Host arrays follow the
 * ISTL row/col iteration (kernels_cpp.hh:644-655): rowptr[nb_rows+1] (int64), col[nnzb]
 * (int32 block column, ascending per row), vals[nnzb*br*bc] (row-major blocks, FieldMatrix
 * layout).  Supported blocks: br, bc in 1..4 (any combination).  The device copy is a sliced
 * ELLPACK (SELL-64, one wavefront per 64-row slice) that keeps every row's stored order, so
 * y = A x is bitwise identical to BCRSMatrix::mv. */
int eig_mat_create_bcsr(eig_ctx_t ctx, int64_t nb_rows, int64_t nb_cols, int br, int bc,
                        const int64_t *rowptr_host, const int32_t *col_host, const double *vals_host,
                        eig_mat_t *mat);
/* Row-partitioned variant: this rank owns global block rows [row_begin, row_begin+nb_rows_local);
 * rowptr/col/vals describe those rows only, col holds GLOBAL block columns.  Collective over
 * the context's communicator (the halo plan is agreed with the other ranks). */
int eig_mat_create_bcsr_dist(eig_ctx_t ctx, int64_t nb_rows_global, int64_t row_begin,
                             int64_t nb_rows_local, int br, int bc, const int64_t *rowptr_host,
                             const int32_t *col_host, const double *vals_host, eig_mat_t *mat);
/* Kernel-image policy of a matrix, fixed at creation (the _ex variants; 0 = the default, which
 * picks the fastest image the matrix admits).  These exist for A/B measurements and for the tests
 * that pin every image against the oracle:
 *   EIG_MAT_NO_BAND      no symmetric band image: the scalar kernels read the SELL / stencil image
 *   EIG_MAT_BAND_GATHER  band image, but every offset through its own gather (no DPP lane shifts)
 *   EIG_MAT_NO_STENCIL   SELL slices keep explicit column indices (no per-slice offsets + row masks)
 *   EIG_MAT_NO_MARCH     no plane-marching kernels (band image: the row kernels)
 *   EIG_MAT_NO_CLASS     the 32-column box kernels keep the box image even when every row's entries
 *                        equal those of its geometric class (row-class image, k_box.hip)
 *   EIG_MAT_NO_UNIFORM   the plane-march kernels load the band values even when every stored entry
 *                        of each band diagonal has one value (constant-coefficient stencils) */
enum {
  EIG_MAT_NO_BAND = 1,
  EIG_MAT_BAND_GATHER = 2,
  EIG_MAT_NO_STENCIL = 4,
  EIG_MAT_NO_MARCH = 8,
  EIG_MAT_NO_CLASS = 16,
  EIG_MAT_NO_UNIFORM = 32,
  EIG_MAT_FLAGS_ALL = 63
};
int eig_mat_create_bcsr_ex(eig_ctx_t ctx, int64_t nb_rows, int64_t nb_cols, int br, int bc,
                           const int64_t *rowptr_host, const int32_t *col_host, const double *vals_host, int flags,
                           eig_mat_t *mat);
int eig_mat_create_bcsr_dist_ex(eig_ctx_t ctx, int64_t nb_rows_global, int64_t row_begin,
                                int64_t nb_rows_local, int br, int bc, const int64_t *rowptr_host,
                                const int32_t *col_host, const double *vals_host, int flags, eig_mat_t *mat);
int eig_mat_destroy(eig_mat_t mat);

typedef struct eig_mat_info {
  int64_t n;            /* owned scalar rows (nb_rows_local * br) */
  int64_t n_global;     /* global scalar rows */
  int64_t ncols;        /* scalar columns (global) */
  int64_t row_begin;    /* first owned global scalar row */
  int64_t window;       /* length of a distributed vector buffer (scalar entries) */
  int64_t own_offset;   /* offset of the owned rows inside the window */
  int64_t nnzb;         /* stored blocks (true, not padded) */
  int64_t nnzb_padded;  /* blocks in the SELL-64 image including padding */
  int64_t nslices;
  int br, bc;
  int64_t halo_recv;    /* ghost scalar entries received per exchange */
  int64_t halo_send;    /* scalar entries sent per exchange */
  int64_t device_bytes; /* matrix image size in HBM */
  int64_t stencil_slices; /* slices read through per-slice column offsets + row masks */
  int64_t rows_per_lane;  /* R of the SELL-C image (C = 64 R) */
  int64_t sym_offsets;    /* offsets of the symmetric band image (0 = none; the scalar SpMV and
                             Lanczos kernels then read the upper-triangle band arrays) */
  int64_t sym_arrays;     /* band arrays (distinct |offset|), 8 B per row each */
  int64_t sym_mask_bytes; /* row-mask bytes per row (1 or 4) */
  int64_t sym_uniform;    /* 1: every stored entry of each band diagonal has one value (constant-
                             coefficient stencil): the plane-march kernels stream the row mask and
                             the vectors only; 2: besides, the rows form a grid whose rows store
                             exactly their in-grid neighbours, and the march derives the row masks
                             from the coordinates (vectors only); EIG_MAT_NO_UNIFORM: 0 */
  int64_t sym_geo;        /* 1: the rows form a grid whose rows store exactly their in-grid
                             neighbours (geometric row masks; a property of the pattern, any values) */
  int64_t march_variant;  /* plane-march variant of a whole-matrix fused Lanczos launch (-1: no
                             march, the row kernels): 0 band arrays + loaded masks, 1 uniform values +
                             loaded masks, 2..9 uniform values + geometric masks, 10 / 11 band arrays
                             streamed + geometric masks (the value march; 11 one plane ahead, 14 / 15
                             through global addresses, 15 on a pair-packed copy of the arrays), 12 / 16
                             the P1 Kuhn 15-point box march (16 on its pair-packed values) */
  int64_t march_variant_mv; /* the same for eig_mv (BCRSMatrix::mv) */
} eig_mat_info;
int eig_mat_get_info(eig_mat_t mat, eig_mat_info *info);

/* Measurement helper: the kernel a whole-matrix Lanczos step launch uses on this matrix image
 * (fused = 1: the one-reduction step; 0: the classic SpMV kernel K1) and its algorithmic HBM bytes
 * per launch for that image: SELL/stencil images 12 nnz + 4(n+1) + vectors,
 * the symmetric band image 8 nup n + mask bytes + vectors.  `name` gets at most name_len bytes. */
int eig_lanczos_kernel_info(eig_mat_t mat, int fused, char *name, int name_len, int64_t *bytes);
/* Kernel family a whole-matrix launch of `op` picks on this matrix image (its creation flags
 * included): EIG_OP_SPMV (eig_mv), EIG_OP_LANCZOS_K1, EIG_OP_LANCZOS_FUSED,
 * EIG_OP_SPMM8 (eig_spmm_mv8, per 8-column block), EIG_OP_CHEB8 (eig_mass_solve_mv8's step). */
enum { EIG_OP_SPMV = 0, EIG_OP_LANCZOS_K1 = 1, EIG_OP_LANCZOS_FUSED = 2, EIG_OP_SPMM8 = 3, EIG_OP_CHEB8 = 4,
       EIG_OP_SPMM32 = 5, EIG_OP_CHEB32 = 6 /* m % 32 == 0: the 3-D box-stencil kernel where it applies */ };
int eig_mat_kernel_info(eig_mat_t mat, int op, char *name, int name_len);

/* Measurement / tuning override of a launch parameter the library otherwise derives from the
 * image and the device (no environment switches): EIG_TUNE_MARCH_RUNS = plane runs per 64-row column
 * of the plane-march kernels (value 0 = automatic: one work item per resident wave slot);
 * EIG_TUNE_BOX_SEGS = z segments per tile column of the 3-D box kernels (0 = automatic; results
 * bitwise unchanged, every row's sum is formed in one place).  Results are otherwise unchanged except
 * for the summation order of the step's reductions. */
enum { EIG_TUNE_MARCH_RUNS = 1, EIG_TUNE_BOX_SEGS = 2, EIG_TUNE_MARCH_PREFETCH = 3, EIG_TUNE_HALO = 4,
       EIG_TUNE_CACHE = 5, EIG_TUNE_BOX_COLS = 6, EIG_TUNE_BOX_MAP = 7, EIG_TUNE_SELL_CPF = 8,
       EIG_TUNE_MARCH_LINES = 9 };
/* EIG_TUNE_MARCH_LINES (value marches on 3-D geometric bands): 4 = a workgroup's 4 waves march the
 * same 64 x of 4 consecutive grid lines (their +-nx gathers mostly read the lines their sibling
 * waves just loaded), 0 = the 4 x runs of one line (default; measurement switch: the fused step at
 * 256^3 measured the same either way, 222.5 vs 222.7 us, FETCH_SIZE 2 % lower).  eig_mv bitwise
 * unchanged; the fused step's reductions sum in another order. */
/* EIG_TUNE_SELL_CPF (explicit-column SELL slices; measurement switch): 1 = the next slice's column
 * indices loaded while this slice's gathers are in flight (one memory round trip per slice instead
 * of two), in the fused Lanczos step (5 waves per SIMD instead of 6) and in eig_mv; 0 / 2 = off (the
 * default: measured slower, 437 vs 402 us for the general 256^3 fused step).  eig_mv and every
 * row's products bitwise identical; the fused step's three sums are added in another order where
 * the occupancy-derived grid differs (large matrices), so its alpha / beta agree to rounding there. */
/* EIG_TUNE_BOX_MAP (measurement; k_box_mv32): 1 = XCD-contiguous tile map (the workgroups resident on
 * one XCD hold whole rows of adjacent tiles), 0 = dispatch order.  Results bitwise identical. */
/* EIG_TUNE_BOX_COLS (box-image kernels, EIG_OP_SPMM32 / EIG_OP_CHEB32 on matrices without a row-class
 * image): 32 = k_box_mv32 (32 columns per workgroup, three X planes in LDS), 16 = k_box_mv16p (16
 * columns per workgroup, one X plane in LDS, sums pushed to the rows of planes p - 1, p, p + 1);
 * 0 = automatic.  Results bitwise identical. */
/* EIG_TUNE_CACHE (measurement; fused value march): bit 0 = the (t, u) pairs stored with plain (MALL-
 * allocating) stores instead of nontemporal ones, bit 1 = the value streams with the default cache
 * policy, bit 2 = the +D pair stream nontemporal.  Results unchanged. */
/* EIG_TUNE_HALO (distributed Lanczos steps): 0 = the interior planes run while the halo is in flight
 * and the boundary planes after it (two launches, the default); 1 = the exchange first, then ONE
 * launch over all owned rows (no second launch's fixed cost; the exchange is exposed).  The step's
 * sums are then formed in another (fixed) order. */
/* EIG_TUNE_MARCH_PREFETCH (geometric uniform-band images, eig_mat_info.sym_uniform = 2): 1 = the
 * plain march, 2 / 3 / 4 = the +D operand loaded 1 / 2 / 3 planes ahead, 5 = 3 planes ahead and the
 * neighbour gathers 1 plane ahead; 6 / 7 / 8 = the variants of 2 / 3 / 5 without row masks or
 * selects (missing neighbours read as exact zeros; grids whose x extent is a multiple of 64);
 * on geometric bands whose values are not uniform (or EIG_MAT_NO_UNIFORM): 1 = the plain masked
 * march on the band arrays, 9 = the value march (eig_mat_info.march_variant 10: the band arrays
 * streamed, masks from the coordinates), 10 = the same with the value streams one plane ahead (11),
 * 11 = the value march on a packed copy of the 4 arrays (13: {+D, 0, +1, +nx} per row, two 16-B loads);
 * 16 / 17 / 18 = that pack marched TWO grid lines per wave (march variants 22 / 23 / 24: 5 / 4 / 6
 * waves per SIMD; 7-point bands, an even line count) -- the +-nx neighbours across the pair from
 * registers, half the gathers; the fused step's sums then add the rows in another order;
 * 0 = automatic: the fused step on 3-D value images takes variant 22 on ranks of at least
 * EIG_MARCH_2L_MIN_ROWS owned rows, else 15.  Bitwise the same rows for every value. */
#define EIG_MARCH_2L_MIN_ROWS 4194304
int eig_mat_tune(eig_mat_t mat, int key, int value);

/* a13: A += shift*I on the diagonal of every diagonal block (eigensolver.hh:59-66). */
int eig_mat_shift_diag(eig_mat_t mat, double shift);

/* a4: y = A x  (BCRSMatrix::mv; the ARPACK++ multMvB callback, arpack_geneo_wrapper.hh:269-279).
 * x: window layout (ghosts exchanged here when distributed); y: owned rows written at own_offset. */
int eig_mv(eig_mat_t mat, const double *x, double *y);
/* Same with caller-owned HOST arrays of length n (ARPACK's workd): stage, multiply, copy back. */
int eig_mv_host(eig_mat_t mat, const double *x_host, double *y_host);
/* Measurement helper: `reps` back-to-back eig_mv launches bracketed by HIP events on the
 * context stream; *avg_ms = elapsed / reps (synchronous). */
int eig_mv_timed(eig_mat_t mat, const double *x, double *y, int reps, double *avg_ms);

/* ---------------------------------------------------------------- BlockVector ops ---------- */
/* n = owned length; pointers address the owned slice.  Results to device memory. */
int eig_dot(eig_ctx_t ctx, int64_t n, const double *x, const double *y, double *result);
int eig_nrm2(eig_ctx_t ctx, int64_t n, const double *x, double *result);
int eig_axpy(eig_ctx_t ctx, int64_t n, double a, const double *x, double *y);   /* y += a x */
int eig_scal(eig_ctx_t ctx, int64_t n, double a, double *x);                    /* x *= a */
int eig_copy(eig_ctx_t ctx, int64_t n, const double *x, double *y);
/* The Lanczos update an external Krylov driver applies to the vector its operator callback returned
 * (ARPACK's dsaitr after multMv, arpack_geneo_wrapper.hh:257-279; SURVEY 8(b) "BlockVector ops"),
 * as ONE pass instead of axpy + axpy + nrm2 (+ dot):
 *   w <- (w - alpha v) - beta vprev;   result[0] = ||w||_2,  result[1] = v . w   (of the new w)
 * alpha, beta: device scalars (vprev == NULL: no beta term, beta may be NULL); result: 2 device
 * doubles.  result[1] is the loss of orthogonality a DGKS test compares with eta ||w||.  With a
 * communicator both sums are global (one allreduce of 2 values). */
int eig_lanczos_update(eig_ctx_t ctx, int64_t n, const double *alpha, const double *beta, const double *v,
                       const double *vprev, double *w, double *result);
/* Measurement helper: `reps` launches of a 16-B-per-lane nontemporal stream copy y = x (n doubles;
 * 16 n bytes moved per launch) bracketed by HIP events; *avg_ms per launch.  The measured HBM peak
 * the bench's roofline fractions are also quoted against.  mode: bit 0 nontemporal
 * loads / stores, bit 1 one element per thread over a full grid (else a resident striding grid). */
int eig_stream_copy_timed(eig_ctx_t ctx, int64_t n, const double *x, double *y, int reps, int mode,
                          double *avg_ms);

/* ---------------------------------------------------------------- MultiVector<double,8> ---- */
/* a2: Qout = A Qin, m columns (m % 8 == 0), br = bc = 1 (kernels_cpp.hh:626-657). */
int eig_spmm_mv8(eig_mat_t mat, int64_t m, const double *Qin, double *Qout);
/* a5: dp[j] = q1_j . q2_j, j < m (kernels_cpp.hh:24-55).  dp: device, m doubles. */
int eig_dot_diag_mv8(eig_ctx_t ctx, int64_t n, int64_t m, const double *Q1, const double *Q2, double *dp);
/* a6: G = Q1^T Q2 (m1 x m2, row-major, device) -- the tall-skinny panel product, on MFMA
 * (v_mfma_f64_16x16x4f64).  Q1 has m1 columns, Q2 m2 columns, both MultiVector<double,8>. */
int eig_gram_mv8(eig_ctx_t ctx, int64_t n, int64_t m1, int64_t m2, const double *Q1, const double *Q2, double *G);
/* a9 / a10: orthonormalise the m columns of Q in place.
 * EIG_ORTHO_MGS    = orthonormalize_blocked (kernels_cpp.hh:180-351): diagonal block by column MGS,
 *                    later blocks by one block-CGS pass.
 * EIG_ORTHO_CHOLQR = orthonormalize_avx2_b8_v2 / _neon_b8_v2 (kernels_avx2.hh:385-622): CholQR of
 *                    the diagonal block, one 8x8 projection per later block.
 * EIG_ORTHO_CHOLQR_SPLIT = orthonormalize_avx2_b8 (kernels_avx2.hh:64-381): the same CholQR of the
 *                    diagonal block, later blocks projected in two halves (columns 0-3, then 4-7
 *                    against the updated block). */
enum eig_ortho_variant { EIG_ORTHO_MGS = 0, EIG_ORTHO_CHOLQR = 1, EIG_ORTHO_CHOLQR_SPLIT = 2 };
/* or-ed into `variant`: the grid-wide MGS passes (the default for every n since round 5; kept as a
 * flag for A/B and tests) */
enum { EIG_ORTHO_GRID = 0x100 };
/* or-ed into `variant` for EIG_ORTHO_MGS on one rank: the diagonal block's 8 MGS steps in ONE
 * workgroup that keeps the block in registers (n <= 4096).  Measured slower than the default
 * look-ahead at every such n (17.8-28.9 us against 16.0-17.5 us per 8-column block, n = 512-4096,
 * profiles/r05zs_small_ortho_kernel_stats.csv): an alternative for A/B and tests. */
enum { EIG_ORTHO_ONE_WG = 0x400 };
/* or-ed into `variant`: the look-ahead MGS without its barrier-capable last launch (the worst case
 * of refused look-aheads enqueued as 9 launches; A/B and tests) */
enum { EIG_ORTHO_NO_COOP = 0x200 };
/* or-ed into `variant` for EIG_ORTHO_MGS on one rank: at most L (1..8) MGS steps per read pass of
 * the diagonal block (Gram look-ahead: the window's later steps from the Schur complement of its
 * Gram rows, taken only while a column keeps >= 1/16 of its squared norm, else that step runs
 * direct in the next pass).  L = 1: one pass per step, as kernels_cpp.hh:202-229 orders them.
 * 0: the library default (8, or EIGMI_MGS_LOOKAHEAD). */
#define EIG_ORTHO_LOOKAHEAD_SHIFT 12
#define EIG_ORTHO_LOOKAHEAD(L) ((L) << EIG_ORTHO_LOOKAHEAD_SHIFT)
/* StandardLargest's fused pair (eigensolver.hh:78-85 with the product reused),
 * exported so a caller's loop can run exactly what eig_standard_largest runs:
 *   eig_spmm_dot_gram_mv8: Qout = A Qin (m = 8), dp[j] = qin_j . qout_j (8 device doubles) and
 *     gram[8 w + c] = qout_w . qout_c (8 x 8 device doubles, c >= w used) -- summed in the product's
 *     epilogue while the rows are in registers (else a separate panel Gram);
 *   eig_orthonormalize_gram_mv8: eig_orthonormalize_mv8 (MGS) whose first block starts from that Gram
 *     instead of reading the block for its first look-ahead pass. */
int eig_spmm_dot_gram_mv8(eig_mat_t mat, int64_t m, const double *Qin, double *Qout, double *dp, double *gram);
int eig_orthonormalize_gram_mv8(eig_ctx_t ctx, int64_t n, int64_t m, double *Q, const double *gram);
/* Asynchronous like every kernel op.  The look-ahead MGS's last launch synchronises its workgroups
 * with grid barriers (bounded wait): if they are not co-resident in time the block is set to NaN and
 * the next eig_ctx_sync (or the driver that called it) returns EIG_ERR_HIP. */
int eig_orthonormalize_mv8(eig_ctx_t ctx, int64_t n, int64_t m, double *Q, int variant);
/* Diagnostics: read passes the last look-ahead MGS on ctx took for its last diagonal block (-1
 * when none ran).  Synchronises the context stream. */
int eig_orthonormalize_passes(eig_ctx_t ctx, int *passes);
/* a8: orthonormalize_naive on a column-major (MultiVector<double,1>) block (kernels_cpp.hh:121-155). */
int eig_orthonormalize_naive(eig_ctx_t ctx, int64_t n, int64_t m, double *Q);
/* a11: B-orthonormalise Q (B_orthonormalize_blocked, kernels_cpp.hh:356-591); *norm (device)
 * receives the max off-diagonal R coefficient the reference returns. */
int eig_b_orthonormalize_mv8(eig_mat_t B, int64_t m, double *Q, double *norm);
/* eigensolver.hh:49-55 start block: mt19937(seed) + normal_distribution(0,1), fill order
 * (block, row, col); generated on the host (bitwise the reference's numbers), uploaded. */
int eig_random_mv8(eig_ctx_t ctx, int64_t n, int64_t m, unsigned seed, double *Q);
/* Host only (no device): `count` N(0, 1) variates, bitwise std::normal_distribution<double>{0, 1}
 * drawn from std::mt19937{seed} (libstdc++), the start blocks of eigensolver.hh:50-55 that the
 * drivers and eig_random_mv8 use. */
int eig_random_normal(int64_t count, unsigned seed, double *out);
/* x[0..count) = N(0,1) numbers from a counter-based generator on the device (seeded; NOT the
 * reference's mt19937 sequence -- for synthetic workloads and measurements). */
int eig_fill_normal(eig_ctx_t ctx, int64_t count, unsigned seed, double *x);

/* ---------------------------------------------------------------- drivers ------------------ */
/* a12: StandardLargest (eigensolver.hh:28-112) on the device.  Mutates the matrix when
 * shift != 0 (like the reference).  eval_host[nev] (column order, unsorted, like the reference);
 * evec_host: nev vectors of n doubles each, or NULL.  *iters: the k at exit. */
int eig_standard_largest(eig_mat_t A, double shift, double tol, int maxiter, int nev, unsigned seed,
                         double *eval_host, double *evec_host, int *iters, int verbose);

/* Lanczos three-term recurrence on A (the loop ARPACK's dsaupd runs around multMv):
 * `steps` steps from the start vector u0 (device, window layout; NULL = mt19937(seed) normal).
 * Only three vectors are kept (no basis); alpha_host[steps], beta_host[steps+1] receive the
 * tridiagonal T (beta[0] = ||u0||).  This is the benchmark's unit of work. */
typedef struct eig_timing {
  double total_ms;        /* wall time of the stepping loop (device events, first to last) */
  double spmv_ms;         /* summed duration of the fused SpMV kernel launches */
  double update_ms;       /* summed duration of the fused axpy/norm kernel launches (TIME_DETAIL) */
  double comm_ms;         /* summed duration of the allreduce segments (TIME_DETAIL) */
  int64_t spmv_launches;  /* number of SpMV kernel launches timed */
} eig_timing;
enum eig_lanczos_flags {
  EIG_LANCZOS_TIME_KERNELS = 1, /* HIP events around every fused SpMV launch (spmv_ms) */
  EIG_LANCZOS_TIME_DETAIL = 2,  /* + events after each allreduce and update (update_ms, comm_ms) */
  /* One-reduction fused step: u_k = t_{k-1} - c u_{k-1} is formed inside the next
   * SpMV's gathers and its squared norm is predicted as ||t||^2 - (t.u)^2/||u||^2 from the three
   * sums (t.u, t.t, u.u) the previous step reduced, so a step is ONE kernel + ONE allreduce of
   * three doubles (2 pair vectors instead of 3 vectors).  Guarded: the step runs on A - mu I with
   * mu = trace(A)/n (alpha reported unshifted), and a launch whose prediction keeps less than 1e-2
   * of ||t||^2 repairs instead (forms u_k, reduces its exact norm; the next launch takes the step),
   * decided on the device.  beta[k] of eig_lanczos_tridiag is always the exact ||u_k||.  Same
   * Krylov process as the two-kernel step; alpha/beta agree with it to its own rounding spread. */
  EIG_LANCZOS_FUSED = 4,
  /* Pipelined one-reduction step, for N > 1 ranks: the same scalars, guard and
   * repairs as EIG_LANCZOS_FUSED, but a step's SpMV multiplies t_{k-1} (S = A t_{k-1}, an eig_mv
   * launch that needs no scalar of the previous step) and a row kernel forms u_k = t_{k-1} - c u_{k-1},
   * z_k = S - c z_{k-1} (= A u_k) and t_k; so the previous step's 3-value allreduce (second RCCL
   * communicator, its own stream) overlaps the SpMV and the halo of t (8 B per row, not 16).
   * Costs 56 B per row more than the fused step on one GPU.  Exclusive with EIG_LANCZOS_FUSED. */
  EIG_LANCZOS_PIPELINED = 8,
  /* Pick per matrix at creation: EIG_LANCZOS_FUSED for every 1x1 (scalar) matrix image -- band,
   * stencil or scattered (256^3 scrambled + RCM: 415 us per fused step vs 436 for the two-kernel
   * step) -- the two-kernel step for blocked images.  eig_lanczos_ws_info reports the
   * choice. */
  EIG_LANCZOS_AUTO = 16
};
int eig_lanczos_run(eig_mat_t A, int steps, const double *u0, unsigned seed, int flags,
                    double *alpha_host, double *beta_host, eig_timing *timing);

/* The same recurrence as a persistent workspace (ARPACK's reverse-communication shape): create
 * allocates the three window vectors and the device scalar arrays for up to max_steps steps and
 * normalises the start vector; each eig_lanczos_step call advances `steps` more steps
 * (synchronous at return); eig_lanczos_tridiag copies alpha[0..k), beta[0..k] of the k steps
 * done so far.  No host synchronisation happens inside a step batch. */
typedef struct eig_lanczos_s *eig_lanczos_t;
int eig_lanczos_create(eig_mat_t A, int max_steps, const double *u0, unsigned seed, eig_lanczos_t *ws);
/* flags: 0 (two-kernel step, as eig_lanczos_create), EIG_LANCZOS_FUSED or EIG_LANCZOS_PIPELINED. */
int eig_lanczos_create_ex(eig_mat_t A, int max_steps, const double *u0, unsigned seed, int flags,
                          eig_lanczos_t *ws);
int eig_lanczos_step(eig_lanczos_t ws, int steps, int flags, eig_timing *timing);
int eig_lanczos_tridiag(eig_lanczos_t ws, int *k, double *alpha_host, double *beta_host);
int eig_lanczos_destroy(eig_lanczos_t ws);
/* Logical steps taken and kernel launches issued (fused: steps + repairs + forced final repairs;
 * two-kernel: = steps). */
int eig_lanczos_info(eig_lanczos_t ws, int *steps, int *launches);
/* The recurrence the workspace runs (*variant: 0 two-kernel, EIG_LANCZOS_FUSED or
 * EIG_LANCZOS_PIPELINED, after EIG_LANCZOS_AUTO resolved it), its step kernel (name, at most
 * name_len bytes) and that kernel's algorithmic bytes per launch (as eig_lanczos_kernel_info). */
int eig_lanczos_ws_info(eig_lanczos_t ws, int *variant, char *name, int name_len, int64_t *bytes);
/* hipGraph form of eig_lanczos_step: capture the next `steps` steps (kernels, halo exchange,
 * allreduces; plus per-step kernel events when flags has EIG_LANCZOS_TIME_KERNELS) into one
 * graph and instantiate it -- nothing runs yet.  eig_lanczos_replay launches it once
 * (synchronous) and advances the step count.  *captured = 0 when the runtime refused the capture
 * (the replay then runs the same steps eagerly). */
int eig_lanczos_capture(eig_lanczos_t ws, int steps, int flags, int *captured);
int eig_lanczos_replay(eig_lanczos_t ws, eig_timing *timing);

/* Lanczos eigensolver: ncv-step Lanczos with full re-orthogonalisation (classical Gram-Schmidt
 * twice, the DGKS scheme ARPACK uses) and Ritz extraction from T.  which: EIG_WHICH_LA (largest
 * algebraic) or EIG_WHICH_SA (smallest algebraic).  eval_host[nev] sorted (LA: descending,
 * SA: ascending); evec_host: nev owned-row vectors or NULL; resid_host[nev] (optional):
 * ||A y - theta y|| of each returned pair (computed on the device). */
enum eig_which { EIG_WHICH_LA = 0, EIG_WHICH_SA = 1 };
int eig_lanczos_solve(eig_mat_t A, int nev, int ncv, int which, unsigned seed, double *eval_host,
                      double *evec_host, double *resid_host);

/* ---------------------------------------------------------------- exported LU factors ------ */
/* Mirror of UMFPackFactorizedMatrix (umfpacktools.hh:16-199): the factors of P R A Q = L U that
 * umfpack_dl_get_numeric exports -- L (n x n, unit lower) in compressed ROW form with the unit
 * diagonal LAST in each row (Lp[n+1], Lj, Lx), U in compressed COLUMN form with the diagonal LAST
 * in each column (Up[n+1], Ui, Ux), row permutation P[n], column permutation Q[n], row scaling
 * Rs[n] (do_recip: row i multiplied by Rs[i], else divided).  Host arrays, copied. */
typedef struct eig_lu_s *eig_lu_t;
int eig_lu_create(eig_ctx_t ctx, int64_t n, const int64_t *Lp, const int64_t *Lj, const double *Lx,
                  const int64_t *Up, const int64_t *Ui, const double *Ux, const int64_t *P, const int64_t *Q,
                  const double *Rs, int do_recip, eig_lu_t *lu);
/* Host factorisation into the same form (stand-in for umfpack_dl_symbolic / _numeric when
 * SuiteSparse is absent): reverse Cuthill-McKee symmetric ordering (P = Q), row-sum scaling
 * (do_recip = 0), envelope LU WITHOUT pivoting -- for SPD, diagonally dominant or positively
 * shifted matrices; EIG_ERR_BREAKDOWN on a zero pivot.  BCRS input as eig_mat_create_bcsr (br = bc,
 * zero entries of blocks skipped like umfpacktools.hh:66-93).  ctx == NULL: host-only factors (no device
 * image; eig_lu_export works, eig_inverse_mv8 refuses). */
int eig_lu_create_bcsr(eig_ctx_t ctx, int64_t nb_rows, int br, const int64_t *rowptr, const int32_t *col,
                       const double *vals, eig_lu_t *lu);
int eig_lu_info(eig_lu_t lu, int64_t *n, int64_t *lnz, int64_t *unz, int *do_recip);
/* Triangular-solve kernels eig_inverse_mv8 uses for these factors (default EIG_TRSV_AUTO: the
 * block-inverse solve where the factors have its image, else the block-staged / row-CSR
 * substitution).  EIG_TRSV_STAGED and EIG_TRSV_CSR are bitwise the reference arithmetic
 * (matmul_inverse_tallskinny_blocked, kernels_cpp.hh:660-755); the block-inverse solve agrees to
 * rounding. */
enum { EIG_TRSV_AUTO = 0, EIG_TRSV_BLOCKINV = 1, EIG_TRSV_STAGED = 2, EIG_TRSV_CSR = 3 };
int eig_lu_set_solver(eig_lu_t lu, int kind);
/* The kernels eig_inverse_mv8 runs now (*kind: EIG_TRSV_BLOCKINV / _STAGED / _CSR) and the coupled
 * 64-row blocks of the L / U envelopes (the block-inverse chain takes up to 8). */
int eig_lu_solver_info(eig_lu_t lu, int *kind, int *coupled_l, int *coupled_u);
/* Copy the factors out (sizes from eig_lu_info: Lp/Up n+1, Lj/Lx lnz, Ui/Ux unz, P/Q/Rs n). */
int eig_lu_export(eig_lu_t lu, int64_t *Lp, int64_t *Lj, double *Lx, int64_t *Up, int64_t *Ui, double *Ux,
                  int64_t *P, int64_t *Q, double *Rs);
int eig_lu_destroy(eig_lu_t lu);
/* Qout = A^-1 Qin for m columns (matmul_inverse_tallskinny_blocked, kernels_cpp.hh:660-755;
 * MultiVector<double,8> layout, n rows, single rank).  Qin is used as scratch (its contents afterwards are
 * unspecified), as the reference allows (kernels_cpp.hh:659).
 * Default: factors whose envelope fits (every coupling within 4 blocks of 64 rows; RCM envelope
 * factors of bandwidth <= 256) take the block-inverse solve (products with the inverted 64 x 64
 * diagonal blocks; within 1e-13 of the largest |entry| of the reference's result, not bitwise).
 * Environment EIGMI_TRSV=staged / csr selects the substitution kernels, bitwise the reference's
 * arithmetic when the L rows are stored in ascending column order (as are all other factors). */
int eig_inverse_mv8(eig_lu_t lu, int64_t m, double *Qin, double *Qout);

/* StandardInverse (eigensolver.hh:116-198): inverse subspace iteration for the nev smallest
 * eigenvalues of A (+ shift; mutates A like the reference when shift != 0).  The LU of the shifted
 * A is computed on the host (eig_lu_create_bcsr) unless `lu` is given (factors of the SHIFTED A).
 * eval_host[nev] unsorted (column order), evec_host nev x n or NULL, *iters = k at exit. */
int eig_standard_inverse(eig_mat_t A, eig_lu_t lu, double shift, double tol, int maxiter, int nev, unsigned seed,
                         double *eval_host, double *evec_host, int *iters, int verbose);
/* GeneralizedInverse (eigensolver.hh:204-351): A x = lambda B x by inverse subspace iteration with
 * B-orthonormalisation; factors A + shift B + reg I (a copy: A itself is not modified, like the
 * reference's copy at :208).  pattern(A) must contain pattern(B) (:202-203).  Stops when
 * iter > 10 and max|delta ra| / max(ra) < tol (:315-324). */
int eig_generalized_inverse(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double shift, double reg, double tol, int maxiter,
                            int nev, unsigned seed, double *eval_host, double *evec_host, int *iters, int verbose);

/* computeGenSymShiftInvertMinMagnitude (arpack_geneo_wrapper.hh:581-658): the nev eigenpairs of
 * A x = lambda B x nearest sigma ("LM" on OP = (A - sigma B)^-1 B, the operator ARSymGenEig's 'S'
 * mode builds from multMv / multMvB, :621-622), by thick-restart Lanczos in the B-inner product with
 * full (DGKS) re-orthogonalisation.  B = NULL: standard problem.  The LU of A - sigma B (A's pattern
 * must contain B's, :599-600) is computed on the host unless `lu` (factors of A - sigma B) is given.
 * ncv = 0: min(n, max(2 nev + 1, 20)); tol = 0: machine precision; maxit = 0: 100 nev restarts
 * (ARPACK++ defaults).  Converged when |beta_m y_m,i| <= tol |theta_i| for the nev wanted pairs.
 * eval_host[nev] ascending (the reference sorts the unshifted values, :636-648); evec_host nev x n
 * B-normalised, or NULL; *restarts: thick restarts taken. */
int eig_shift_invert_solve(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double sigma, int nev, int ncv, double tol,
                           int maxit, unsigned seed, double *eval_host, double *evec_host, int *restarts);
/* The same with the Krylov method chosen.  EIG_SI_SINGLE: the one-vector thick-restart Lanczos
 * above (ARPACK's dsaupd recurrence; one OP application per basis vector).  EIG_SI_BLOCK: block
 * Lanczos with Krylov-Schur restarts on p = max(16, 8 ceil(nev / 8)) columns -- one OP application
 * is a latency-bound block-inverse chain per 8 columns that costs about the same for 16 columns as
 * for one, so the block space reaches the wanted pairs in far fewer applications; the same wanted
 * pairs, B-inner product, convergence test (||R y_i|| <= tol |theta_i|, R the residual block's
 * coupling) and purified vectors; ncv = a lower bound on the search dimension; *restarts counts block
 * restarts.  EIG_SI_AUTO (0, what eig_shift_invert_solve and eig_shift_invert_adaptive use): the block
 * method when its basis (at most ~4 p + 1.5 nev columns) is at most n / 4 and its projection Gram
 * (basis x p, in 16 x 16 tiles) fits the 64 device reduction slots, else the one-vector one;
 * EIG_SI_BLOCK with an nev past that limit returns EIG_ERR_ARG. */
#define EIG_SI_AUTO 0
#define EIG_SI_SINGLE 1
#define EIG_SI_BLOCK 2
int eig_shift_invert_solve_ex(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double sigma, int nev, int ncv, double tol,
                              int maxit, unsigned seed, double *eval_host, double *evec_host, int *restarts,
                              int flags);
/* computeGenSymShiftInvertMinMagnitudeAdaptive (arpack_geneo_wrapper.hh:661-774): every eigenvalue of
 * the pencil below `threshold`, nev growing from initial_nev by x1.3 (the reference's code) up to
 * max_nev (= the reference's x.size(); at nev <= 3, where int(nev * 1.3) == nev would repeat the same
 * solve forever in the reference, by one); one factorisation of A - sigma B for all passes.  Outputs
 * as eig_shift_invert_solve for the final nev (*nev_out; eval_host / evec_host sized for max_nev):
 * ascending, the last one >= threshold unless nev reached max_nev.  maxit_per_nev: restarts allowed
 * per eigenvalue (the reference's nIterationsMax_; <= 0: 100 nev). */
int eig_shift_invert_adaptive(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double sigma, double threshold, int initial_nev,
                              int max_nev, double tol, int maxit_per_nev, unsigned seed, double *eval_host,
                              double *evec_host, int *nev_out, int *passes);
/* Non-symmetric modes (arpack_geneo_wrapper.hh:428-578), nev eigenvalues of A x = lambda B x nearest
 * sigma ("LM" on OP = (A - sigma B)^-1 B, B = NULL: identity), by Arnoldi with Krylov-Schur restarts
 * (CGS2 per step; the projected matrix's eigenproblem on the host):
 *   EIG_ARNOLDI_STD = computeStdNonSymMinMagnitude (:428-499, ARNonSymStdEig): Euclidean inner
 *                     product, lambda = sigma + 1 / Re(nu) (the reference unshifts the real part);
 *   EIG_ARNOLDI_GEN = computeGenNonSymShiftInvertMinMagnitude (:502-578, ARNonSymGenEig, real
 *                     shift-invert mode): B-inner product, start vector in range(OP), lambda =
 *                     sigma + 1 / nu.
 * eval_re[nev] ascending (both modes sort by the real part, :484-498 / :556-571), eval_im[nev] (or
 * NULL) the imaginary parts; evec_host nev x n (or NULL): unit 2-norm eigenvectors, for a complex
 * conjugate pair ARPACK's raw storage (the real part of the eigenvector of the member with
 * Im nu > 0, the imaginary part for its partner).  ncv = 0: min(n, max(2 nev + 1, 20)) (needs
 * nev + 2 <= ncv); tol = 0: machine precision; maxit = 0: 100 nev restarts.  Converged when
 * ||f|| |c^T y_i| <= tol |nu_i| for the nev wanted Ritz pairs.  The LU of A - sigma B is computed on
 * the host unless `lu` is given. */
enum { EIG_ARNOLDI_STD = 0, EIG_ARNOLDI_GEN = 1 };
int eig_arnoldi_shift_invert(eig_mat_t A, eig_mat_t B, eig_lu_t lu, double sigma, int nev, int ncv, double tol,
                             int maxit, unsigned seed, int mode, double *eval_re, double *eval_im, double *evec_host,
                             int *restarts);

/* ---------------------------------------------------------------- block Lanczos (config C5) */
/* Generalised symmetric-definite eigenproblem K x = lambda M x by block Lanczos in the M-inner
 * product on the operator M^-1 K (the pencil GeneralizedInverse solves, eigensolver.hh:204-351,
 * and ARPACK's computeGenSymShiftInvertMinMagnitude, arpack_geneo_wrapper.hh:581-658; both need a
 * sparse LU that does not exist at C5's size).  Per step j (block size b, basis V_0..V_j):
 *   W = K V_j,  A_j = V_j^T W;  Z = M^-1 W by `degree` Chebyshev-Jacobi steps on the spectrum
 *   bounds [lmin, lmax] of diag(M)^-1 M (P1 tetrahedra: [0.5, 2.5], Wathen's element bound; the
 *   solve has no reductions);  two classical Gram-Schmidt passes of Z against V_0..V_j in the
 *   M-inner product (panel V^T (M Z) on MFMA);  CholQR2:  Z = V_{j+1} B_{j+1}.
 * K and M: same rows / column window (shared pattern, e.g. eig_gen kinds 6 and 7), 1x1 blocks;
 * with a communicator, row-partitioned (eig_mat_create_bcsr_dist) and every panel allreduced.
 * The start block is mt19937(seed) normal numbers in MultiVector fill order (eigensolver.hh:49-55). */
typedef struct eig_blanczos_s *eig_blanczos_t;
typedef struct eig_blanczos_timing {
  double total_ms;   /* device time of the step batch (events, first to last) */
  double kspmm_ms;   /* W = K V_j + the A_j Gram */
  double cheb_ms;    /* the Chebyshev mass solve (degree - 1 fused M SpMM steps) */
  double orth_ms;    /* two CGS passes: M SpMM + MFMA panel Gram + panel update */
  double norm_ms;    /* CholQR2: 2 x (M SpMM + Gram + host 32x32 Cholesky + triangular update) */
  int64_t steps;
  int64_t cheb_launches; /* fused Chebyshev kernel launches (one per 32 columns per Chebyshev step) */
  int64_t cholqr_recomputed; /* CholQR2 second passes (since creation) that recomputed M Z because the
                                first pass's R was ill-conditioned (diagonal spread > 1e4) */
} eig_blanczos_timing;
int eig_blanczos_create(eig_mat_t K, eig_mat_t M, int block, int max_steps, int degree, double lmin, double lmax,
                        unsigned seed, eig_blanczos_t *ws);
/* Spectral transformation: the operator (K - sigma M)^-1 M (ARPACK mode 3, arpack_geneo_wrapper.hh:
 * 581-658) for the end of the pencil nearest sigma -- the smallest eigenvalues GeneralizedInverse
 * (eigensolver.hh:204-351) returns for sigma below the spectrum.  Ks = K - sigma M (K for sigma = 0),
 * solved by `degree` Chebyshev-Jacobi steps with spec(diag(Ks)^-1 Ks) in [lmin, lmax].
 * eig_blanczos_ritz then returns lambda = sigma + 1 / theta for the nev theta of largest |theta|,
 * ascending (EIG_WHICH_SA) or descending (EIG_WHICH_LA). */
int eig_blanczos_create_si(eig_mat_t K, eig_mat_t M, eig_mat_t Ks, double sigma, int block, int max_steps, int degree,
                           double lmin, double lmax, unsigned seed, eig_blanczos_t *ws);
/* Geometric multigrid for a matrix on an nx x ny x nz box grid (lexicographic rows k = (z ny + y) nx
 * + x; 1x1 blocks, one rank; every entry within one grid step per direction, e.g. the 7-point and P1
 * Kuhn stencils): coarse grids keep the nodes of odd index per direction, trilinear P, Galerkin
 * P^T A P on the host (27-point, bitwise symmetric), Chebyshev-Jacobi smoothing of degree
 * smooth_degree on [lmax / smooth_ratio, lmax] (lmax = Gershgorin bound of diag(A)^-1 A), the
 * coarsest level (<= 64 rows) solved to 1e-15 by Chebyshev on its exact spectrum.  max_cols: the
 * widest multivector a solve takes (workspace: 6 x rows x max_cols doubles per level). */
typedef struct eig_mg_s *eig_mg_t;
int eig_mg_create(eig_mat_t A, int nx, int ny, int nz, int max_cols, int smooth_degree, double smooth_ratio,
                  eig_mg_t *mg);
int eig_mg_info(eig_mg_t mg, int *levels, int64_t *coarse_rows, int *coarse_degree, double *lmax_fine);
/* X = S B, m columns (window layout = plain MultiVector<double,8> on one rank), S = `cycles`
 * stationary iterations x += V (b - A x) from x = 0 with V one symmetric V-cycle: a fixed symmetric
 * linear operator (no inner products inside).  resid_host (or NULL): max over the columns of
 * ||B - A X|| / ||B|| afterwards (a measurement; synchronous either way).  X must not alias B. */
int eig_mg_solve(eig_mg_t mg, int64_t m, const double *B, double *X, int cycles, double *resid_host);
int eig_mg_destroy(eig_mg_t mg);
/* eig_blanczos_create_si with the Ks solve by `cycles` multigrid iterations (mg built on Ks with
 * max_cols >= block) instead of Chebyshev-Jacobi -- the smallest end of the pencil at 256^3, where
 * kappa(diag(K)^-1 K) ~ 2.7e4 would need ~2,500 Chebyshev steps per application. */
int eig_blanczos_create_si_mg(eig_mat_t K, eig_mat_t M, eig_mat_t Ks, double sigma, eig_mg_t mg, int cycles, int block,
                              int max_steps, unsigned seed, eig_blanczos_t *ws);
int eig_blanczos_step(eig_blanczos_t ws, int steps, eig_blanczos_timing *timing);
/* Ritz pairs of the k steps taken: eval_host[nev] (LA descending / SA ascending), evec_host: nev
 * owned-row vectors with y^T M y = 1 (or NULL), resid_host[nev]: ||K y - theta M y||_2 (or NULL). */
int eig_blanczos_ritz(eig_blanczos_t ws, int nev, int which, double *eval_host, double *evec_host, double *resid_host);
/* The block tridiagonal T (dim = steps * block; T_host dim x dim row-major, or NULL for the size). */
int eig_blanczos_tmatrix(eig_blanczos_t ws, int *dim, double *T_host);
int eig_blanczos_destroy(eig_blanczos_t ws);
/* X = M^-1 B for m columns (window layout) by `degree` Chebyshev-Jacobi steps (the operator's solve);
 * X must not alias B (EIG_ERR_ARG). */
int eig_mass_solve_mv8(eig_mat_t M, int64_t m, int degree, double lmin, double lmax, const double *B, double *X);
/* Tall-skinny panel kernels on n-row MultiVector<double,8> buffers (single rank):
 * Y = beta Y + alpha Q S (Q n x m1, S m1 x m2 row-major device, m2 in {8,16,24,32}; Y may be Q), and
 * G = Q1^T Q2 (m1 x m2 row-major device) on MFMA with a deterministic two-stage reduction. */
int eig_panel_update_mv8(eig_ctx_t ctx, int64_t n, int64_t m1, int64_t m2, const double *Q, const double *S,
                         double alpha, double beta, double *Y);
int eig_panel_gram_mv8(eig_ctx_t ctx, int64_t n, int64_t m1, int64_t m2, const double *Q1, const double *Q2, double *G);

/* a14: the reference's analytic GS models (kernels_cpp.hh:98-116, :157-175). */
double eig_flops_orthonormalize(int64_t n, int64_t m);
double eig_bytes_orthonormalize_blocked(int64_t n, int64_t m, int b);

/* ---------------------------------------------------------------- generators --------------- */
/* Synthetic matrices of the reference harness (src/dune-eigensolver.cc:98-156) and SURVEY 8(d),
 * produced on the host into caller buffers (sizes from the *_nnz functions).  kind:
 *   0 2-D Dirichlet 5-pt N*N (setupLaplacian)      1 2-D Neumann (.cc:105-121)
 *   2 2-D partition-of-unity B (.cc:124-143)       3 2-D identity pattern (.cc:145-156)
 *   4 3-D Poisson 7-pt N^3                          5 3-D Q1 "elasticity" L_Q1 (x) C, 3x3 blocks
 *   6 3-D P1 stiffness K, Kuhn 6-tet split, N^3     7 3-D P1 consistent mass M, same 15-pt pattern
 *     interior nodes, h = 1/(N+1) (config C5)            (pattern(K) == pattern(M), config C5)
 *   8 3-D 7-pt variable-coefficient diffusion N^3: kind 4's pattern, a hashed conductance in
 *     [0.5, 1.5) per grid edge (bitwise symmetric), diagonal = the six face conductances' sum
 *   9 / 10 the P1 K / M of kinds 6 / 7 with a hashed coefficient in [0.5, 1.5) per tetrahedron
 *     (bitwise symmetric; the C5 variable-coefficient variant) */
int64_t eig_gen_nnzb(int kind, int N);
int eig_gen_matrix(int kind, int N, int overlap, int64_t *rowptr, int32_t *col, double *vals);
/* Rows [row_begin, row_begin + nrows) of the same matrix (for eig_mat_create_bcsr_dist). */
int64_t eig_gen_nnzb_rows(int kind, int N, int64_t row_begin, int64_t nrows);
int eig_gen_matrix_rows(int kind, int N, int64_t row_begin, int64_t nrows, int64_t *rowptr,
                        int32_t *col, double *vals);

/* ---------------------------------------------------------------- Matrix Market ---------- */
/* Host reordering for imported (unstructured) matrices: reverse Cuthill-McKee of the symmetrised
 * pattern of an n x n CSR matrix, perm[k] = old row of new row k (pseudo-peripheral start per
 * component, neighbours by increasing degree); and B = P A P^T (B[k][l] = A[perm[k]][perm[l]]) with
 * each row's columns ascending.  Output arrays sized like the input (rowptr n+1, col / vals nnz). */
int eig_reorder_rcm(int64_t n, const int64_t *rowptr, const int32_t *col, int64_t *perm);
int eig_permute_symmetric(int64_t n, const int64_t *rowptr, const int32_t *col, const double *vals,
                          const int64_t *perm, int64_t *rowptr_out, int32_t *col_out, double *vals_out);

/* Import / export of real matrices in Matrix Market coordinate form (the format
 * Dune::storeMatrixMarket writes), host-only.  Read: real | integer | pattern, general | symmetric
 * (mirrored), 1-based, duplicates summed, columns ascending; br > 1 groups the scalar entries into
 * br x br blocks (row-major FieldMatrix layout) -> arrays for eig_mat_create_bcsr.  Sizes first
 * with eig_mm_read_info (rowptr nb_rows+1, col nnzb, vals nnzb*br*br).  Write: every stored scalar
 * of the blocks (symmetric != 0: the lower triangle only, header "symmetric"). */
int eig_mm_read_info(const char *path, int br, int64_t *nb_rows, int64_t *nb_cols, int64_t *nnzb);
int eig_mm_read(const char *path, int br, int64_t *rowptr, int32_t *col, double *vals);
int eig_mm_write(const char *path, int64_t nb_rows, int64_t nb_cols, int br, int bc, const int64_t *rowptr,
                 const int32_t *col, const double *vals, int symmetric);

/* ---------------------------------------------------------------- partition planning ------ */
/* Host-only helpers (no device needed) used by eig_mat_create_bcsr_dist; exported so the
 * partition / halo logic can be exercised and reused by other front ends.
 * eig_plan_window: from a rank's rows (global block columns) compute
 *   out[0] = window begin (global BLOCK column of window index 0, padded so that the owned rows
 *            start at a multiple of 8 scalar entries), out[1] = window length (scalar, multiple
 *            of 8), out[2] = own_offset (scalar), out[3] = cmin, out[4] = cmax (referenced block
 *            columns [cmin, cmax) including the owned rows).
 * eig_plan_halo: given every rank's (row_begin, nb_local, cmin, cmax) in ranks[4*nranks], list
 *   what rank `me` receives (recv[3*k] = peer, offset in the window (scalar), count) and sends
 *   (send[3*k] = peer, offset in the window of the owned rows, count); *nrecv / *nsend entries. */
int eig_plan_window(int64_t row_begin, int64_t nb_local, int bc, const int64_t *rowptr_host,
                    const int32_t *col_host, int64_t out[5]);
int eig_plan_halo(int nranks, int me, const int64_t *ranks, int bc, int64_t win_begin_blk,
                  int64_t *recv, int *nrecv, int64_t *send, int *nsend);

#ifdef __cplusplus
}
#endif
#endif /* EIGMI_H */
