"""Python binding of libeigmi's C ABI (include/eigmi.h) -- the ctypes stub a maintainer would
add on the reference side, plus thin host-side helpers for tests and the benchmark.

The compute path is libeigmi.so (hand-written HIP for gfx950).  Loading fails loudly when the
library is missing; there is no CPU fallback in this module.
"""
import atexit
import ctypes
import itertools
import os
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# EIGMI_LIB_VARIANT=san loads the host-sanitizer build (make sanitize; tests/test_sanitize.py only)
LIB_PATH = os.path.join(_HERE, "lib", "libeigmi_san.so" if os.environ.get("EIGMI_LIB_VARIANT") == "san"
                        else "libeigmi.so")

EIG_OK, EIG_ERR_SHAPE, EIG_ERR_BLOCKSIZE, EIG_ERR_HIP, EIG_ERR_RCCL, EIG_ERR_BREAKDOWN, EIG_ERR_ARG, EIG_ERR_NODEVICE = range(8)
ORTHO_MGS, ORTHO_CHOLQR, ORTHO_CHOLQR_SPLIT = 0, 1, 2
ORTHO_GRID = 0x100  # or-ed into the variant: grid-wide MGS passes even for blocks one workgroup holds
ORTHO_NO_COOP = 0x200  # or-ed into the variant: look-ahead MGS as 9 launches (no in-kernel fallback passes)
ORTHO_ONE_WG = 0x400  # or-ed into ORTHO_MGS: the one-workgroup MGS for n <= 4096 (slower than the default; A/B)


def ORTHO_LOOKAHEAD(L):
    """or-ed into ORTHO_MGS: at most L steps per read pass of the diagonal block (include/eigmi.h)"""
    return int(L) << 12

# matrix kernel-image flags (eig_mat_create_bcsr_ex)
MAT_NO_BAND, MAT_BAND_GATHER, MAT_NO_STENCIL, MAT_NO_MARCH, MAT_NO_CLASS, MAT_NO_UNIFORM = 1, 2, 4, 8, 16, 32
# triangular-solve kernels of an LU (eig_lu_set_solver)
TRSV_AUTO, TRSV_BLOCKINV, TRSV_STAGED, TRSV_CSR = 0, 1, 2, 3
TRSV_KINDS = {None: TRSV_AUTO, "auto": TRSV_AUTO, "blockinv": TRSV_BLOCKINV, "staged": TRSV_STAGED, "csr": TRSV_CSR}
COMM_MAILBOX = 1
COMM_ALWAYS = 2  # collectives through RCCL even at one rank (eig_comm_init_ex)
STREAM_COPY_MODE = 3  # eig_stream_copy_timed: nontemporal, full grid -- 6.70 TB/s vs 6.28 plain (tools/copy_sweep.py)
WHICH_LA, WHICH_SA = 0, 1
LANCZOS_TIME_KERNELS = 1
LANCZOS_TIME_DETAIL = 2
LANCZOS_FUSED = 4
LANCZOS_PIPELINED = 8
LANCZOS_AUTO = 16
IPC_HANDLE_BYTES = 64
MARCH_2L_MIN_ROWS = 4194304  # EIG_MARCH_2L_MIN_ROWS: owned rows from which the fused step marches line pairs
ALLREDUCE_KINDS = {0: "none", 1: "rccl", 2: "xgmi-mailbox", 3: "loopback", 4: "xgmi-mailbox-step"}


def _tflags(timed):
    """timed: False | True (fused-SpMV events) | "detail" (+ update / allreduce boundaries)."""
    if timed == "detail":
        return LANCZOS_TIME_KERNELS | LANCZOS_TIME_DETAIL
    return LANCZOS_TIME_KERNELS if timed else 0


GEN_LAPLACE2D, GEN_NEUMANN2D, GEN_PU2D, GEN_IDENTITY2D, GEN_POISSON3D, GEN_Q1ELAST3D, GEN_P1STIFF3D, GEN_P1MASS3D, \
    GEN_VARCOEF3D, GEN_P1STIFF3D_VAR, GEN_P1MASS3D_VAR = range(11)


class EigError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class EigShapeError(EigError, ValueError):
    """SHAPE / BLOCKSIZE errors: the reference throws std::invalid_argument for these."""


class _MatInfo(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in ("n", "n_global", "ncols", "row_begin", "window", "own_offset", "nnzb",
                                              "nnzb_padded", "nslices")] + \
               [("br", ctypes.c_int), ("bc", ctypes.c_int)] + \
               [(k, ctypes.c_int64) for k in ("halo_recv", "halo_send", "device_bytes", "stencil_slices",
                                              "rows_per_lane", "sym_offsets", "sym_arrays",
                                              "sym_mask_bytes", "sym_uniform", "sym_geo",
                                              "march_variant", "march_variant_mv")]


class BlockTiming(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in ("total_ms", "kspmm_ms", "cheb_ms", "orth_ms", "norm_ms")] + \
               [("steps", ctypes.c_int64), ("cheb_launches", ctypes.c_int64), ("cholqr_recomputed", ctypes.c_int64)]


class Timing(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("spmv_ms", ctypes.c_double), ("update_ms", ctypes.c_double),
                ("comm_ms", ctypes.c_double), ("spmv_launches", ctypes.c_int64)]


_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_dbl = ctypes.c_double
_u = ctypes.c_uint

# name -> (restype, argtypes); this is the complete exported surface of include/eigmi.h
SIGNATURES = {
    "eig_ctx_create": (_int, [_int, ctypes.POINTER(_vp)]),
    "eig_ctx_destroy": (_int, [_vp]),
    "eig_last_error": (ctypes.c_char_p, [_vp]),
    "eig_ctx_sync": (_int, [_vp]),
    "eig_ctx_stream": (_int, [_vp, ctypes.POINTER(_vp)]),
    "eig_device_count": (_int, [ctypes.POINTER(_int)]),
    "eig_version": (ctypes.c_char_p, []),
    "eig_comm_unique_id": (_int, [ctypes.c_char_p]),
    "eig_comm_init": (_int, [_vp, _int, _int, ctypes.c_char_p]),
    "eig_comm_init_ex": (_int, [_vp, _int, _int, ctypes.c_char_p, _int]),
    "eig_comm_allreduce_sum": (_int, [_vp, _vp, _i64]),
    "eig_comm_barrier": (_int, [_vp]),
    "eig_loopback_create": (_int, [_int, ctypes.POINTER(_vp)]),
    "eig_loopback_destroy": (_int, [_vp]),
    "eig_comm_init_loopback": (_int, [_vp, _vp, _int]),
    "eig_comm_loopback_mailbox": (_int, [_vp]),
    "eig_comm_ipc_handle": (_int, [_vp, _int, _int, ctypes.c_char_p]),
    "eig_comm_ipc_open": (_int, [_vp, ctypes.c_char_p]),
    "eig_comm_ipc_open_ex": (_int, [_vp, ctypes.c_char_p, _int]),
    "eig_comm_info": (_int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_int), ctypes.POINTER(_int),
                             ctypes.POINTER(_int)]),
    "eig_comm_counters": (_int, [_vp, ctypes.POINTER(_i64)]),
    "eig_comm_select_allreduce": (_int, [_vp, _int]),
    "eig_comm_select_halo": (_int, [_vp, _int]),
    "eig_malloc": (_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "eig_free": (_int, [_vp, _vp]),
    "eig_memcpy_h2d": (_int, [_vp, _vp, _vp, ctypes.c_size_t]),
    "eig_memcpy_d2h": (_int, [_vp, _vp, _vp, ctypes.c_size_t]),
    "eig_memcpy_d2d": (_int, [_vp, _vp, _vp, ctypes.c_size_t]),
    "eig_memset": (_int, [_vp, _vp, _int, ctypes.c_size_t]),
    "eig_mat_create_bcsr": (_int, [_vp, _i64, _i64, _int, _int, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    "eig_mat_create_bcsr_dist": (_int, [_vp, _i64, _i64, _i64, _int, _int, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    "eig_mat_create_bcsr_ex": (_int, [_vp, _i64, _i64, _int, _int, _vp, _vp, _vp, _int, ctypes.POINTER(_vp)]),
    "eig_mat_create_bcsr_dist_ex": (_int, [_vp, _i64, _i64, _i64, _int, _int, _vp, _vp, _vp, _int,
                                           ctypes.POINTER(_vp)]),
    "eig_lu_set_solver": (_int, [_vp, _int]),
    "eig_lu_solver_info": (_int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "eig_shift_invert_adaptive": (_int, [_vp, _vp, _vp, _dbl, _dbl, _int, _int, _dbl, _int, _u, _vp, _vp,
                                         ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "eig_arnoldi_shift_invert": (_int, [_vp, _vp, _vp, _dbl, _int, _int, _dbl, _int, _u, _int, _vp, _vp, _vp,
                                        ctypes.POINTER(_int)]),
    "eig_reorder_rcm": (_int, [_i64, _vp, _vp, _vp]),
    "eig_permute_symmetric": (_int, [_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "eig_mat_destroy": (_int, [_vp]),
    "eig_mat_get_info": (_int, [_vp, ctypes.POINTER(_MatInfo)]),
    "eig_mat_shift_diag": (_int, [_vp, _dbl]),
    "eig_mat_tune": (_int, [_vp, _int, _int]),
    "eig_fill_normal": (_int, [_vp, _i64, _u, _vp]),
    "eig_lanczos_kernel_info": (_int, [_vp, _int, ctypes.c_char_p, _int, ctypes.POINTER(_i64)]),
    "eig_mat_kernel_info": (_int, [_vp, _int, ctypes.c_char_p, _int]),
    "eig_mv": (_int, [_vp, _vp, _vp]),
    "eig_mv_host": (_int, [_vp, _vp, _vp]),
    "eig_mv_timed": (_int, [_vp, _vp, _vp, _int, ctypes.POINTER(_dbl)]),
    "eig_dot": (_int, [_vp, _i64, _vp, _vp, _vp]),
    "eig_nrm2": (_int, [_vp, _i64, _vp, _vp]),
    "eig_axpy": (_int, [_vp, _i64, _dbl, _vp, _vp]),
    "eig_scal": (_int, [_vp, _i64, _dbl, _vp]),
    "eig_copy": (_int, [_vp, _i64, _vp, _vp]),
    "eig_lanczos_update": (_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "eig_spmm_dot_gram_mv8": (_int, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "eig_orthonormalize_gram_mv8": (_int, [_vp, _i64, _i64, _vp, _vp]),
    "eig_stream_copy_timed": (_int, [_vp, _i64, _vp, _vp, _int, _int, ctypes.POINTER(_dbl)]),
    "eig_spmm_mv8": (_int, [_vp, _i64, _vp, _vp]),
    "eig_dot_diag_mv8": (_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "eig_gram_mv8": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp]),
    "eig_orthonormalize_mv8": (_int, [_vp, _i64, _i64, _vp, _int]),
    "eig_orthonormalize_passes": (_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    "eig_orthonormalize_naive": (_int, [_vp, _i64, _i64, _vp]),
    "eig_b_orthonormalize_mv8": (_int, [_vp, _i64, _vp, _vp]),
    "eig_random_mv8": (_int, [_vp, _i64, _i64, _u, _vp]),
    "eig_random_normal": (_int, [_i64, _u, _vp]),
    "eig_standard_largest": (_int, [_vp, _dbl, _dbl, _int, _int, _u, _vp, _vp, ctypes.POINTER(_int), _int]),
    "eig_lanczos_run": (_int, [_vp, _int, _vp, _u, _int, _vp, _vp, ctypes.POINTER(Timing)]),
    "eig_lanczos_solve": (_int, [_vp, _int, _int, _int, _u, _vp, _vp, _vp]),
    "eig_lanczos_create": (_int, [_vp, _int, _vp, _u, ctypes.POINTER(_vp)]),
    "eig_lanczos_create_ex": (_int, [_vp, _int, _vp, _u, _int, ctypes.POINTER(_vp)]),
    "eig_lanczos_step": (_int, [_vp, _int, _int, ctypes.POINTER(Timing)]),
    "eig_lanczos_tridiag": (_int, [_vp, ctypes.POINTER(_int), _vp, _vp]),
    "eig_lanczos_destroy": (_int, [_vp]),
    "eig_lanczos_info": (_int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "eig_lanczos_capture": (_int, [_vp, _int, _int, ctypes.POINTER(_int)]),
    "eig_lanczos_ws_info": (_int, [_vp, ctypes.POINTER(_int), ctypes.c_char_p, _int, ctypes.POINTER(_i64)]),
    "eig_lanczos_replay": (_int, [_vp, ctypes.POINTER(Timing)]),
    "eig_lu_create": (_int, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _int, ctypes.POINTER(_vp)]),
    "eig_lu_create_bcsr": (_int, [_vp, _i64, _int, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    "eig_lu_info": (_int, [_vp, ctypes.POINTER(_i64), ctypes.POINTER(_i64), ctypes.POINTER(_i64), ctypes.POINTER(_int)]),
    "eig_lu_export": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "eig_lu_destroy": (_int, [_vp]),
    "eig_inverse_mv8": (_int, [_vp, _i64, _vp, _vp]),
    "eig_standard_inverse": (_int, [_vp, _vp, _dbl, _dbl, _int, _int, _u, _vp, _vp, ctypes.POINTER(_int), _int]),
    "eig_generalized_inverse": (_int, [_vp, _vp, _vp, _dbl, _dbl, _dbl, _int, _int, _u, _vp, _vp, ctypes.POINTER(_int),
                                       _int]),
    "eig_shift_invert_solve": (_int, [_vp, _vp, _vp, _dbl, _int, _int, _dbl, _int, _u, _vp, _vp, ctypes.POINTER(_int)]),
    "eig_shift_invert_solve_ex": (_int, [_vp, _vp, _vp, _dbl, _int, _int, _dbl, _int, _u, _vp, _vp,
                                         ctypes.POINTER(_int), _int]),
    "eig_blanczos_create": (_int, [_vp, _vp, _int, _int, _int, _dbl, _dbl, _u, ctypes.POINTER(_vp)]),
    "eig_blanczos_create_si": (_int, [_vp, _vp, _vp, _dbl, _int, _int, _int, _dbl, _dbl, _u, ctypes.POINTER(_vp)]),
    "eig_blanczos_step": (_int, [_vp, _int, ctypes.POINTER(BlockTiming)]),
    "eig_mg_create": (_int, [_vp, _int, _int, _int, _int, _int, _dbl, ctypes.POINTER(_vp)]),
    "eig_mg_info": (_int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_i64), ctypes.POINTER(_int),
                           ctypes.POINTER(_dbl)]),
    "eig_mg_solve": (_int, [_vp, _i64, _vp, _vp, _int, ctypes.POINTER(_dbl)]),
    "eig_mg_destroy": (_int, [_vp]),
    "eig_blanczos_create_si_mg": (_int, [_vp, _vp, _vp, _dbl, _vp, _int, _int, _int, _u, ctypes.POINTER(_vp)]),
    "eig_blanczos_ritz": (_int, [_vp, _int, _int, _vp, _vp, _vp]),
    "eig_blanczos_tmatrix": (_int, [_vp, ctypes.POINTER(_int), _vp]),
    "eig_blanczos_destroy": (_int, [_vp]),
    "eig_mass_solve_mv8": (_int, [_vp, _i64, _int, _dbl, _dbl, _vp, _vp]),
    "eig_panel_update_mv8": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _dbl, _dbl, _vp]),
    "eig_panel_gram_mv8": (_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp]),
    "eig_flops_orthonormalize": (_dbl, [_i64, _i64]),
    "eig_bytes_orthonormalize_blocked": (_dbl, [_i64, _i64, _int]),
    "eig_gen_nnzb": (_i64, [_int, _int]),
    "eig_gen_matrix": (_int, [_int, _int, _int, _vp, _vp, _vp]),
    "eig_gen_nnzb_rows": (_i64, [_int, _int, _i64, _i64]),
    "eig_gen_matrix_rows": (_int, [_int, _int, _i64, _i64, _vp, _vp, _vp]),
    "eig_mm_read_info": (_int, [ctypes.c_char_p, _int, ctypes.POINTER(_i64), ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    "eig_mm_read": (_int, [ctypes.c_char_p, _int, _vp, _vp, _vp]),
    "eig_mm_write": (_int, [ctypes.c_char_p, _i64, _i64, _int, _int, _vp, _vp, _vp, _int]),
    "eig_plan_window": (_int, [_i64, _i64, _int, _vp, _vp, _vp]),
    "eig_plan_halo": (_int, [_int, _int, _vp, _int, _i64, _vp, ctypes.POINTER(_int), _vp, ctypes.POINTER(_int)]),
}


def load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libeigmi.so not built ({LIB_PATH}); run `make -C dune-eigensolver_amd` "
                          "or __graft_entry__.build() -- there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = load()

# Every live handle, so that an interpreter exit releases them while the HIP runtime (and a
# profiler's API hooks) are still up: Python's atexit handlers run before the C runtime's exit
# handlers, whereas a module-global Context would otherwise be finalised in any order relative to
# libamdhip64's own teardown (an exit-time SIGSEGV under rocprofv3 --kernel-trace, round 5).
_LIVE = weakref.WeakValueDictionary()
_SEQ = itertools.count()


def _track(obj):
    _LIVE[next(_SEQ)] = obj


@atexit.register
def release_all():
    """Destroy every handle still alive: newest first, contexts last (eig_ctx_destroy after every
    matrix / workspace / buffer of that context), then wait for the device."""
    objs = [o for _, o in sorted(_LIVE.items(), key=lambda kv: kv[0], reverse=True)]
    for o in objs:
        if not isinstance(o, Context):
            try:
                (o.free if isinstance(o, DeviceArray) else o.close)()
            except Exception:
                pass
    for o in objs:
        if isinstance(o, Context):
            try:
                o.close()
            except Exception:
                pass


def build_id():
    """Identity of the kernel sources the loaded library was built from: sha1 over csrc/ (the .hip
    kernels, host .cpp and headers) -- bench lines and committed PMC summaries carry it, so a
    summary is matched to the build it measured."""
    import hashlib
    h = hashlib.sha1()
    src = os.path.join(_HERE, "csrc")
    for f in sorted(os.listdir(src)):
        if f.endswith((".hip", ".cpp", ".h")):
            h.update(f.encode())
            with open(os.path.join(src, f), "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:12]


def _np_ptr(a):
    return a.ctypes.data_as(_vp)


def device_count():
    c = _int(0)
    lib.eig_device_count(ctypes.byref(c))
    return c.value


class Context:
    """eig_ctx_t: one GPU, one HIP stream, optional RCCL communicator."""

    def __init__(self, device=0):
        h = _vp()
        rc = lib.eig_ctx_create(device, ctypes.byref(h))
        if rc != EIG_OK:
            raise EigError(rc, lib.eig_last_error(None).decode())
        self.h = h
        self.device = device
        self.nranks, self.rank = 1, 0
        _track(self)

    def check(self, rc):
        if rc != EIG_OK:
            msg = lib.eig_last_error(self.h).decode()
            if rc in (EIG_ERR_SHAPE, EIG_ERR_BLOCKSIZE):
                raise EigShapeError(rc, msg)
            raise EigError(rc, msg)

    def close(self):
        if self.h:
            lib.eig_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        self.check(lib.eig_ctx_sync(self.h))

    # --- communicator
    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(128)
        rc = lib.eig_comm_unique_id(buf)
        if rc != EIG_OK:
            raise EigError(rc, lib.eig_last_error(None).decode())
        return buf.raw

    def comm_init(self, nranks, rank, uid, mailbox=False, always=False):
        """RCCL communicator (ncclAllReduce for dots); mailbox=True also sets up the xGMI mailbox
        allreduce (eig_comm_init_ex, EIG_COMM_MAILBOX); always=True routes the collectives through
        RCCL even at nranks == 1 (EIG_COMM_ALWAYS: the one-GPU rehearsal of the transport)."""
        flags = (COMM_MAILBOX if mailbox else 0) | (COMM_ALWAYS if always else 0)
        self.check(lib.eig_comm_init_ex(self.h, nranks, rank, uid, flags))
        self.nranks, self.rank = nranks, rank

    def comm_init_loopback(self, hub, rank, mailbox=False):
        """Attach this context as virtual rank `rank` of a loopback hub (eig_comm_init_loopback; halo
        and allreduce by device copies + a host barrier).  mailbox=True: also the in-process xGMI
        mailbox between the virtual ranks (eig_comm_loopback_mailbox, a collective of all ranks)."""
        self.check(lib.eig_comm_init_loopback(self.h, hub, rank))
        if mailbox:
            self.check(lib.eig_comm_loopback_mailbox(self.h))
        info = self.comm_info()
        self.nranks, self.rank = info["nranks"], info["rank"]

    def comm_loopback_mailbox(self):
        self.check(lib.eig_comm_loopback_mailbox(self.h))

    def comm_counters(self):
        """Collectives the library has enqueued on its communicators (eig_comm_counters)."""
        v = (_i64 * 4)()
        self.check(lib.eig_comm_counters(self.h, v))
        return {"allreduce": v[0], "allreduce_split": v[1], "halo_groups": v[2], "p2p": v[3]}

    def barrier(self):
        self.check(lib.eig_comm_barrier(self.h))

    def ipc_handle(self, nranks, rank):
        """Export this rank's xGMI mailbox (64 bytes); see eig_comm_ipc_handle."""
        buf = ctypes.create_string_buffer(IPC_HANDLE_BYTES)
        self.check(lib.eig_comm_ipc_handle(self.h, nranks, rank, buf))
        return buf.raw

    def ipc_open(self, handles, always=False):
        """handles: the nranks exported handles concatenated in rank order; always: collectives through
        the mailbox even at one rank (eig_comm_ipc_open_ex EIG_COMM_ALWAYS)."""
        self.check(lib.eig_comm_ipc_open_ex(self.h, bytes(handles), COMM_ALWAYS if always else 0))
        info = self.comm_info()
        self.nranks, self.rank = info["nranks"], info["rank"]

    def allreduce_sum(self, arr, count=None):
        self.check(lib.eig_comm_allreduce_sum(self.h, arr.ptr, arr.n if count is None else count))

    def select_allreduce(self, kind):
        """eig_comm_select_allreduce: "rccl", "mailbox" or "mailbox-step" (the mailbox, and the fused
        Lanczos step's sums exchanged inside the step kernel); the mailbox kinds need it set up and
        validated (comm_init(mailbox=True) or ipc_open); every rank must select the same."""
        self.check(lib.eig_comm_select_allreduce(self.h, {"rccl": 1, "mailbox": 2, "mailbox-step": 4}[kind]))

    def select_halo(self, kind):
        """eig_comm_select_halo: "rccl" (ncclSend / ncclRecv) or "mailbox" (the halo mailbox); every rank
        must select the same."""
        self.check(lib.eig_comm_select_halo(self.h, {"rccl": 1, "mailbox": 2}[kind]))

    def comm_info(self):
        v = [_int(0) for _ in range(4)]
        self.check(lib.eig_comm_info(self.h, *[ctypes.byref(x) for x in v]))
        return {"nranks": v[0].value, "rank": v[1].value, "allreduce": ALLREDUCE_KINDS[v[2].value],
                "mailbox_errors": v[3].value}

    # --- memory
    def empty(self, n):
        return DeviceArray(self, n)

    def array(self, host):
        host = np.ascontiguousarray(host, dtype=np.float64)
        d = DeviceArray(self, host.size)
        d.upload(host)
        return d

    def zeros(self, n):
        d = DeviceArray(self, n)
        self.check(lib.eig_memset(self.h, d.ptr, 0, max(n, 1) * 8))
        return d


class DeviceArray:
    """A float64 device buffer owned by the library allocator."""

    def __init__(self, ctx, n):
        self.ctx, self.n = ctx, int(n)
        p = _vp()
        ctx.check(lib.eig_malloc(ctx.h, max(self.n, 1) * 8, ctypes.byref(p)))
        self.ptr = p
        _track(self)

    def offset(self, k):
        """Raw pointer to element k (for window / owned-slice addressing)."""
        return _vp(self.ptr.value + 8 * int(k))

    def upload(self, host, at=0):
        host = np.ascontiguousarray(host, dtype=np.float64)
        assert at + host.size <= self.n
        self.ctx.check(lib.eig_memcpy_h2d(self.ctx.h, self.offset(at), _np_ptr(host), host.size * 8))

    def get(self, count=None, at=0):
        count = self.n - at if count is None else count
        out = np.empty(count, np.float64)
        self.ctx.check(lib.eig_memcpy_d2h(self.ctx.h, _np_ptr(out), self.offset(at), count * 8))
        return out

    def free(self):
        if self.ptr is not None and self.ctx.h:
            lib.eig_free(self.ctx.h, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Matrix:
    """eig_mat_t: a BCRSMatrix<FieldMatrix<double,br,bc>> in HBM (SELL-64 image)."""

    def __init__(self, ctx, handle):
        self.ctx, self.h = ctx, handle
        _track(self)
        self.info  # noqa: B018  (validates the handle)

    @property
    def info(self):
        """eig_mat_get_info, queried now (tuning and shifts change the march variant / uniformity)."""
        info = _MatInfo()
        self.ctx.check(lib.eig_mat_get_info(self.h, ctypes.byref(info)))
        return info

    OPS = {"spmv": 0, "k1": 1, "fused": 2, "spmm8": 3, "cheb8": 4, "spmm32": 5, "cheb32": 6}

    def kernel(self, op):
        """Kernel family a whole-matrix launch of `op` ("spmv", "k1", "fused", "spmm8", "cheb8")
        picks on this image now (eig_mat_kernel_info)."""
        buf = ctypes.create_string_buffer(64)
        self.ctx.check(lib.eig_mat_kernel_info(self.h, self.OPS[op], buf, 64))
        return buf.value.decode()

    def lanczos_kernel_info(self, fused=True):
        """-> (kernel name, algorithmic HBM bytes per launch) of a whole-matrix Lanczos step launch
        on this image (eig_lanczos_kernel_info)."""
        buf = ctypes.create_string_buffer(64)
        b = _i64()
        self.ctx.check(lib.eig_lanczos_kernel_info(self.h, int(bool(fused)), buf, 64, ctypes.byref(b)))
        return buf.value.decode(), int(b.value)

    @classmethod
    def from_bcsr(cls, ctx, rowptr, col, vals, br=1, bc=1, ncols_blocks=None, flags=0):
        """flags: MAT_NO_BAND | MAT_BAND_GATHER | MAT_NO_STENCIL | MAT_NO_MARCH | MAT_NO_CLASS | MAT_NO_UNIFORM
        (eig_mat_create_bcsr_ex)."""
        rowptr = np.ascontiguousarray(rowptr, np.int64)
        col = np.ascontiguousarray(col, np.int32)
        vals = np.ascontiguousarray(vals, np.float64)
        nb = rowptr.size - 1
        nbc = nb if ncols_blocks is None else ncols_blocks
        h = _vp()
        ctx.check(lib.eig_mat_create_bcsr_ex(ctx.h, nb, nbc, br, bc, _np_ptr(rowptr), _np_ptr(col), _np_ptr(vals),
                                             int(flags), ctypes.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_rows(cls, ctx, nb_global, row_begin, rowptr, col, vals, br=1, bc=1, flags=0):
        rowptr = np.ascontiguousarray(rowptr, np.int64)
        col = np.ascontiguousarray(col, np.int32)
        vals = np.ascontiguousarray(vals, np.float64)
        h = _vp()
        ctx.check(lib.eig_mat_create_bcsr_dist_ex(ctx.h, nb_global, row_begin, rowptr.size - 1, br, bc,
                                                  _np_ptr(rowptr), _np_ptr(col), _np_ptr(vals), int(flags),
                                                  ctypes.byref(h)))
        return cls(ctx, h)

    def close(self):
        if self.h and self.ctx.h:  # a destroyed context already released the device
            lib.eig_mat_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n(self):
        return self.info.n

    def window_vector(self, owned=None):
        """Zeroed window-layout vector; `owned` (host, n) goes to the owned slice."""
        v = self.ctx.zeros(self.info.window)
        if owned is not None:
            v.upload(owned, at=self.info.own_offset)
        return v

    def owned(self, v):
        return v.get(self.info.n, at=self.info.own_offset)

    def mv(self, x, y):
        self.ctx.check(lib.eig_mv(self.h, x.ptr, y.ptr))

    def mv_timed(self, x, y, reps):
        """Average device time (ms) of `reps` back-to-back y = A x launches (HIP events)."""
        ms = _dbl(0.0)
        self.ctx.check(lib.eig_mv_timed(self.h, x.ptr, y.ptr, reps, ctypes.byref(ms)))
        return ms.value

    def mv_host(self, x):
        x = np.ascontiguousarray(x, np.float64)
        y = np.zeros(self.info.n)
        self.ctx.check(lib.eig_mv_host(self.h, _np_ptr(x), _np_ptr(y)))
        return y

    def tune(self, march_runs=None, box_segs=None, march_prefetch=None, halo_whole=None, cache=None,
             box_cols=None, box_map=None, sell_cpf=None, march_lines=None):
        """eig_mat_tune, only for the keys given (None leaves a key as it is): EIG_TUNE_MARCH_RUNS =
        plane runs per column of the plane-march kernels, EIG_TUNE_BOX_SEGS = z segments per tile
        column of the box kernels, EIG_TUNE_MARCH_PREFETCH = the geometric march variant (eigmi.h;
        0 = automatic), EIG_TUNE_HALO = distributed steps: exchange first + one launch."""
        if march_runs is not None:
            self.ctx.check(lib.eig_mat_tune(self.h, 1, int(march_runs)))
        if box_segs is not None:
            self.ctx.check(lib.eig_mat_tune(self.h, 2, int(box_segs)))
        if march_prefetch is not None:
            self.ctx.check(lib.eig_mat_tune(self.h, 3, int(march_prefetch)))
        if halo_whole is not None:  # EIG_TUNE_HALO: distributed steps, exchange first + one launch
            self.ctx.check(lib.eig_mat_tune(self.h, 4, int(halo_whole)))
        if cache is not None:  # EIG_TUNE_CACHE: cache-policy bits of the value march (measurement)
            self.ctx.check(lib.eig_mat_tune(self.h, 5, int(cache)))
        if box_cols is not None:  # EIG_TUNE_BOX_COLS: box-image kernel, 32 = k_box_mv32, 16 = k_box_mv16p
            self.ctx.check(lib.eig_mat_tune(self.h, 6, int(box_cols)))
        if box_map is not None:  # EIG_TUNE_BOX_MAP: 1 = XCD-contiguous tile map of k_box_mv32
            self.ctx.check(lib.eig_mat_tune(self.h, 7, int(box_map)))
        if sell_cpf is not None:  # EIG_TUNE_SELL_CPF: explicit slices' column prefetch (0 / 1 / 2 = auto)
            self.ctx.check(lib.eig_mat_tune(self.h, 8, int(sell_cpf)))
        if march_lines is not None:  # EIG_TUNE_MARCH_LINES: 4 = line-group mapping of the value march
            self.ctx.check(lib.eig_mat_tune(self.h, 9, int(march_lines)))

    def shift_diag(self, shift):
        self.ctx.check(lib.eig_mat_shift_diag(self.h, shift))


# --------------------------------------------------------------------------------------- ops
def dot(ctx, n, x, y, out, xo=0, yo=0):
    ctx.check(lib.eig_dot(ctx.h, n, x.offset(xo), y.offset(yo), out.ptr))


def nrm2(ctx, n, x, out, xo=0):
    ctx.check(lib.eig_nrm2(ctx.h, n, x.offset(xo), out.ptr))


def axpy(ctx, n, a, x, y):
    ctx.check(lib.eig_axpy(ctx.h, n, a, x.ptr, y.ptr))


def scal(ctx, n, a, x):
    ctx.check(lib.eig_scal(ctx.h, n, a, x.ptr))


def lanczos_update(ctx, n, alpha, beta, v, vprev, w, result):
    """eig_lanczos_update: w <- (w - alpha v) - beta vprev; result[0] = ||w||, result[1] = v.w (device
    scalars alpha / beta / result are DeviceArrays; vprev None: no beta term)."""
    ctx.check(lib.eig_lanczos_update(ctx.h, n, alpha.ptr, beta.ptr if beta is not None else None, v.ptr,
                                     vprev.ptr if vprev is not None else None, w.ptr, result.ptr))


def copy(ctx, n, x, y):
    ctx.check(lib.eig_copy(ctx.h, n, x.ptr, y.ptr))


def stream_copy_GBs(ctx, n=1 << 27, reps=20, mode=None):
    """Measured HBM copy rate (eig_stream_copy_timed over n doubles, default 1 GiB each way): 16 n B per
    launch / average launch time, in GB/s."""
    x, y = ctx.zeros(n), ctx.zeros(n)
    ms = _dbl(0)
    ctx.check(lib.eig_stream_copy_timed(ctx.h, n, x.ptr, y.ptr, reps, STREAM_COPY_MODE if mode is None else mode,
                                        ctypes.byref(ms)))
    x.free()
    y.free()
    return 16.0 * n / (ms.value * 1e-3) / 1e9


def spmm_mv8(A, m, Qin, Qout):
    A.ctx.check(lib.eig_spmm_mv8(A.h, m, Qin.ptr, Qout.ptr))


def dot_diag_mv8(ctx, n, m, Q1, Q2, dp):
    ctx.check(lib.eig_dot_diag_mv8(ctx.h, n, m, Q1.ptr, Q2.ptr, dp.ptr))


def gram_mv8(ctx, n, m1, m2, Q1, Q2, G):
    ctx.check(lib.eig_gram_mv8(ctx.h, n, m1, m2, Q1.ptr, Q2.ptr, G.ptr))


def orthonormalize_mv8(ctx, n, m, Q, variant=ORTHO_MGS):
    ctx.check(lib.eig_orthonormalize_mv8(ctx.h, n, m, Q.ptr, variant))


def spmm_dot_gram_mv8(A, m, Qin, Qout, dp, gram):
    """eig_spmm_dot_gram_mv8: Qout = A Qin, dp = diag(Qin^T Qout), gram = Qout's 8 x 8 window Gram (m = 8)."""
    A.ctx.check(lib.eig_spmm_dot_gram_mv8(A.h, m, Qin.ptr, Qout.ptr, dp.ptr, gram.ptr))


def orthonormalize_gram_mv8(ctx, n, m, Q, gram):
    """eig_orthonormalize_gram_mv8: MGS orthonormalize_blocked whose first block starts from `gram`."""
    ctx.check(lib.eig_orthonormalize_gram_mv8(ctx.h, n, m, Q.ptr, gram.ptr))


def orthonormalize_passes(ctx):
    """read passes the last look-ahead MGS on ctx took (its last diagonal block; -1: none)"""
    p = ctypes.c_int(0)
    ctx.check(lib.eig_orthonormalize_passes(ctx.h, ctypes.byref(p)))
    return p.value


def orthonormalize_naive(ctx, n, m, Q):
    ctx.check(lib.eig_orthonormalize_naive(ctx.h, n, m, Q.ptr))


def b_orthonormalize_mv8(B, m, Q, norm):
    B.ctx.check(lib.eig_b_orthonormalize_mv8(B.h, m, Q.ptr, norm.ptr))


def random_mv8(ctx, n, m, seed, Q):
    ctx.check(lib.eig_random_mv8(ctx.h, n, m, seed, Q.ptr))


def random_normal(count, seed=123):
    """The drivers' start-vector variates on the host (no device): bitwise
    std::normal_distribution<double>{0, 1} over std::mt19937{seed} (eigensolver.hh:50-55)."""
    out = np.zeros(count)
    rc = lib.eig_random_normal(count, seed, _np_ptr(out))
    if rc != 0:
        raise EigError(rc, "eig_random_normal failed")
    return out


def standard_largest(A, shift, tol, maxiter, nev, seed=123, want_evec=True, verbose=0):
    ev = np.zeros(nev)
    evec = np.zeros(nev * A.n) if want_evec else None
    it = _int(0)
    A.ctx.check(lib.eig_standard_largest(A.h, shift, tol, maxiter, nev, seed, _np_ptr(ev),
                                         _np_ptr(evec) if want_evec else None, ctypes.byref(it), verbose))
    return ev, (evec.reshape(nev, A.n) if want_evec else None), it.value


def _lflags(fused, pipelined):
    """fused: True / False / "auto" (EIG_LANCZOS_AUTO: fused on every 1x1 image)."""
    if pipelined:
        return LANCZOS_PIPELINED
    return LANCZOS_AUTO if fused == "auto" else LANCZOS_FUSED if fused else 0


def lanczos_run(A, steps, u0=None, seed=123, timed=False, fused=False, pipelined=False):
    """fused: the one-reduction single-kernel step (EIG_LANCZOS_FUSED) instead of K1 + K2;
    pipelined: the one-reduction step with the SpMV on t_{k-1} (EIG_LANCZOS_PIPELINED)."""
    alpha = np.zeros(max(steps, 1))
    beta = np.zeros(steps + 1)
    t = Timing()
    A.ctx.check(lib.eig_lanczos_run(A.h, steps, u0.ptr if u0 is not None else None, seed,
                                    _tflags(timed) | _lflags(fused, pipelined), _np_ptr(alpha), _np_ptr(beta),
                                    ctypes.byref(t)))
    return alpha[:steps], beta, t


class LanczosWorkspace:
    """eig_lanczos_t: the three-term recurrence as a persistent workspace (setup outside any
    timed region; step() advances and returns the eig_timing of that batch)."""

    def __init__(self, A, max_steps, u0=None, seed=123, fused=False, pipelined=False):
        self.A = A
        h = _vp()
        A.ctx.check(lib.eig_lanczos_create_ex(A.h, max_steps, u0.ptr if u0 is not None else None, seed,
                                              _lflags(fused, pipelined), ctypes.byref(h)))
        self.h = h
        _track(self)
        self.variant, self.kernel, self.kernel_bytes = self.ws_info()
        self.fused = self.variant in ("fused", "pipelined")
        self.pipelined = self.variant == "pipelined"

    def ws_info(self):
        """(variant: "classic" | "fused" | "pipelined", step kernel, its algorithmic bytes per launch)."""
        v, b = _int(0), _i64(0)
        name = ctypes.create_string_buffer(96)
        self.A.ctx.check(lib.eig_lanczos_ws_info(self.h, ctypes.byref(v), name, 96, ctypes.byref(b)))
        return ({0: "classic", LANCZOS_FUSED: "fused", LANCZOS_PIPELINED: "pipelined"}[v.value],
                name.value.decode(), b.value)

    def step(self, steps, timed=False):
        t = Timing()
        self.A.ctx.check(lib.eig_lanczos_step(self.h, steps, _tflags(timed), ctypes.byref(t)))
        return t

    def capture(self, steps, timed=False):
        """Record the next `steps` steps as one hipGraph (nothing runs); True when the runtime
        accepted the capture, False when replay() will take the steps eagerly."""
        c = _int(0)
        self.A.ctx.check(lib.eig_lanczos_capture(self.h, steps, _tflags(timed),
                                                 ctypes.byref(c)))
        return bool(c.value)

    def replay(self):
        t = Timing()
        self.A.ctx.check(lib.eig_lanczos_replay(self.h, ctypes.byref(t)))
        return t

    def info(self):
        """(logical steps taken, kernel launches issued); fused: launches - steps = repairs."""
        k, L = _int(0), _int(0)
        self.A.ctx.check(lib.eig_lanczos_info(self.h, ctypes.byref(k), ctypes.byref(L)))
        return k.value, L.value

    def tridiag(self):
        k = _int(0)
        self.A.ctx.check(lib.eig_lanczos_tridiag(self.h, ctypes.byref(k), None, None))
        alpha = np.zeros(max(k.value, 1))
        beta = np.zeros(k.value + 1)
        self.A.ctx.check(lib.eig_lanczos_tridiag(self.h, ctypes.byref(k), _np_ptr(alpha), _np_ptr(beta)))
        return alpha[:k.value], beta

    def close(self):
        if self.h and self.A.h and self.A.ctx.h:
            lib.eig_lanczos_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def lanczos_solve(A, nev, ncv, which=WHICH_LA, seed=123, want_evec=True):
    ev = np.zeros(nev)
    evec = np.zeros(nev * A.n) if want_evec else None
    res = np.zeros(nev)
    A.ctx.check(lib.eig_lanczos_solve(A.h, nev, ncv, which, seed, _np_ptr(ev), _np_ptr(evec) if want_evec else None,
                                      _np_ptr(res)))
    return ev, (evec.reshape(nev, A.n) if want_evec else None), res


def panel_update_mv8(ctx, n, m1, m2, Q, S, alpha, beta, Y):
    ctx.check(lib.eig_panel_update_mv8(ctx.h, n, m1, m2, Q.ptr, S.ptr, alpha, beta, Y.ptr))


def panel_gram_mv8(ctx, n, m1, m2, Q1, Q2, G):
    ctx.check(lib.eig_panel_gram_mv8(ctx.h, n, m1, m2, Q1.ptr, Q2.ptr, G.ptr))


def mass_solve_mv8(M, m, degree, B, X, lmin=0.5, lmax=2.5):
    M.ctx.check(lib.eig_mass_solve_mv8(M.h, m, degree, lmin, lmax, B.ptr, X.ptr))


class LU:
    """eig_lu_t: exported LU factors on the device (UMFPackFactorizedMatrix mirror)."""

    def __init__(self, ctx, handle):
        self.ctx, self.h = ctx, handle
        _track(self)

    @classmethod
    def from_factors(cls, ctx, Lp, Lj, Lx, Up, Ui, Ux, P, Q, Rs, do_recip=0):
        c = np.ascontiguousarray
        arrs = [c(Lp, np.int64), c(Lj, np.int64), c(Lx, np.float64), c(Up, np.int64), c(Ui, np.int64),
                c(Ux, np.float64), c(P, np.int64), c(Q, np.int64), c(Rs, np.float64)]
        h = _vp()
        ctx.check(lib.eig_lu_create(ctx.h, arrs[0].size - 1, *[_np_ptr(a) for a in arrs], int(do_recip),
                                    ctypes.byref(h)))
        lu = cls(ctx, h)
        lu._keep = arrs
        return lu

    @classmethod
    def from_bcsr(cls, ctx, rowptr, col, vals, br=1):
        """Host factorisation (eig_lu_create_bcsr); ctx=None gives host-only factors for export."""
        rowptr = np.ascontiguousarray(rowptr, np.int64)
        col = np.ascontiguousarray(col, np.int32)
        vals = np.ascontiguousarray(vals, np.float64)
        h = _vp()
        rc = lib.eig_lu_create_bcsr(ctx.h if ctx else None, rowptr.size - 1, br, _np_ptr(rowptr), _np_ptr(col),
                                    _np_ptr(vals), ctypes.byref(h))
        if rc != EIG_OK:
            raise EigError(rc, lib.eig_last_error(ctx.h if ctx else None).decode())
        return cls(ctx, h)

    def export(self):
        """-> dict of the factor arrays (Lp, Lj, Lx, Up, Ui, Ux, P, Q, Rs, do_recip)."""
        n, lnz, unz, rec = _i64(0), _i64(0), _i64(0), _int(0)
        self._check(lib.eig_lu_info(self.h, ctypes.byref(n), ctypes.byref(lnz), ctypes.byref(unz), ctypes.byref(rec)))
        n, lnz, unz = n.value, lnz.value, unz.value
        d = {"Lp": np.zeros(n + 1, np.int64), "Lj": np.zeros(lnz, np.int64), "Lx": np.zeros(lnz),
             "Up": np.zeros(n + 1, np.int64), "Ui": np.zeros(unz, np.int64), "Ux": np.zeros(unz),
             "P": np.zeros(n, np.int64), "Q": np.zeros(n, np.int64), "Rs": np.zeros(n)}
        self._check(lib.eig_lu_export(self.h, *[_np_ptr(d[k]) for k in ("Lp", "Lj", "Lx", "Up", "Ui", "Ux", "P",
                                                                        "Q", "Rs")]))
        d["do_recip"] = rec.value
        return d

    def _check(self, rc):
        if self.ctx:
            self.ctx.check(rc)
        elif rc != EIG_OK:
            raise EigError(rc, lib.eig_last_error(None).decode())

    def inverse_mv8(self, m, Qin, Qout):
        self.ctx.check(lib.eig_inverse_mv8(self.h, m, Qin.ptr, Qout.ptr))

    def solver_info(self):
        """-> (kernel in use: "blockinv" | "staged" | "csr", coupled blocks of L, of U)."""
        k, gl, gu = _int(0), _int(0), _int(0)
        self._check(lib.eig_lu_solver_info(self.h, ctypes.byref(k), ctypes.byref(gl), ctypes.byref(gu)))
        return {TRSV_BLOCKINV: "blockinv", TRSV_STAGED: "staged", TRSV_CSR: "csr"}[k.value], gl.value, gu.value

    def set_solver(self, kind):
        """kind: None / "auto", "blockinv", "staged" or "csr" (eig_lu_set_solver)."""
        self._check(lib.eig_lu_set_solver(self.h, TRSV_KINDS[kind]))

    def close(self):
        if self.h and (self.ctx is None or self.ctx.h):
            lib.eig_lu_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def standard_inverse(A, shift, tol, maxiter, nev, seed=123, lu=None, want_evec=True, verbose=0):
    ev = np.zeros(nev)
    evec = np.zeros(nev * A.n) if want_evec else None
    it = _int(0)
    A.ctx.check(lib.eig_standard_inverse(A.h, lu.h if lu else None, shift, tol, maxiter, nev, seed, _np_ptr(ev),
                                         _np_ptr(evec) if want_evec else None, ctypes.byref(it), verbose))
    return ev, (evec.reshape(nev, A.n) if want_evec else None), it.value


def generalized_inverse(A, B, shift, reg, tol, maxiter, nev, seed=123, lu=None, want_evec=True, verbose=0):
    ev = np.zeros(nev)
    evec = np.zeros(nev * A.n) if want_evec else None
    it = _int(0)
    A.ctx.check(lib.eig_generalized_inverse(A.h, B.h, lu.h if lu else None, shift, reg, tol, maxiter, nev, seed,
                                            _np_ptr(ev), _np_ptr(evec) if want_evec else None, ctypes.byref(it),
                                            verbose))
    return ev, (evec.reshape(nev, A.n) if want_evec else None), it.value


SI_AUTO, SI_SINGLE, SI_BLOCK = 0, 1, 2
_SI_METHODS = {"auto": SI_AUTO, "single": SI_SINGLE, "block": SI_BLOCK}


def shift_invert_solve(A, nev, sigma=0.0, B=None, ncv=0, tol=0.0, maxit=0, seed=123, lu=None, want_evec=True,
                       method="auto"):
    """computeGenSymShiftInvertMinMagnitude: (eigenvalues ascending, B-normalised vectors, restarts).
    method: "auto" | "single" (one-vector thick-restart Lanczos) | "block" (block Krylov-Schur)."""
    ev = np.zeros(nev)
    evec = np.zeros(nev * A.n) if want_evec else None
    r = _int(0)
    A.ctx.check(lib.eig_shift_invert_solve_ex(A.h, B.h if B is not None else None, lu.h if lu else None, sigma, nev,
                                              ncv, tol, maxit, seed, _np_ptr(ev), _np_ptr(evec) if want_evec else None,
                                              ctypes.byref(r), _SI_METHODS[method]))
    return ev, (evec.reshape(nev, A.n) if want_evec else None), r.value


def shift_invert_adaptive(A, threshold, initial_nev, max_nev, sigma=0.0, B=None, tol=0.0, maxit_per_nev=0, seed=123,
                          lu=None, want_evec=True):
    """computeGenSymShiftInvertMinMagnitudeAdaptive: every eigenvalue below `threshold` (nev grows x1.3
    from initial_nev up to max_nev) -> (eigenvalues ascending, B-normalised vectors, passes)."""
    ev = np.zeros(max_nev)
    evec = np.zeros(max_nev * A.n) if want_evec else None
    nv, ps = _int(0), _int(0)
    A.ctx.check(lib.eig_shift_invert_adaptive(A.h, B.h if B is not None else None, lu.h if lu else None, sigma,
                                              threshold, initial_nev, max_nev, tol, maxit_per_nev, seed, _np_ptr(ev),
                                              _np_ptr(evec) if want_evec else None, ctypes.byref(nv),
                                              ctypes.byref(ps)))
    k = nv.value
    return ev[:k], (evec[:k * A.n].reshape(k, A.n) if want_evec else None), ps.value


ARNOLDI_STD, ARNOLDI_GEN = 0, 1


def arnoldi_shift_invert(A, nev, sigma=0.0, B=None, mode="std", ncv=0, tol=0.0, maxit=0, seed=123, lu=None,
                         want_evec=True):
    """computeStdNonSymMinMagnitude (mode "std") / computeGenNonSymShiftInvertMinMagnitude (mode
    "gen"): (eigenvalues ascending by real part as a complex array, eigenvectors in ARPACK's raw
    storage or None, restarts)."""
    er, ei = np.zeros(nev), np.zeros(nev)
    evec = np.zeros(nev * A.n) if want_evec else None
    r = _int(0)
    A.ctx.check(lib.eig_arnoldi_shift_invert(A.h, B.h if B is not None else None, lu.h if lu else None, sigma, nev,
                                             ncv, tol, maxit, seed, ARNOLDI_GEN if mode == "gen" else ARNOLDI_STD,
                                             _np_ptr(er), _np_ptr(ei), _np_ptr(evec) if want_evec else None,
                                             ctypes.byref(r)))
    return er + 1j * ei, (evec.reshape(nev, A.n) if want_evec else None), r.value


class Multigrid:
    """eig_mg_t: geometric multigrid on a box-grid matrix (include/eigmi.h eig_mg_create)."""

    def __init__(self, A, dims, max_cols=32, smooth_degree=2, smooth_ratio=10.0):
        self.A = A
        h = _vp()
        A.ctx.check(lib.eig_mg_create(A.h, dims[0], dims[1], dims[2], max_cols, smooth_degree, smooth_ratio,
                                      ctypes.byref(h)))
        self.h = h
        _track(self)

    def info(self):
        lv, cr, cd, lm = _int(0), _i64(0), _int(0), _dbl(0)
        self.A.ctx.check(lib.eig_mg_info(self.h, ctypes.byref(lv), ctypes.byref(cr), ctypes.byref(cd), ctypes.byref(lm)))
        return {"levels": lv.value, "coarse_rows": cr.value, "coarse_degree": cd.value, "lmax_fine": lm.value}

    def solve(self, m, B, X, cycles, resid=False):
        """X = S_cycles B (device MultiVector buffers); returns max_j ||B - A X|| / ||B|| when resid."""
        r = _dbl(0)
        self.A.ctx.check(lib.eig_mg_solve(self.h, m, B.ptr, X.ptr, cycles, ctypes.byref(r) if resid else None))
        return r.value if resid else None

    def close(self):
        if self.h and self.A.h and self.A.ctx.h:
            lib.eig_mg_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BlockLanczos:
    """eig_blanczos_t: block Lanczos for K x = lambda M x (config C5), see include/eigmi.h."""

    def __init__(self, K, M, block=32, max_steps=8, degree=36, lmin=0.5, lmax=2.5, seed=123, Ks=None, sigma=0.0,
                 mg=None, cycles=0):
        """Ks given: the spectral transformation (K - sigma M)^-1 M with Ks = K - sigma M and
        (degree, lmin, lmax) the Chebyshev-Jacobi solve of Ks (eig_blanczos_create_si), or with
        mg (a Multigrid on Ks) `cycles` multigrid iterations (eig_blanczos_create_si_mg); otherwise
        M^-1 K with (degree, lmin, lmax) the mass solve."""
        self.K, self.M, self.block = K, M, block
        self.mg = mg
        h = _vp()
        if mg is not None:
            K.ctx.check(lib.eig_blanczos_create_si_mg(K.h, M.h, Ks.h, sigma, mg.h, cycles, block, max_steps, seed,
                                                      ctypes.byref(h)))
        elif Ks is None:
            K.ctx.check(lib.eig_blanczos_create(K.h, M.h, block, max_steps, degree, lmin, lmax, seed, ctypes.byref(h)))
        else:
            K.ctx.check(lib.eig_blanczos_create_si(K.h, M.h, Ks.h, sigma, block, max_steps, degree, lmin, lmax, seed,
                                                   ctypes.byref(h)))
        self.h = h
        _track(self)

    def step(self, steps):
        t = BlockTiming()
        self.K.ctx.check(lib.eig_blanczos_step(self.h, steps, ctypes.byref(t)))
        return t

    def tmatrix(self):
        d = _int(0)
        self.K.ctx.check(lib.eig_blanczos_tmatrix(self.h, ctypes.byref(d), None))
        T = np.zeros((d.value, d.value))
        self.K.ctx.check(lib.eig_blanczos_tmatrix(self.h, ctypes.byref(d), _np_ptr(T)))
        return T

    def ritz(self, nev, which=WHICH_LA, want_evec=False, want_resid=True):
        ev = np.zeros(nev)
        n = self.K.info.n
        evec = np.zeros(nev * n) if want_evec else None
        res = np.zeros(nev) if want_resid else None
        self.K.ctx.check(lib.eig_blanczos_ritz(self.h, nev, which, _np_ptr(ev), _np_ptr(evec) if want_evec else None,
                                               _np_ptr(res) if want_resid else None))
        return ev, (evec.reshape(nev, n) if want_evec else None), res

    def close(self):
        if self.h and self.K.h and self.K.ctx.h:
            lib.eig_blanczos_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# --------------------------------------------------------------------------------------- loopback
def loopback_create(nranks):
    """eig_loopback_create: a hub for `nranks` virtual ranks on one device (one host thread and one
    Context per rank; ctypes releases the GIL, so the ranks' calls run concurrently)."""
    h = _vp()
    rc = lib.eig_loopback_create(int(nranks), ctypes.byref(h))
    if rc != EIG_OK:
        raise EigError(rc, lib.eig_last_error(None).decode())
    return h


def loopback_destroy(hub):
    lib.eig_loopback_destroy(hub)


# --------------------------------------------------------------------------------------- generators
def gen_matrix(kind, N, overlap=3):
    nnzb = lib.eig_gen_nnzb(kind, N)
    nrows = N * N if kind <= 3 else N ** 3
    bb = 9 if kind == GEN_Q1ELAST3D else 1
    rp = np.zeros(nrows + 1, np.int64)
    c = np.zeros(nnzb, np.int32)
    v = np.zeros(nnzb * bb, np.float64)
    rc = lib.eig_gen_matrix(kind, N, overlap, _np_ptr(rp), _np_ptr(c), _np_ptr(v))
    if rc != EIG_OK:
        raise EigError(rc, "eig_gen_matrix failed")
    return rp, c, v


def gen_rows(kind, N, row_begin, nrows):
    nnzb = lib.eig_gen_nnzb_rows(kind, N, row_begin, nrows)
    bb = 9 if kind == GEN_Q1ELAST3D else 1
    rp = np.zeros(nrows + 1, np.int64)
    c = np.zeros(max(nnzb, 1), np.int32)
    v = np.zeros(max(nnzb, 1) * bb, np.float64)
    rc = lib.eig_gen_matrix_rows(kind, N, row_begin, nrows, _np_ptr(rp), _np_ptr(c), _np_ptr(v))
    if rc != EIG_OK:
        raise EigError(rc, "eig_gen_matrix_rows failed")
    return rp, c, v


def mm_read(path, br=1):
    """Matrix Market file -> (rowptr, col, vals, nb_cols) for Matrix.from_bcsr (eig_mm_read)."""
    nr, nc, nz = _i64(0), _i64(0), _i64(0)
    p = os.fsencode(path)
    rc = lib.eig_mm_read_info(p, br, ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(nz))
    if rc != EIG_OK:
        raise EigError(rc, f"eig_mm_read_info({path})")
    rp = np.zeros(nr.value + 1, np.int64)
    c = np.zeros(max(nz.value, 1), np.int32)
    v = np.zeros(max(nz.value, 1) * br * br)
    rc = lib.eig_mm_read(p, br, _np_ptr(rp), _np_ptr(c), _np_ptr(v))
    if rc != EIG_OK:
        raise EigError(rc, f"eig_mm_read({path})")
    return rp, c[:nz.value], v[:nz.value * br * br], nc.value


def mm_write(path, rowptr, col, vals, ncols_blocks=None, br=1, bc=1, symmetric=False):
    rowptr = np.ascontiguousarray(rowptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    vals = np.ascontiguousarray(vals, np.float64)
    nb = rowptr.size - 1
    rc = lib.eig_mm_write(os.fsencode(path), nb, nb if ncols_blocks is None else ncols_blocks, br, bc, _np_ptr(rowptr),
                          _np_ptr(col), _np_ptr(vals), int(symmetric))
    if rc != EIG_OK:
        raise EigError(rc, f"eig_mm_write({path})")


def reorder_rcm(rowptr, col):
    """Reverse Cuthill-McKee permutation of the symmetrised pattern (eig_reorder_rcm):
    perm[k] = old row of new row k."""
    rowptr = np.ascontiguousarray(rowptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    perm = np.zeros(rowptr.size - 1, np.int64)
    rc = lib.eig_reorder_rcm(rowptr.size - 1, _np_ptr(rowptr), _np_ptr(col), _np_ptr(perm))
    if rc != EIG_OK:
        raise EigError(rc, lib.eig_last_error(None).decode())
    return perm


def permute_symmetric(rowptr, col, vals, perm):
    """B = P A P^T, B[k][l] = A[perm[k]][perm[l]], columns ascending (eig_permute_symmetric)."""
    rowptr = np.ascontiguousarray(rowptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    vals = np.ascontiguousarray(vals, np.float64)
    perm = np.ascontiguousarray(perm, np.int64)
    rp, c, v = np.zeros_like(rowptr), np.zeros_like(col), np.zeros_like(vals)
    rc = lib.eig_permute_symmetric(rowptr.size - 1, _np_ptr(rowptr), _np_ptr(col), _np_ptr(vals), _np_ptr(perm),
                                   _np_ptr(rp), _np_ptr(c), _np_ptr(v))
    if rc != EIG_OK:
        raise EigError(rc, lib.eig_last_error(None).decode())
    return rp, c, v


def scrambled_rcm(rowptr, col, vals, seed=123):
    """The general-CSR bench / test matrix: a seeded random symmetric permutation
    of A followed by reverse Cuthill-McKee -- nnz and symmetry kept, the constant-offset band and
    the per-slice stencil structure gone, so the explicit-column SELL kernels run."""
    p0 = np.random.default_rng(seed).permutation(rowptr.size - 1).astype(np.int64)
    rp, c, v = permute_symmetric(rowptr, col, vals, p0)
    p1 = reorder_rcm(rp, c)
    return permute_symmetric(rp, c, v, p1)


def row_partition(n, nranks, rank, align=1):
    """Contiguous row block of `rank` (z-slabs for the 3-D stencil when align = N*N)."""
    units = n // align
    b = (units * rank) // nranks
    e = (units * (rank + 1)) // nranks
    if rank == nranks - 1:
        return b * align, n - b * align
    return b * align, (e - b) * align


# Algorithmic byte models (DESIGN.md "Roofline accounting")
def bytes_spmv(n, nnz):
    return 12 * nnz + 4 * (n + 1) + 16 * n


def image_bytes(M, op, m=8):
    """Algorithmic HBM bytes of one launch sequence on M's device image:
    op "spmv" (y = A x) or "spmm" (m columns).  The symmetric band image streams 8 B per band slot
    and the row mask once per 8-column block (the plane march; a uniform band only the mask in the
    scalar march); the row-class image (3-D box
    stencils with class-constant rows) no matrix data at all; other images the SURVEY 8(d) CSR
    count (12 B per nonzero + row pointers), which the SELL/stencil kernels stream at most."""
    info = M.info
    n, nnz = info.n, info.nnzb
    band = info.sym_offsets > 0
    mat = (8 * info.sym_arrays + info.sym_mask_bytes) * n if band else 12 * nnz + 4 * (n + 1)
    if op == "spmv":
        if band and M.kernel("spmv") == "k_spmv_march":
            v = info.march_variant_mv
            if v >= 10:  # the value marches: band values streamed, geometric masks (no mask stream)
                return 8 * (4 if v in (15, 18) else info.sym_arrays) * n + 16 * n
            if v >= 1:
                # uniform band: the values ride in the arguments (2..9: the row masks are geometric too)
                return (0 if v >= 2 else info.sym_mask_bytes * n) + 16 * n
        return mat + 16 * n
    if op == "spmm":
        if M.kernel("spmm8") == "k_boxc_mv8":  # row-class image: the class table lives in LDS
            return 16 * m * n
        return (m // 8 if band else 1) * mat + 16 * m * n
    raise ValueError(op)


def bytes_lanczos_step(n, nnz):
    return bytes_spmv(n, nnz) + 32 * n


def bytes_lanczos_k1(n, nnz):
    """Fused SpMV kernel of a Lanczos step: CSR stream + x + y write + u_{j-1} read."""
    return bytes_spmv(n, nnz) + 8 * n


def bytes_lanczos_fused(n, nnz):
    """Fused one-reduction step kernel: CSR stream + gathers of t_{k-1} and u_{k-1} + writes of
    t_k and u_k (the whole step; 16n fewer than bytes_lanczos_step)."""
    return 12 * nnz + 4 * (n + 1) + 32 * n


# --------------------------------------------------------------------------------------- planning
def plan_window(row_begin, nb_local, rowptr, col, bc=1):
    """-> (win_begin_blk, window, own_offset, cmin, cmax) -- eig_plan_window."""
    out = np.zeros(5, np.int64)
    rowptr = np.ascontiguousarray(rowptr, np.int64)
    col = np.ascontiguousarray(col, np.int32)
    rc = lib.eig_plan_window(row_begin, nb_local, bc, _np_ptr(rowptr), _np_ptr(col), _np_ptr(out))
    if rc != EIG_OK:
        raise EigError(rc, "eig_plan_window failed")
    return tuple(int(v) for v in out)


def plan_halo(nranks, me, ranks, win_begin_blk, bc=1):
    """ranks: (nranks, 4) int64 [row_begin, nb_local, cmin, cmax] -> (recvs, sends), lists of
    (peer, window offset, count) -- eig_plan_halo."""
    ranks = np.ascontiguousarray(ranks, np.int64).reshape(-1)
    rv = np.zeros(3 * nranks, np.int64)
    sd = np.zeros(3 * nranks, np.int64)
    nr, ns = _int(0), _int(0)
    rc = lib.eig_plan_halo(nranks, me, _np_ptr(ranks), bc, win_begin_blk, _np_ptr(rv), ctypes.byref(nr),
                           _np_ptr(sd), ctypes.byref(ns))
    if rc != EIG_OK:
        raise EigError(rc, "eig_plan_halo failed")
    recvs = [tuple(int(x) for x in rv[3 * k:3 * k + 3]) for k in range(nr.value)]
    sends = [tuple(int(x) for x in sd[3 * k:3 * k + 3]) for k in range(ns.value)]
    return recvs, sends
