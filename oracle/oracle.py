"""ctypes wrapper of oracle/liboracle.so -- the CPU restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.  See oracle/oracle.cc for the per-function
reference citations and DESIGN.md "Oracle" for how the restatement is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")

_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i64 = ctypes.c_int64
_int = ctypes.c_int


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load(path=_LIB):
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(os.path.join(_HERE, "oracle.cc")):
        build()
    lib = ctypes.CDLL(path)
    sig = {
        "orc_laplace2d_nnz": (_i64, [_int]),
        "orc_laplace2d": (None, [_int, _i64p, _i32p, _f64p]),
        "orc_laplace2d_neumann": (None, [_int, _i64p, _i32p, _f64p]),
        "orc_laplace2d_pu": (None, [_int, _int, _i64p, _i32p, _f64p]),
        "orc_identity2d": (None, [_int, _i64p, _i32p, _f64p]),
        "orc_poisson3d_nnz": (_i64, [_int]),
        "orc_poisson3d": (None, [_int, _i64p, _i32p, _f64p]),
        "orc_q1elast_nnzb": (_i64, [_int]),
        "orc_q1elast": (None, [_int, _i64p, _i32p, _f64p]),
        "orc_eig_laplace2d": (None, [_int, _f64p]),
        "orc_csr_mv": (None, [_i64, _i64p, _i32p, _f64p, _f64p, _f64p]),
        "orc_bcsr_mv": (None, [_i64, _int, _int, _i64p, _i32p, _f64p, _f64p, _f64p]),
        "orc_spmm_mv8": (None, [_i64, _i64, _i64p, _i32p, _f64p, _f64p, _f64p]),
        "orc_dot_diag_mv8": (None, [_i64, _i64, _f64p, _f64p, _f64p]),
        "orc_gram_mv8": (None, [_i64, _i64, _f64p, _f64p, _f64p]),
        "orc_orthonormalize_naive": (None, [_i64, _i64, _f64p]),
        "orc_orthonormalize_mv8": (None, [_i64, _i64, _f64p]),
        "orc_orthonormalize_cholqr_mv8": (None, [_i64, _i64, _f64p]),
        "orc_orthonormalize_cholqr_split_mv8": (None, [_i64, _i64, _f64p]),
        "orc_b_orthonormalize_mv8": (ctypes.c_double, [_i64, _i64, _i64p, _i32p, _f64p, _f64p]),
        "orc_flops_orthonormalize": (ctypes.c_double, [_int, _int]),
        "orc_bytes_orthonormalize_naive": (ctypes.c_double, [_int, _int]),
        "orc_bytes_orthonormalize_blocked": (ctypes.c_double, [_int, _int, _int]),
        "orc_random_mv8": (None, [_i64, _i64, ctypes.c_uint, _f64p]),
        "orc_random_vec": (None, [_i64, ctypes.c_uint, _f64p]),
        "orc_shift_diag": (None, [_i64, _i64p, _i32p, _f64p, ctypes.c_double]),
        "orc_standard_largest": (_int, [_i64, _i64p, _i32p, _f64p, ctypes.c_double, ctypes.c_double,
                                        _int, _int, ctypes.c_uint, _f64p, _f64p]),
        "orc_lanczos": (None, [_i64, _i64p, _i32p, _f64p, _int, _f64p, _f64p, _f64p]),
        "orc_inverse_mv8": (None, [_i64, _i64, _i64p, _i64p, _f64p, _i64p, _i64p, _f64p, _i64p, _i64p, _f64p, _int,
                                   _f64p, _f64p]),
        "orc_standard_inverse": (_int, [_i64, _i64p, _i32p, _f64p] + [_i64p, _i64p, _f64p, _i64p, _i64p, _f64p, _i64p,
                                                                      _i64p, _f64p, _int] +
                                 [ctypes.c_double, ctypes.c_double, _int, _int, ctypes.c_uint, _f64p, _f64p]),
        "orc_generalized_inverse": (_int, [_i64, _i64p, _i32p, _f64p, _i64p, _i32p, _f64p] +
                                    [_i64p, _i64p, _f64p, _i64p, _i64p, _f64p, _i64p, _i64p, _f64p, _int] +
                                    [ctypes.c_double, ctypes.c_double, ctypes.c_double, _int, _int, ctypes.c_uint,
                                     _f64p, _f64p]),
        "orc_lanczos_rotating": (None, [_i64, _i64p, _i32p, _f64p, _int, _f64p, _f64p, _f64p, _f64p, _f64p]),
        "orc_lanczos_fused": (None, [_i64, _i64p, _i32p, _f64p, _int, _f64p, _f64p, _f64p, ctypes.c_void_p]),
        "orc_lanczos_pipelined": (None, [_i64, _i64p, _i32p, _f64p, _int, _f64p, _f64p, _f64p, ctypes.c_void_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()
_fast = None


def fast_lib():
    """liboracle_fast.so: the same restatement built -O3 -march=x86-64-v3 (FMA contraction on) -- the
    CPU baseline bench.py times; never used as a parity checker."""
    global _fast
    if _fast is None:
        _fast = _load(os.path.join(_HERE, "liboracle_fast.so"))
    return _fast


class CSR:
    """Host CSR (or BCSR when br/bc > 1): int64 rowptr, int32 col, float64 val (row-major blocks)."""

    def __init__(self, nrows, rowptr, col, val, br=1, bc=1):
        self.nrows, self.rowptr, self.col, self.val, self.br, self.bc = nrows, rowptr, col, val, br, bc

    @property
    def n(self):
        return self.nrows * self.br

    @property
    def nnz(self):
        return int(self.rowptr[-1])

    def to_scipy(self):
        import scipy.sparse as sp
        if self.br == 1 and self.bc == 1:
            return sp.csr_matrix((self.val, self.col, self.rowptr), shape=(self.nrows, self.nrows))
        data = self.val.reshape(-1, self.br, self.bc)
        return sp.bsr_matrix((data, self.col, self.rowptr), shape=(self.nrows * self.br, self.nrows * self.bc))


def _alloc(nrows, nnz, blk=1):
    return np.zeros(nrows + 1, np.int64), np.zeros(nnz, np.int32), np.zeros(nnz * blk, np.float64)


def laplace2d(N, kind="dirichlet", overlap=3):
    nnz = lib.orc_laplace2d_nnz(N)
    rp, c, v = _alloc(N * N, nnz)
    if kind == "dirichlet":
        lib.orc_laplace2d(N, rp, c, v)
    elif kind == "neumann":
        lib.orc_laplace2d_neumann(N, rp, c, v)
    elif kind == "pu":
        lib.orc_laplace2d_pu(N, overlap, rp, c, v)
    elif kind == "identity":
        lib.orc_identity2d(N, rp, c, v)
    else:
        raise ValueError(kind)
    return CSR(N * N, rp, c, v)


def poisson3d(N):
    nnz = lib.orc_poisson3d_nnz(N)
    rp, c, v = _alloc(N ** 3, nnz)
    lib.orc_poisson3d(N, rp, c, v)
    return CSR(N ** 3, rp, c, v)


def q1elast(N):
    nnzb = lib.orc_q1elast_nnzb(N)
    rp, c, v = _alloc(N ** 3, nnzb, 9)
    lib.orc_q1elast(N, rp, c, v)
    return CSR(N ** 3, rp, c, v, 3, 3)


def eig_laplace2d(N):
    ev = np.zeros(N * N)
    lib.orc_eig_laplace2d(N, ev)
    return ev


def csr_mv(A, x):
    y = np.zeros(A.nrows * A.br)
    if A.br == 1 and A.bc == 1:
        lib.orc_csr_mv(A.nrows, A.rowptr, A.col, A.val, np.ascontiguousarray(x, np.float64), y)
    else:
        lib.orc_bcsr_mv(A.nrows, A.br, A.bc, A.rowptr, A.col, A.val, np.ascontiguousarray(x, np.float64), y)
    return y


def spmm_mv8(A, Q, m):
    out = np.zeros_like(Q)
    lib.orc_spmm_mv8(A.nrows, m, A.rowptr, A.col, A.val, Q, out)
    return out


def dot_diag_mv8(Q1, Q2, n, m):
    dp = np.zeros(m)
    lib.orc_dot_diag_mv8(n, m, Q1, Q2, dp)
    return dp


def gram_mv8(Q1, Q2, n, m):
    G = np.zeros((m, m))
    lib.orc_gram_mv8(n, m, Q1, Q2, G.reshape(-1))
    return G


def orthonormalize_mv8(Q, n, m, variant="mgs"):
    Q = Q.copy()
    if variant == "mgs":
        lib.orc_orthonormalize_mv8(n, m, Q)
    elif variant == "cholqr":
        lib.orc_orthonormalize_cholqr_mv8(n, m, Q)
    elif variant == "cholqr_split":
        lib.orc_orthonormalize_cholqr_split_mv8(n, m, Q)
    else:
        raise ValueError(variant)
    return Q


def orthonormalize_naive(Q, n, m):
    Q = Q.copy()
    lib.orc_orthonormalize_naive(n, m, Q)
    return Q


def b_orthonormalize_mv8(B, Q, n, m):
    Q = Q.copy()
    norm = lib.orc_b_orthonormalize_mv8(n, m, B.rowptr, B.col, B.val, Q)
    return Q, norm


def random_mv8(n, m, seed=123):
    Q = np.zeros(n * m)
    lib.orc_random_mv8(n, m, seed, Q)
    return Q


def random_vec(n, seed=123):
    x = np.zeros(n)
    lib.orc_random_vec(n, seed, x)
    return x


def standard_largest(A, shift, tol, maxiter, nev, seed=123):
    val = A.val.copy()
    ev = np.zeros(nev)
    evec = np.zeros(nev * A.n)
    it = lib.orc_standard_largest(A.n, A.rowptr, A.col, val, shift, tol, maxiter, nev, seed, ev, evec)
    return ev, evec.reshape(nev, A.n), it


class LU:
    """Exported LU factors (UMFPackFactorizedMatrix's public arrays, umfpacktools.hh:20-39)."""

    def __init__(self, Lp, Lj, Lx, Up, Ui, Ux, P, Q, Rs, do_recip):
        c = np.ascontiguousarray
        self.Lp, self.Lj, self.Lx = c(Lp, np.int64), c(Lj, np.int64), c(Lx, np.float64)
        self.Up, self.Ui, self.Ux = c(Up, np.int64), c(Ui, np.int64), c(Ux, np.float64)
        self.P, self.Q, self.Rs, self.do_recip = c(P, np.int64), c(Q, np.int64), c(Rs, np.float64), int(do_recip)
        self.n = self.Lp.size - 1

    def args(self):
        return (self.Lp, self.Lj, self.Lx, self.Up, self.Ui, self.Ux, self.P, self.Q, self.Rs, self.do_recip)


def inverse_mv8(lu, Qin, m):
    """matmul_inverse_tallskinny_blocked: returns (Qout, Qin after the call)."""
    pin = np.ascontiguousarray(Qin, np.float64).copy()
    out = np.zeros_like(pin)
    lib.orc_inverse_mv8(lu.n, m, *lu.args(), pin, out)
    return out, pin


def standard_inverse(A, lu, shift, tol, maxiter, nev, seed=123):
    val = A.val.copy()
    ev = np.zeros(nev)
    evec = np.zeros(nev * A.n)
    it = lib.orc_standard_inverse(A.n, A.rowptr, A.col, val, *lu.args(), shift, tol, maxiter, nev, seed, ev, evec)
    return ev, evec.reshape(nev, A.n), it


def generalized_inverse(A, B, lu, shift, reg, tol, maxiter, nev, seed=123):
    ev = np.zeros(nev)
    evec = np.zeros(nev * A.n)
    it = lib.orc_generalized_inverse(A.n, A.rowptr, A.col, A.val, B.rowptr, B.col, B.val, *lu.args(), shift, reg, tol,
                                     maxiter, nev, seed, ev, evec)
    return ev, evec.reshape(nev, A.n), it


def lanczos(A, u0, k):
    U = np.zeros((k + 1) * A.n)
    U[: A.n] = u0
    alpha = np.zeros(k)
    beta = np.zeros(k + 1)
    lib.orc_lanczos(A.n, A.rowptr, A.col, A.val, k, U, alpha, beta)
    return U.reshape(k + 1, A.n), alpha, beta


def lanczos_fused(A, u0, k, with_launches=False, pipelined=False):
    """The guarded fused one-reduction recurrence (orc_lanczos_fused): alpha[k], beta[k+1]
    (beta[k] exact, as eig_lanczos_tridiag returns it); with_launches: also the launch count
    (steps + repairs + the forced final repair).  pipelined: orc_lanczos_pipelined (the SpMV of
    a launch multiplies t_{k-1}; A u_k by the z recurrence)."""
    alpha = np.zeros(max(k, 1))
    beta = np.zeros(k + 1)
    L = ctypes.c_int(0)
    f = lib.orc_lanczos_pipelined if pipelined else lib.orc_lanczos_fused
    f(A.n, A.rowptr, A.col, A.val, k, np.ascontiguousarray(u0, dtype=np.float64), alpha, beta,
                          ctypes.byref(L))
    if with_launches:
        return alpha[:k], beta, L.value
    return alpha[:k], beta


def mv_index(n, i, j):
    """MultiVector<double,8> flat index (multivector.hh:130-139)."""
    return ((j // 8) * n + i) * 8 + (j % 8)


def mv_to_cols(Q, n, m):
    """Block-column-major MultiVector<double,8> -> (n, m) dense array."""
    return Q.reshape(m // 8, n, 8).transpose(1, 0, 2).reshape(n, m)


def cols_to_mv(X):
    n, m = X.shape
    return np.ascontiguousarray(X.reshape(n, m // 8, 8).transpose(1, 0, 2).reshape(-1))


# ------------------------------------------------------------------------------- config C5 (numpy)
# Independent restatements for the generalised block Lanczos: the P1 matrices by GLOBAL element
# assembly (the product generator, dune-eigensolver_amd/csrc/gen.cpp kinds 6/7, assembles row by
# row), and the block Lanczos recurrence in dense numpy.  There is no reference block Lanczos; the
# reference's generalised path is GeneralizedInverse (eigensolver.hh:204-351) / ARPACK shift-invert
# (arpack_geneo_wrapper.hh:581-658), whose answer -- the eigenpairs of (K, M) -- scipy.linalg.eigh
# gives exactly at these sizes; that is the parity anchor of the tests.

_KUHN_PERMS = ((0, 1, 2), (0, 2, 1), (1, 0, 2), (1, 2, 0), (2, 0, 1), (2, 1, 0))
_PATH = np.array([[1, -1, 0, 0], [-1, 2, -1, 0], [0, -1, 2, -1], [0, 0, -1, 1]], np.float64)


def p1_kuhn(N):
    """(K, M) scipy CSR for P1 on the Kuhn 6-tetrahedra split of the unit cube, N^3 interior nodes
    (lexicographic, x fastest), Dirichlet nodes eliminated; K and M share the 15-point edge
    pattern (K's entries on the face / body diagonals are exact zeros)."""
    import scipy.sparse as sp
    h = 1.0 / (N + 1)
    c = np.arange(N + 1)
    cz, cy, cx = np.meshgrid(c, c, c, indexing="ij")
    corners = np.stack([cx.ravel(), cy.ravel(), cz.ravel()], axis=1)  # cube lower corners (x, y, z)
    rows, cols, kv, mv = [], [], [], []
    Ke = (h / 6.0) * _PATH
    Me = (h ** 3 / 120.0) * (np.ones((4, 4)) + np.eye(4))
    for p in _KUHN_PERMS:
        v = [corners.copy()]
        v1 = corners.copy()
        v1[:, p[0]] += 1
        v2 = v1.copy()
        v2[:, p[1]] += 1
        v.extend([v1, v2, corners + 1])
        ids = []
        for vert in v:
            inside = np.all((vert >= 1) & (vert <= N), axis=1)
            g = ((vert[:, 2] - 1) * N + (vert[:, 1] - 1)) * N + (vert[:, 0] - 1)
            ids.append(np.where(inside, g, -1))
        for a in range(4):
            for b in range(4):
                ok = (ids[a] >= 0) & (ids[b] >= 0)
                rows.append(ids[a][ok])
                cols.append(ids[b][ok])
                kv.append(np.full(ok.sum(), Ke[a, b]))
                mv.append(np.full(ok.sum(), Me[a, b]))
    r, cc = np.concatenate(rows), np.concatenate(cols)
    n = N ** 3
    K = sp.coo_matrix((np.concatenate(kv), (r, cc)), shape=(n, n)).tocsr()
    M = sp.coo_matrix((np.concatenate(mv), (r, cc)), shape=(n, n)).tocsr()
    K.sort_indices()
    M.sort_indices()
    return K, M


def cheb_solve(M, B, degree, lmin=0.5, lmax=2.5):
    """x_degree of the Golub-Varga Chebyshev semi-iteration for M X = B with the Jacobi splitting
    (the same recurrence as k_sell_mv8<kCheb>, dune-eigensolver_amd/csrc/k_block.hip)."""
    dinv = 1.0 / M.diagonal()
    gamma, mu = 2.0 / (lmin + lmax), (lmax - lmin) / (lmax + lmin)
    x_prev = np.zeros_like(B)
    x = gamma * dinv[:, None] * B
    omega = 1.0
    for k in range(1, degree):
        omega = 1.0 / (1.0 - 0.5 * mu * mu) if k == 1 else 1.0 / (1.0 - 0.25 * mu * mu * omega)
        x_new = omega * (x + gamma * dinv[:, None] * (B - M @ x) - x_prev) + x_prev
        x_prev, x = x, x_new
    return x


def block_lanczos_gen(K, M, V0, steps, degree=36, lmin=0.5, lmax=2.5):
    """Block Lanczos in the M-inner product on M^-1 K (include/eigmi.h, eig_blanczos_*): returns
    the block tridiagonal T (steps*b square) and the basis [V_0 .. V_steps]."""
    def mcholqr2(Z):
        Rt = np.eye(Z.shape[1])
        for _ in range(2):
            G = Z.T @ (M @ Z)
            G = 0.5 * (G + G.T)
            R = np.linalg.cholesky(G).T
            Z = np.linalg.solve(R.T, Z.T).T
            Rt = R @ Rt
        return Z, Rt
    b = V0.shape[1]
    V, _ = mcholqr2(V0)
    basis = [V]
    A, Bs = [], []
    for j in range(steps):
        W = K @ basis[j]
        Aj = basis[j].T @ W
        A.append(0.5 * (Aj + Aj.T))
        Z = cheb_solve(M, W, degree, lmin, lmax)
        Vall = np.hstack(basis)
        for _ in range(2):
            Z = Z - Vall @ (Vall.T @ (M @ Z))
        Z, R = mcholqr2(Z)
        basis.append(Z)
        Bs.append(R)
    T = np.zeros((steps * b, steps * b))
    for j in range(steps):
        T[j * b:(j + 1) * b, j * b:(j + 1) * b] = A[j]
        if j + 1 < steps:
            T[(j + 1) * b:(j + 2) * b, j * b:(j + 1) * b] = Bs[j]
            T[j * b:(j + 1) * b, (j + 1) * b:(j + 2) * b] = Bs[j].T
    return T, basis
