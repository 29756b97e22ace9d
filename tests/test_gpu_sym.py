"""GPU parity of the symmetric band image (internal.h eig_mat_s::sym_*, api.cpp build_sym).

A square 1x1 matrix whose rows draw their columns from at most 32 offsets and whose stored mirror
pairs are bitwise equal keeps its values once, in upper-triangle band arrays; the scalar SpMV and
the Lanczos kernels read the lower entries through the mirrored upper slot.  Every row still sums
its own stored entries in ascending-column order, so the bar stays BITWISE equality with the
reference row loop (oracle.csr_mv = matmul_sparse_tallskinny_naive, kernels_cpp.hh:596-621)."""

import numpy as np
import pytest

import eigmi
import oracle

pytestmark = pytest.mark.gpu


def upload(ctx, A, sym=True, flags=0):
    """sym=False: no band image (eig_mat_create_bcsr_ex EIG_MAT_NO_BAND; the SELL kernels)."""
    return eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, A.br, A.bc,
                                  flags=flags | (0 if sym else eigmi.MAT_NO_BAND))


def band_matrix(n, offsets, seed, drop=0.0, symmetric=True):
    """Random-valued band matrix on the given non-negative offsets (mirrored to negative ones).
    `drop`: probability that an upper entry is stored without its mirror (a structurally
    unsymmetric pattern whose stored pairs are still equal)."""
    rng = np.random.default_rng(seed)
    ups = {}
    for p in offsets:
        m = n - p
        v = rng.standard_normal(m)
        keep_lo = rng.random(m) >= drop
        keep_up = rng.random(m) >= drop if p else np.ones(m, bool)
        ups[p] = (v, keep_up, keep_lo)
    rows = [[] for _ in range(n)]
    for p, (v, ku, kl) in ups.items():
        for i in range(n - p):
            if ku[i]:
                rows[i].append((i + p, v[i]))
            if p and kl[i]:
                rows[i + p].append((i, v[i] if symmetric else v[i] * (1 + 1e-15 * (i % 3 == 1))))
    rowptr, col, val = [0], [], []
    for r in rows:
        r.sort()
        col.extend(c for c, _ in r)
        val.extend(x for _, x in r)
        rowptr.append(len(col))
    return oracle.CSR(n, np.array(rowptr, np.int64), np.array(col, np.int32), np.array(val, np.float64))


def check_mv(ctx, A, expect_sym):
    M = upload(ctx, A)
    assert (M.info.sym_offsets > 0) == expect_sym
    rng = np.random.default_rng(7)
    for x in (rng.standard_normal(A.n), np.ones(A.n)):
        y = M.mv_host(x)
        ref = oracle.csr_mv(A, x)
        assert np.array_equal(y, ref), f"max diff {np.abs(y - ref).max()}"
    return M


@pytest.mark.parametrize("N", [16, 33])
def test_poisson_uses_sym_image_bitwise(ctx, N):
    A = oracle.poisson3d(N)
    M = check_mv(ctx, A, True)
    assert M.info.sym_offsets == 7


def test_2d_laplacians_bitwise(ctx):
    check_mv(ctx, oracle.laplace2d(64), True)
    check_mv(ctx, oracle.laplace2d(64, "neumann"), True)


def test_random_symmetric_band_u8_mask(ctx):
    check_mv(ctx, band_matrix(5000, [0, 1, 7, 130], 1), True)


def test_structurally_unsymmetric_pattern(ctx):
    """Pairs with one side missing: the slot carries the stored side, the mask hides the other."""
    A = band_matrix(3001, [0, 1, 64, 200], 2, drop=0.3)
    check_mv(ctx, A, True)


def test_many_offsets_u32_mask(ctx):
    """More than 8 offsets (here 2*12-1 = 23): 32-bit row masks."""
    A = band_matrix(4100, [0, 1, 2, 3, 5, 8, 13, 21, 34, 55, 89, 144], 3, drop=0.1)
    M = check_mv(ctx, A, True)
    assert M.info.sym_offsets == 23


def test_not_bitwise_symmetric_keeps_sell(ctx):
    A = band_matrix(2000, [0, 1, 9], 4, symmetric=False)
    check_mv(ctx, A, False)


def test_wide_offsets_keep_sell(ctx):
    A = band_matrix(600, list(range(0, 40)), 5)  # 79 offsets > 32
    check_mv(ctx, A, False)


def test_shift_diag_updates_band(ctx):
    A = band_matrix(3000, [0, 1, 50], 6)
    M = upload(ctx, A)
    assert M.info.sym_offsets > 0
    M.shift_diag(-0.625)
    val = A.val.copy()
    oracle.lib.orc_shift_diag(A.n, A.rowptr, A.col, val, -0.625)
    B = oracle.CSR(A.nrows, A.rowptr, A.col, val)
    x = np.random.default_rng(0).standard_normal(A.n)
    assert np.array_equal(M.mv_host(x), oracle.csr_mv(B, x))


@pytest.mark.parametrize("fused", [False, True])
def test_lanczos_sym_equals_sell(ctx, fused):
    """Same Krylov process through the band image and through the SELL image: per-row sums are
    bitwise equal and both kernels run on the same grid, so alpha/beta agree to rounding of the
    reductions (bitwise when the grids coincide)."""
    A = oracle.poisson3d(24)
    Ms, Mp = upload(ctx, A, True), upload(ctx, A, False)
    assert Ms.info.sym_offsets == 7 and Mp.info.sym_offsets == 0
    a1, b1, _ = eigmi.lanczos_run(Ms, 40, seed=123, fused=fused)
    a2, b2, _ = eigmi.lanczos_run(Mp, 40, seed=123, fused=fused)
    assert np.allclose(a1, a2, rtol=1e-12, atol=0) and np.allclose(b1, b2, rtol=1e-12, atol=0)
    ra, rb = (oracle.lanczos_fused(A, oracle.random_vec(A.n, 123), 40) if fused
              else oracle.lanczos(A, oracle.random_vec(A.n, 123), 40)[1:])
    assert np.allclose(a1, ra, rtol=1e-11, atol=0) and np.allclose(b1, rb, rtol=1e-11, atol=0)


# ---- plane march (k_*_march): widest offset D a multiple of 64, rows marched plane by plane ----

@pytest.mark.parametrize("n,offs,drop", [
    (5000, [0, 1, 5, 128], 0.0),        # 39.06 planes: partial last plane
    (4096, [0, 1, 64], 0.2),            # 2-D-like, structurally unsymmetric
    (6000, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 192], 0.1),  # 23 offsets: u32 masks
    (3000, [0, 2, 64], 0.0),            # no +-1: band path without lane shifts, no march
])
def test_march_spmv_bitwise(ctx, n, offs, drop):
    A = band_matrix(n, offs, 11, drop=drop)
    M = check_mv(ctx, A, True)
    name, _ = M.lanczos_kernel_info(fused=False)
    assert name == ("k_lanczos_spmv_march" if 1 in offs else "k_lanczos_spmv_b1")


def test_march_kernel_names_and_bytes(ctx):
    A = oracle.poisson3d(16)
    n = A.n
    # constant coefficients on a grid: the uniform-band march streams the vectors only (values in
    # the arguments, row masks from the coordinates)
    M = upload(ctx, A)
    assert M.lanczos_kernel_info(True) == ("k_lanczos_fused_march", 32 * n)
    assert M.lanczos_kernel_info(False) == ("k_lanczos_spmv_march", 24 * n)
    M = upload(ctx, A, flags=eigmi.MAT_NO_UNIFORM)
    assert M.lanczos_kernel_info(True) == ("k_lanczos_fused_march", 8 * 4 * n + n + 32 * n)
    assert M.lanczos_kernel_info(False) == ("k_lanczos_spmv_march", 8 * 4 * n + n + 24 * n)
    B = upload(ctx, band_matrix(5000, [0, 1, 5, 128], 11))  # random values: not uniform
    assert B.lanczos_kernel_info(True) == ("k_lanczos_fused_march", 8 * 4 * 5000 + 5000 + 32 * 5000)
    P = upload(ctx, A, sym=False)
    assert P.lanczos_kernel_info(True)[0] == "k_lanczos_fused_b1"


def _box_poisson(nx, ny, nz):
    """7-point Poisson (6 on the diagonal, -1 to each in-grid neighbour) on an nx x ny x nz box."""
    import scipy.sparse as sp

    def lap(k):
        return sp.diags([-np.ones(k - 1), 2 * np.ones(k), -np.ones(k - 1)], [-1, 0, 1])
    I = [sp.identity(k) for k in (nx, ny, nz)]
    L = (sp.kron(sp.kron(I[2], I[1]), lap(nx)) + sp.kron(sp.kron(I[2], lap(ny)), I[0]) +
         sp.kron(sp.kron(lap(nz), I[1]), I[0])).tocsr()
    L.sort_indices()
    return oracle.CSR(L.shape[0], L.indptr.astype(np.int64), L.indices.astype(np.int32), L.data.astype(np.float64))


def _drop_pair(A, i, d=1):
    """A without the symmetric pair (i, i + d) / (i + d, i): still a uniform band, but row masks that
    are no longer those of the grid."""
    keep = np.ones(A.val.size, bool)
    for r, c in ((i, i + d), (i + d, i)):
        keep[A.rowptr[r] + int(np.nonzero(A.col[A.rowptr[r]:A.rowptr[r + 1]] == c)[0][0])] = False
    counts = np.diff(A.rowptr) - np.add.reduceat(~keep, A.rowptr[:-1]).astype(np.int64)
    rp = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return oracle.CSR(A.n, rp, A.col[keep].copy(), A.val[keep].copy())


@pytest.mark.parametrize("mat", ["poisson16", "poisson24", "poisson32x16", "laplace64", "laplace64neu",
                                 "poisson16hole"])
def test_uniform_band_march_bitwise(ctx, mat):
    """Constant-coefficient stencils (every stored entry of a band diagonal one value): the march
    kernels take the values from their arguments instead of the band arrays, and on a grid whose
    rows store exactly their in-grid neighbours the row masks from the coordinates (poisson16hole:
    one pair missing, so the loaded masks).  eig_mv is bitwise the
    reference row loop; the classic and the fused Lanczos recurrences give alpha / beta bitwise equal
    to the array-loading kernels (EIG_MAT_NO_UNIFORM: same grid, same per-row sums), also after
    A += sigma I (the diagonal constant follows the shift).  The Neumann Laplacian's boundary rows
    have another diagonal value: not uniform, the arrays are loaded."""
    A = {"poisson16": lambda: oracle.poisson3d(16), "poisson24": lambda: oracle.poisson3d(24),
         "laplace64": lambda: oracle.laplace2d(64), "laplace64neu": lambda: oracle.laplace2d(64, "neumann"),
         "poisson16hole": lambda: _drop_pair(oracle.poisson3d(16), 1000),
         "poisson32x16": lambda: _box_poisson(32, 16, 20)}[mat]()
    kind = {"laplace64neu": 0, "poisson16hole": 1}.get(mat, 2)  # 2: uniform values + grid masks
    M = check_mv(ctx, A, True)
    R = upload(ctx, A, flags=eigmi.MAT_NO_UNIFORM)
    n = A.n
    assert M.info.sym_uniform == kind and R.info.sym_uniform == 0
    assert M.lanczos_kernel_info(True)[1] == {0: R.lanczos_kernel_info(True)[1], 1: n + 32 * n, 2: 32 * n}[kind]
    for shift in (None, 0.375):
        if shift is not None:
            M.shift_diag(shift)
            R.shift_diag(shift)
            val = A.val.copy()
            oracle.lib.orc_shift_diag(A.n, A.rowptr, A.col, val, shift)
            x = np.random.default_rng(3).standard_normal(n)
            assert np.array_equal(M.mv_host(x), oracle.csr_mv(oracle.CSR(A.nrows, A.rowptr, A.col, val), x))
        for fused in (False, True):
            a1, b1, _ = eigmi.lanczos_run(M, 30, seed=5, fused=fused)
            a2, b2, _ = eigmi.lanczos_run(R, 30, seed=5, fused=fused)
            assert np.array_equal(a1, a2) and np.array_equal(b1, b2), (shift, fused)


@pytest.mark.parametrize("fused", [False, True])
def test_march_lanczos_partial_plane(ctx, fused):
    """Lanczos on a band matrix whose rows are not a whole number of planes, march vs SELL image."""
    A = band_matrix(9000, [0, 1, 9, 128], 12)
    Ms, Mp = upload(ctx, A, True), upload(ctx, A, False)
    assert Ms.lanczos_kernel_info(fused)[0].endswith("_march")
    a1, b1, _ = eigmi.lanczos_run(Ms, 30, seed=9, fused=fused)
    a2, b2, _ = eigmi.lanczos_run(Mp, 30, seed=9, fused=fused)
    assert np.allclose(a1, a2, rtol=1e-11, atol=1e-13) and np.allclose(b1, b2, rtol=1e-11, atol=1e-13)


# ---- a2 SpMM on the band march (k_spmm8_march): 16-row wave columns, D a multiple of 16 ----

@pytest.mark.parametrize("mat,m", [
    ("poisson16", 8), ("poisson16", 24), ("laplace64", 16),
    ("band_partial", 8),     # 5000 rows, D = 144: partial last plane
    ("band_u32", 16),        # 23 offsets (u32 masks), structurally unsymmetric
    ("band_no_pm1", 8),      # no +-1: not marched (row kernels)
])
def test_march_spmm_bitwise(ctx, mat, m):
    A = {"poisson16": lambda: oracle.poisson3d(16),
         "laplace64": lambda: oracle.laplace2d(64),
         "band_partial": lambda: band_matrix(5000, [0, 1, 12, 144], 21),
         "band_u32": lambda: band_matrix(3000, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 48], 22, drop=0.1),
         "band_no_pm1": lambda: band_matrix(3000, [0, 2, 64], 23)}[mat]()
    M = upload(ctx, A, flags=eigmi.MAT_NO_CLASS)  # (the 3-D box grids would take the row-class kernel)
    assert M.info.sym_offsets > 0
    assert M.kernel("spmm8") != "k_boxc_mv8"
    Qh = oracle.random_mv8(A.n, m, 5)
    Q, Y = ctx.array(Qh), ctx.zeros(A.n * m)
    eigmi.spmm_mv8(M, m, Q, Y)
    assert np.array_equal(Y.get(), oracle.spmm_mv8(A, Qh, m))


# ---- general band march (k_spmm8_marchg): carried offset P not the widest, spans S1..S4 ----

def _p1(N, which):
    K, Mm = oracle.p1_kuhn(N)
    S = K if which == "K" else Mm
    return oracle.CSR(S.shape[0], S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data.copy())


@pytest.mark.parametrize("mat,m", [
    ("p1mass8", 8), ("p1mass8", 16), ("p1stiff8", 8), ("p1mass16", 8),
    ("band_beyond", 8),   # offsets past the carried P = 32: spans S1 / S4 non-empty
])
def test_marchg_spmm_bitwise(ctx, mat, m):
    A = {"p1mass8": lambda: _p1(8, "M"), "p1stiff8": lambda: _p1(8, "K"), "p1mass16": lambda: _p1(16, "M"),
         "band_beyond": lambda: band_matrix(4000, [0, 1, 5, 32, 35, 40], 31, drop=0.05)}[mat]()
    M = upload(ctx, A, flags=eigmi.MAT_NO_CLASS)
    assert M.info.sym_offsets > 0
    assert M.kernel("spmm8") == "k_spmm8_marchg"
    Qh = oracle.random_mv8(A.n, m, 6)
    Q, Y = ctx.array(Qh), ctx.zeros(A.n * m)
    eigmi.spmm_mv8(M, m, Q, Y)
    assert np.array_equal(Y.get(), oracle.spmm_mv8(A, Qh, m))


@pytest.mark.parametrize("N,m", [(8, 8), (16, 32)])
def test_marchg_chebyshev_matches_sell(ctx, N, m):
    """The fused Chebyshev-Jacobi mass solve (config C5) on the general band march against the
    SELL kernel (both fused multiply-adds in ascending offset order; tolerance: signed zeros)."""
    A = _p1(N, "M")
    M = upload(ctx, A, flags=eigmi.MAT_NO_CLASS)
    assert M.kernel("cheb8") == "k_spmm8_marchg_cheb"
    n = A.n
    Bh = oracle.random_mv8(n, m, 8)
    B = ctx.array(Bh)
    X1, X2 = ctx.zeros(n * m), ctx.zeros(n * m)
    eigmi.mass_solve_mv8(M, m, 12, B, X1)
    Ms = upload(ctx, A, flags=eigmi.MAT_NO_MARCH)
    assert Ms.kernel("cheb8") == "k_sell_mv8q_cheb"
    eigmi.mass_solve_mv8(Ms, m, 12, B, X2)
    a, b = X1.get(), X2.get()
    assert np.allclose(a, b, rtol=1e-13, atol=1e-14 * np.abs(b).max())
    # and the solve is a solve: M x ~ b (degree 12 Chebyshev, kappa(D^-1 M) <= 5: error ~ 2 0.38^12)
    r = oracle.spmm_mv8(A, a, m) - Bh
    assert np.linalg.norm(r) <= 1e-3 * np.linalg.norm(Bh)


# ---- 3-D box stencils, 32 columns per pass (k_box.hip: LDS-tiled plane march, config C5) ----

def _perturbed(A, rows=(1000, 2345)):
    """A with the symmetric pair of entries (i, i + 1) / (i + 1, i) scaled by 1.01 for i in rows: still
    a box stencil with a bitwise-symmetric band, but rows i, i + 1 leave their geometric class."""
    v = A.val.copy()
    for i in rows:
        for r, c in ((i, i + 1), (i + 1, i)):
            p = A.rowptr[r] + int(np.nonzero(A.col[A.rowptr[r]:A.rowptr[r + 1]] == c)[0][0])
            v[p] *= 1.01
    return oracle.CSR(A.n, A.rowptr, A.col, v)


BOX_CLASS = {"p1mass16": True, "p1stiff16": True, "p1mass20": True, "p1mass24": True, "poisson18": True,
             "p1mass16var": False, "poisson18var": False}


@pytest.mark.parametrize("mat,m", [
    ("p1mass16", 32), ("p1stiff16", 32), ("p1mass20", 32),   # 20: ragged tiles in x and y
    ("p1mass24", 64), ("poisson18", 32), ("poisson18", 96),
    ("p1mass16var", 32), ("poisson18var", 64),  # not class-constant: the full box image kernel
])
def test_box_spmm_bitwise(ctx, mat, m):
    """The box kernels' SpMM (separately rounded products and sums, ascending offsets) is bitwise the
    reference matmul_sparse_tallskinny_blocked (kernels_cpp.hh:626-657) restated in oracle.spmm_mv8:
    the row-class kernel (k_boxc_mv8: constant entries per geometric class, values from LDS) and,
    for matrices whose rows leave their class, the box-image kernel (k_box_mv32)."""
    A = {"p1mass16": lambda: _p1(16, "M"), "p1stiff16": lambda: _p1(16, "K"), "p1mass20": lambda: _p1(20, "M"),
         "p1mass24": lambda: _p1(24, "M"), "poisson18": lambda: oracle.poisson3d(18),
         "p1mass16var": lambda: _perturbed(_p1(16, "M")),
         "poisson18var": lambda: _perturbed(oracle.poisson3d(18))}[mat]()
    M = upload(ctx, A)
    assert M.kernel("spmm32") == ("k_boxc_mv8" if BOX_CLASS[mat] else "k_box_mv32")
    Qh = oracle.random_mv8(A.n, m, 7)
    Q, Y = ctx.array(Qh), ctx.zeros(A.n * m)
    eigmi.spmm_mv8(M, m, Q, Y)
    assert np.array_equal(Y.get(), oracle.spmm_mv8(A, Qh, m))


@pytest.mark.parametrize("mat,m", [("poisson16", 8), ("poisson16", 24), ("p1mass16", 8), ("p1stiff20", 16)])
def test_boxc_spmm_any_8_columns(ctx, mat, m):
    """The row-class kernel serves any multiple of 8 columns (one MultiVector block per workgroup):
    bitwise the reference SpMM (kernels_cpp.hh:626-657)."""
    A = {"poisson16": lambda: oracle.poisson3d(16), "p1mass16": lambda: _p1(16, "M"),
         "p1stiff20": lambda: _p1(20, "K")}[mat]()
    M = upload(ctx, A)
    assert M.kernel("spmm8") == "k_boxc_mv8"
    Qh = oracle.random_mv8(A.n, m, 19)
    Q, Y = ctx.array(Qh), ctx.zeros(A.n * m)
    eigmi.spmm_mv8(M, m, Q, Y)
    assert np.array_equal(Y.get(), oracle.spmm_mv8(A, Qh, m))


@pytest.mark.parametrize("N,var", [(16, False), (20, False), (16, True)])
def test_box_chebyshev_matches_sell(ctx, N, var):
    """The fused Chebyshev-Jacobi step on the box kernels (row-class and, var: box image) against the
    SELL kernel (all FMA in ascending offset order: equal up to signed zeros / the rounding of the
    fused update)."""
    A = _p1(N, "M")
    if var:
        A = _perturbed(A)
    M = upload(ctx, A)
    assert M.kernel("cheb32") == ("k_box_mv32_cheb" if var else "k_boxc_mv8_cheb")
    Ms = upload(ctx, A, flags=eigmi.MAT_NO_MARCH)
    assert Ms.kernel("cheb32") == "k_sell_mv8q_cheb"
    n, m = A.n, 32
    Bh = oracle.random_mv8(n, m, 9)
    B = ctx.array(Bh)
    X1, X2 = ctx.zeros(n * m), ctx.zeros(n * m)
    eigmi.mass_solve_mv8(M, m, 20, B, X1)
    eigmi.mass_solve_mv8(Ms, m, 20, B, X2)
    a, b = X1.get(), X2.get()
    assert np.allclose(a, b, rtol=1e-13, atol=1e-14 * np.abs(b).max())
    r = oracle.spmm_mv8(A, a, m) - Bh
    assert np.linalg.norm(r) <= 1e-6 * np.linalg.norm(Bh)


@pytest.mark.parametrize("mat,var", [("p1mass20", False), ("poisson18", False), ("p1mass16", True)])
def test_box_segments_bitwise(ctx, mat, var):
    """EIG_TUNE_BOX_SEGS (z segments per tile column) changes where a row is computed, never how:
    SpMM, residual-free Chebyshev solves of degree 2 / 3 / 7 (first / second / later step epilogues)
    are bitwise those of the automatic choice for 1 .. nz segments (ragged segment lengths included)."""
    A = {"p1mass20": lambda: _p1(20, "M"), "poisson18": lambda: oracle.poisson3d(18),
         "p1mass16": lambda: _p1(16, "M")}[mat]()
    if var:
        A = _perturbed(A)
    M = upload(ctx, A)
    n, m = A.n, 32
    nz = round(n ** (1 / 3))
    Qh = oracle.random_mv8(n, m, 23)
    Q, Y = ctx.array(Qh), ctx.zeros(n * m)
    ref = {}
    for segs in (0, 1, 2, 3, 5, nz):
        M.tune(box_segs=segs)
        eigmi.spmm_mv8(M, m, Q, Y)
        out = {"spmm": Y.get()}
        if mat.startswith("p1"):
            for d in (2, 3, 7):
                eigmi.mass_solve_mv8(M, m, d, Q, Y)
                out[d] = Y.get()
        if segs == 0:
            ref = out
            assert np.array_equal(out["spmm"], oracle.spmm_mv8(A, Qh, m))
        else:
            for k in ref:
                assert np.array_equal(out[k], ref[k]), (segs, k)
    M.tune(box_segs=0)


@pytest.mark.parametrize("mat", ["p1mass16", "poisson18"])
def test_box_no_class_flag(ctx, mat):
    """EIG_MAT_NO_CLASS keeps the box-image kernel on a class-constant matrix; both kernels give the
    reference SpMM bitwise."""
    A = _p1(16, "M") if mat == "p1mass16" else oracle.poisson3d(18)
    M = upload(ctx, A, flags=eigmi.MAT_NO_CLASS)
    assert M.kernel("spmm32") == "k_box_mv32"
    Qh = oracle.random_mv8(A.n, 32, 13)
    Q, Y = ctx.array(Qh), ctx.zeros(A.n * 32)
    eigmi.spmm_mv8(M, 32, Q, Y)
    assert np.array_equal(Y.get(), oracle.spmm_mv8(A, Qh, 32))


def _dropped(A, rows=(1000, 2345)):
    """A without the symmetric pair (i, i + 1) / (i + 1, i) for i in rows: rows that do not store an
    offset staying inside the grid (the box image kernels' runtime-mask path)."""
    keep = np.ones(len(A.col), dtype=bool)
    for i in rows:
        for r, c in ((i, i + 1), (i + 1, i)):
            keep[A.rowptr[r] + int(np.nonzero(A.col[A.rowptr[r]:A.rowptr[r + 1]] == c)[0][0])] = False
    rp = np.concatenate([[0], np.cumsum([keep[A.rowptr[r]:A.rowptr[r + 1]].sum() for r in range(A.n)])])
    return oracle.CSR(A.n, rp.astype(A.rowptr.dtype), A.col[keep], A.val[keep])


@pytest.mark.parametrize("mat", ["p1mass16var", "p1stiff20", "poisson18var", "poisson18drop", "p1mass16drop"])
def test_box_push_kernel_bitwise(ctx, mat):
    """EIG_TUNE_BOX_MAP = 1 (k_box_mv32's XCD-contiguous tile map) and EIG_TUNE_BOX_COLS = 16 (k_box_mv16p: one X plane in LDS, each row's dz = -1 / 0 / +1 groups
    added in three consecutive iterations) against k_box_mv32: the SpMM bitwise the reference
    (kernels_cpp.hh:626-657, oracle.spmm_mv8) and Chebyshev solves of degree 2 / 3 / 7 bitwise equal,
    for 1 / 3 / nz z segments, on compile-time stencils (geometric masks) and runtime masks (rows
    missing an in-grid entry: poisson18drop, p1mass16drop)."""
    A = {"p1mass16var": lambda: _perturbed(_p1(16, "M")), "p1stiff20": lambda: _p1(20, "K"),
         "poisson18var": lambda: _perturbed(oracle.poisson3d(18)),
         "poisson18drop": lambda: _dropped(oracle.poisson3d(18)),
         "p1mass16drop": lambda: _dropped(_p1(16, "M"))}[mat]()
    M = upload(ctx, A, flags=eigmi.MAT_NO_CLASS)
    n, m = A.n, 64
    nz = round(n ** (1 / 3))
    Qh = oracle.random_mv8(n, m, 29)
    Q, Y = ctx.array(Qh), ctx.zeros(n * m)
    ref = None
    for cols, segs, xmap in ((32, 0, 0), (32, 0, 1), (32, 2, 1), (16, 0, 0), (16, 1, 0), (16, 3, 0), (16, nz, 0)):
        M.tune(box_cols=cols, box_segs=segs, box_map=xmap)
        assert M.kernel("spmm32") == ("k_box_mv16p" if cols == 16 else "k_box_mv32")
        eigmi.spmm_mv8(M, m, Q, Y)
        out = {"spmm": Y.get()}
        if not mat.startswith("poisson"):  # (Chebyshev-Jacobi: the SPD mass matrices)
            for d in (2, 3, 7):
                eigmi.mass_solve_mv8(M, m, d, Q, Y)
                out[d] = Y.get()
        if ref is None:
            ref = out
            assert np.array_equal(out["spmm"], oracle.spmm_mv8(A, Qh, m))
        else:
            for k in ref:
                assert np.array_equal(out[k], ref[k]), (cols, segs, xmap, k)
    M.tune(box_cols=0, box_segs=0, box_map=0)


def test_box_shift_rebuilds_image(ctx):
    """eig_mat_shift_diag (A += sigma I) invalidates the box image; the next SpMM uses the new values."""
    A = _p1(16, "K")
    M = upload(ctx, A)
    Qh = oracle.random_mv8(A.n, 32, 11)
    Q, Y = ctx.array(Qh), ctx.zeros(A.n * 32)
    eigmi.spmm_mv8(M, 32, Q, Y)
    M.shift_diag(2.5)
    eigmi.spmm_mv8(M, 32, Q, Y)
    As = oracle.CSR(A.nrows, A.rowptr, A.col, A.val.copy())
    As.val[As.col == np.repeat(np.arange(As.n), np.diff(As.rowptr))] += 2.5
    assert np.array_equal(Y.get(), oracle.spmm_mv8(As, Qh, 32))


def test_box_not_a_grid(ctx):
    """A band that is not a 3-D box stencil (random offsets) keeps the band march / SELL kernels."""
    A = band_matrix(4000, [0, 1, 5, 32, 35, 40], 31, drop=0.05)
    M = upload(ctx, A)
    assert M.kernel("spmm32") not in ("k_box_mv32", "k_boxc_mv8")
    Qh = oracle.random_mv8(A.n, 32, 12)
    Q, Y = ctx.array(Qh), ctx.zeros(A.n * 32)
    eigmi.spmm_mv8(M, 32, Q, Y)
    assert np.array_equal(Y.get(), oracle.spmm_mv8(A, Qh, 32))


def _box_stencil(N, stencil, drop_xfirst_z=False):
    """Symmetric constant-coefficient box stencil on an N^3 grid, Dirichlet truncation: stencil maps
    (dz, dy, dx) -> value (with (-dz, -dy, -dx) the same value).  drop_xfirst_z: rows on the x = 0
    face do not couple along z (an in-grid offset their class does not store)."""
    import scipy.sparse as sp
    n = N ** 3
    r = np.arange(n)
    x, y, z = r % N, (r // N) % N, r // (N * N)
    rows, cols, vals = [], [], []
    for (dz, dy, dx), v in stencil.items():
        ok = (x + dx >= 0) & (x + dx < N) & (y + dy >= 0) & (y + dy < N) & (z + dz >= 0) & (z + dz < N)
        if drop_xfirst_z and dz != 0:
            ok &= x != 0
        rows.append(r[ok])
        cols.append(r[ok] + dz * N * N + dy * N + dx)
        vals.append(np.full(int(ok.sum()), v))
    S = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    S.sort_indices()
    return oracle.CSR(n, S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data.copy())


_P7 = {(0, 0, 0): 6.0, (1, 0, 0): -1.0, (-1, 0, 0): -1.0, (0, 1, 0): -1.0, (0, -1, 0): -1.0,
       (0, 0, 1): -1.0, (0, 0, -1): -1.0}


@pytest.mark.parametrize("kind,var", [("hole", False), ("nine", False), ("hole", True), ("nine", True),
                                      ("full27", False)])
def test_boxc_runtime_offsets(ctx, kind, var):
    """The row-class kernels take the compile-time stencil (7-point, Kuhn 15-point: no masks, every
    offset summed with the zero class entries) only when every offset a class does not store points
    out of the grid; otherwise -- hole: x = 0 rows drop their in-grid z couplings -- and for other
    shapes -- nine: the 7-point plus one face diagonal -- the runtime offset loop with the row masks.
    var: two rows leave their class -- the box-image kernel (k_box_mv32), same rule.  All bitwise
    the reference SpMM; the Chebyshev step equal to the SELL kernel to rounding."""
    st = dict(_P7)
    if kind == "full27":  # every box offset (a Galerkin coarse operator's shape): compile-time 27-point
        st = {(a, b, c): (-0.05 if (a, b, c) != (0, 0, 0) else 2.0) for a in (-1, 0, 1) for b in (-1, 0, 1)
              for c in (-1, 0, 1)}
    if kind == "nine":
        st[(0, 1, 1)] = st[(0, -1, -1)] = -0.25
        st[(0, 0, 0)] = 6.5
    A = _box_stencil(17, st, drop_xfirst_z=(kind == "hole"))
    if var:
        A = _perturbed(A, rows=(1000, 2344))  # (x = 14, 15 on the 17-grid: the pair (i, i + 1) exists)
    M = upload(ctx, A)
    assert M.kernel("spmm32") == ("k_box_mv32" if var else "k_boxc_mv8")
    for m in (8, 32):
        Qh = oracle.random_mv8(A.n, m, 23)
        Q, Y = ctx.array(Qh), ctx.zeros(A.n * m)
        eigmi.spmm_mv8(M, m, Q, Y)
        assert np.array_equal(Y.get(), oracle.spmm_mv8(A, Qh, m))
    Ms = upload(ctx, A, flags=eigmi.MAT_NO_MARCH)
    Bh = oracle.random_mv8(A.n, 32, 29)
    B = ctx.array(Bh)
    X1, X2 = ctx.zeros(A.n * 32), ctx.zeros(A.n * 32)
    lo, hi = 0.1, 2.0  # (the two kernels run the same recurrence; convergence is not the point)
    eigmi.mass_solve_mv8(M, 32, 12, B, X1, lo, hi)
    eigmi.mass_solve_mv8(Ms, 32, 12, B, X2, lo, hi)
    a, b = X1.get(), X2.get()
    assert np.allclose(a, b, rtol=1e-13, atol=1e-14 * np.abs(b).max()), np.abs(a - b).max()


def test_boxc_compile_time_stencils(ctx):
    """The 7-point and Kuhn 15-point stencils with zero (not absent) boundary entries: the
    compile-time kernels sum the shape's offsets with zero class entries -- bitwise the reference,
    which skips absent entries (a sum starting at +0 is unchanged by adding +-0) -- also when X holds
    exact zeros and negative values next to the faces."""
    for A in (oracle.poisson3d(16), _p1(16, "K")):
        M = upload(ctx, A)
        assert M.kernel("spmm32") == "k_boxc_mv8"
        Qh = oracle.random_mv8(A.n, 32, 31)
        Qh[::7] = 0.0
        Qh[1::11] = -0.0
        Q, Y = ctx.array(Qh), ctx.zeros(A.n * 32)
        eigmi.spmm_mv8(M, 32, Q, Y)
        ref = oracle.spmm_mv8(A, Qh, 32)
        got = Y.get()
        assert np.array_equal(got, ref)
        assert np.array_equal(np.signbit(got), np.signbit(ref))


def test_box_chebyshev_first_step_after_other_class_table(ctx):
    """The first Chebyshev step (x_1 = gamma D^-1 b formed as b enters the LDS ring) reads the class
    table in its prologue: right after a row-class SpMM on another matrix (whose table the CU's LDS
    still holds) a degree-2 and a degree-3 solve of the mass matrix equal the SELL kernel's."""
    K, Mh = _p1(16, "K"), _p1(16, "M")
    dK, dM = upload(ctx, K), upload(ctx, Mh)
    dMs = upload(ctx, Mh, flags=eigmi.MAT_NO_MARCH)
    n, m = Mh.n, 32
    Bh = oracle.random_mv8(n, m, 41)
    B, Y = ctx.array(Bh), ctx.zeros(n * m)
    X1, X2 = ctx.zeros(n * m), ctx.zeros(n * m)
    for degree in (2, 3):
        eigmi.spmm_mv8(dK, m, B, Y)  # another class table through the same kernel's LDS
        eigmi.mass_solve_mv8(dM, m, degree, B, X1)
        eigmi.mass_solve_mv8(dMs, m, degree, B, X2)
        a, b = X1.get(), X2.get()
        assert np.all(np.isfinite(a))
        assert np.allclose(a, b, rtol=1e-13, atol=1e-14 * np.abs(b).max()), (degree, np.abs(a - b).max())


@pytest.mark.parametrize("mat", ["poisson16", "poisson24", "laplace64", "poisson32x16"])
def test_geometric_march_prefetch_bitwise(ctx, mat):
    """The geometric march variants (eig_mat_tune EIG_TUNE_MARCH_PREFETCH: 1 = plain march_rows, 2-4 =
    march_rows_geo with the +D operand 1-3 planes ahead, 5 = plus the gathers one plane ahead; 6-8 =
    march_rows_geo2: no masks or selects, missing neighbours read as exact zeros) only reorder loads
    or add exact zeros: eig_mv bitwise the reference row loop, classic and fused Lanczos alpha / beta
    bitwise equal to the plain march at the same plane runs -- including runs whose plane counts leave
    every remainder of the unrolled loop (1, 2, 3, 5 and 7 runs)."""
    A = {"poisson16": lambda: oracle.poisson3d(16), "poisson24": lambda: oracle.poisson3d(24),
         "laplace64": lambda: oracle.laplace2d(64), "poisson32x16": lambda: _box_poisson(32, 16, 20)}[mat]()
    M = check_mv(ctx, A, True)
    assert M.info.sym_uniform == 2
    x = np.random.default_rng(11).standard_normal(A.n)
    ref_mv = oracle.csr_mv(A, x)
    for runs in (0, 1, 2, 3, 5, 7):
        base = {}
        for pf in (1, 2, 3, 4, 5, 6, 7, 8):
            M.tune(runs, march_prefetch=pf)
            assert np.array_equal(M.mv_host(x), ref_mv), (runs, pf)
            for fused in (False, True):
                a, b, _ = eigmi.lanczos_run(M, 25, seed=7, fused=fused)
                if pf == 1:
                    base[fused] = (a, b)
                else:
                    assert np.array_equal(a, base[fused][0]) and np.array_equal(b, base[fused][1]), (runs, pf, fused)
    M.tune(0, march_prefetch=0)


@pytest.mark.parametrize("N", [64, 128])
def test_geo2_grids_vs_oracle(ctx, N):
    """The automatic geometric march on grids whose x extent is a multiple of 64 (geo2: raw buffer
    loads, missing neighbours read as exact zeros) -- and, at these sizes, the fused step's plain
    (MALL-resident) stores: eig_mv bitwise the reference row loop, the fused and classic recurrences
    vs their restatements (rtol 1e-12)."""
    A = oracle.poisson3d(N)
    M = check_mv(ctx, A, True)
    assert M.info.sym_uniform == 2
    assert M.lanczos_kernel_info(True)[0] == "k_lanczos_fused_march"
    fa, fb, _ = eigmi.lanczos_run(M, 20, seed=123, fused=True)
    qa, qb = oracle.lanczos_fused(A, oracle.random_vec(A.n, 123), 20)
    assert np.allclose(fa, qa, rtol=1e-12) and np.allclose(fb, qb, rtol=1e-12)
    ca, cb, _ = eigmi.lanczos_run(M, 20, seed=123)
    _, ra, rb = oracle.lanczos(A, oracle.random_vec(A.n, 123), 20)
    assert np.allclose(ca, ra, rtol=1e-12) and np.allclose(cb, rb, rtol=1e-12)
