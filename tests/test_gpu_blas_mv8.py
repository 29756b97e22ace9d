"""GPU parity: BlockVector ops and the MultiVector<double,8> kernels (SpMM, dots, MFMA Gram,
block Gram-Schmidt, B-Gram-Schmidt) vs the oracle.  Element-wise kernels that keep the
reference's operation order are compared BITWISE; reductions (different summation order) within
the tolerance written at each assert."""
import numpy as np
import pytest

import eigmi
import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 1, 7, 1000, 65537, 1 << 20])
def test_blas1(ctx, n):
    rng = np.random.default_rng(n)
    x, y = rng.standard_normal(n), rng.standard_normal(n)
    dx, dy, out = ctx.array(x), ctx.array(y), ctx.zeros(2)
    eigmi.dot(ctx, n, dx, dy, out)
    d = out.get(1)[0]
    # tolerance: |sum order error| <= n * eps * sum |x_i y_i|
    assert abs(d - np.dot(x, y)) <= 4 * max(n, 1) * 2.3e-16 * np.abs(x * y).sum() + 1e-300
    eigmi.nrm2(ctx, n, dx, out)
    assert abs(out.get(1)[0] - np.sqrt(np.dot(x, x))) <= 1e-13 * max(1.0, np.sqrt(np.dot(x, x)))
    eigmi.axpy(ctx, n, -0.75, dx, dy)
    assert np.array_equal(dy.get(), y + (-0.75) * x)  # y += a x, one rounding per op: bitwise
    eigmi.scal(ctx, n, 3.0, dx)
    assert np.array_equal(dx.get(), x * 3.0)
    dz = ctx.zeros(n)
    eigmi.copy(ctx, n, dx, dz)
    ctx.sync()
    assert np.array_equal(dz.get(), x * 3.0)


@pytest.mark.parametrize("n", [0, 1, 7, 1000, 65537, 1 << 20])
@pytest.mark.parametrize("three_term", [True, False])
def test_lanczos_update(ctx, n, three_term):
    """eig_lanczos_update (SURVEY 8(b) BlockVector ops): the ARPACK-style update of the vector the
    operator callback returned (arpack_geneo_wrapper.hh:257-279), w <- (w - alpha v) - beta vprev,
    BITWISE the same two roundings per entry as numpy's elementwise order; ||w|| and v.w of the new
    w within the summation-order bound."""
    rng = np.random.default_rng(100 + n)
    v, p, w = rng.standard_normal(n), rng.standard_normal(n), rng.standard_normal(n)
    alpha, beta = 0.37, -1.25
    dv, dp, dw = ctx.array(v), ctx.array(p), ctx.array(w)
    da, db, out = ctx.array([alpha]), ctx.array([beta]), ctx.zeros(2)
    eigmi.lanczos_update(ctx, n, da, db if three_term else None, dv, dp if three_term else None, dw, out)
    ref = w - alpha * v
    if three_term:
        ref = ref - beta * p
    got = dw.get()
    assert np.array_equal(got, ref)
    nrm, vw = out.get(2)
    assert abs(nrm - np.sqrt(ref @ ref)) <= 1e-13 * max(1.0, np.sqrt(ref @ ref))
    assert abs(vw - v @ ref) <= 4 * max(n, 1) * 2.3e-16 * np.abs(v * ref).sum() + 1e-300


def test_random_mv8_bitwise(ctx):
    n, m = 1000, 16
    Q = ctx.zeros(n * m)
    eigmi.random_mv8(ctx, n, m, 123, Q)
    assert np.array_equal(Q.get(), oracle.random_mv8(n, m, 123))


@pytest.mark.parametrize("m", [8, 16, 40])
def test_spmm_bitwise(ctx, m):
    A = oracle.poisson3d(12)
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    Qh = oracle.random_mv8(A.n, m, 11)
    Q, Y = ctx.array(Qh), ctx.zeros(A.n * m)
    eigmi.spmm_mv8(M, m, Q, Y)
    assert np.array_equal(Y.get(), oracle.spmm_mv8(A, Qh, m))


def _ragged(n=1000, seed=5):
    """Irregular rows (0 to ~30 entries, n not a multiple of 64, an explicitly stored zero):
    the explicit-column SELL image with padding."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    S = sp.random(n, n, density=0.012, random_state=rng, format="csr")
    S = (S + sp.diags(rng.uniform(1, 2, n))).tocsr()
    S.sort_indices()
    S.data[3] = 0.0
    return oracle.CSR(n, S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data.copy())


@pytest.mark.parametrize("m", [8, 16, 40])
@pytest.mark.parametrize("which", ["ragged", "p1mass"])
def test_spmm_bitwise_explicit_columns(ctx, m, which):
    """Matrices without a stencil image (every mapping: the m = 8 single-block kernel and the
    multi-block one) against the restated matmul_sparse_tallskinny_blocked, bitwise."""
    if which == "ragged":
        A = _ragged()
    else:
        K, Mm = oracle.p1_kuhn(7)
        A = oracle.CSR(Mm.shape[0], Mm.indptr.astype(np.int64), Mm.indices.astype(np.int32), Mm.data.copy())
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    Qh = oracle.random_mv8(A.n, m, 11)
    Q, Y = ctx.array(Qh), ctx.zeros(A.n * m)
    eigmi.spmm_mv8(M, m, Q, Y)
    assert np.array_equal(Y.get(), oracle.spmm_mv8(A, Qh, m))


def test_spmm_rejects_blocks_and_bad_m(ctx):
    A = oracle.q1elast(3)
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, 3, 3)
    Q = ctx.zeros(A.n * 8)
    with pytest.raises(eigmi.EigShapeError):
        eigmi.spmm_mv8(M, 8, Q, Q)
    A1 = oracle.laplace2d(8)
    M1 = eigmi.Matrix.from_bcsr(ctx, A1.rowptr, A1.col, A1.val)
    with pytest.raises(eigmi.EigShapeError):
        eigmi.spmm_mv8(M1, 12, Q, Q)  # "number of cols must be a multiple of block size"


@pytest.mark.parametrize("n,m", [(4096, 8), (4096, 32), (12345, 16)])
def test_dot_diag(ctx, n, m):
    Q1h, Q2h = oracle.random_mv8(n, m, 1), oracle.random_mv8(n, m, 2)
    dp = ctx.zeros(m)
    eigmi.dot_diag_mv8(ctx, n, m, ctx.array(Q1h), ctx.array(Q2h), dp)
    ref = oracle.dot_diag_mv8(Q1h, Q2h, n, m)
    X1, X2 = oracle.mv_to_cols(Q1h, n, m), oracle.mv_to_cols(Q2h, n, m)
    bound = 4 * n * 2.3e-16 * np.einsum("ij,ij->j", np.abs(X1), np.abs(X2))
    assert np.all(np.abs(dp.get() - ref) <= bound)


@pytest.mark.parametrize("n,m1,m2", [(4096, 8, 8), (4096, 16, 16), (3001, 8, 24), (10000, 32, 32), (777, 48, 8),
                                     (1, 8, 8), (13, 24, 40), (5003, 40, 56), (1 << 21, 8, 24), (300007, 32, 32)])
def test_gram_mfma(ctx, n, m1, m2):
    Q1h, Q2h = oracle.random_mv8(n, m1, 3), oracle.random_mv8(n, m2, 4)
    G, G2 = ctx.zeros(m1 * m2), ctx.zeros(m1 * m2)
    dQ1, dQ2 = ctx.array(Q1h), ctx.array(Q2h)
    eigmi.gram_mv8(ctx, n, m1, m2, dQ1, dQ2, G)
    eigmi.gram_mv8(ctx, n, m1, m2, dQ1, dQ2, G2)
    assert np.array_equal(G.get(), G2.get())  # deterministic reduction order
    X1, X2 = oracle.mv_to_cols(Q1h, n, m1), oracle.mv_to_cols(Q2h, n, m2)
    ref = X1.T @ X2
    if m1 == m2:
        assert np.allclose(oracle.gram_mv8(Q1h, Q2h, n, m1), ref, atol=1e-11)
    bound = 4 * n * 2.3e-16 * (np.abs(X1).T @ np.abs(X2))
    assert np.all(np.abs(G.get().reshape(m1, m2) - ref) <= bound)


@pytest.mark.parametrize("variant,name", [(eigmi.ORTHO_MGS, "mgs"), (eigmi.ORTHO_CHOLQR, "cholqr"),
                                          (eigmi.ORTHO_CHOLQR_SPLIT, "cholqr_split")])
@pytest.mark.parametrize("n,m", [(4096, 8), (4096, 32), (5000, 16), (100, 8), (1000, 16), (2048, 8)])
def test_orthonormalize_blocked(ctx, variant, name, n, m):
    Qh = oracle.random_mv8(n, m, 21)
    Q = ctx.array(Qh)
    eigmi.orthonormalize_mv8(ctx, n, m, Q, variant)
    got = oracle.mv_to_cols(Q.get(), n, m)
    ref = oracle.mv_to_cols(oracle.orthonormalize_mv8(Qh, n, m, name), n, m)
    assert np.abs(got.T @ got - np.eye(m)).max() < 1e-13
    # same thin QR as the reference algorithm: elementwise within 1e-12 (random, well conditioned)
    assert np.abs(got - ref).max() < 1e-12


@pytest.mark.parametrize("L", [1, 2, 4, 8])
@pytest.mark.parametrize("n,m", [(20000, 8), (50001, 24)])
def test_mgs_lookahead(ctx, L, n, m):
    """The grid-wide MGS with Gram look-ahead (k_mgs_la, EIG_ORTHO_LOOKAHEAD(L)): at most L steps per
    read pass, the later ones from the Schur complement of the window's Gram rows.  Well conditioned
    input: every look-ahead is taken, so the last diagonal block takes ceil(8 / L) read passes, and Q
    is within 1e-12 of the stepwise restatement orc_orthonormalize_mv8 (kernels_cpp.hh:180-351).
    L = 1 is the stepwise replay (one pass per step)."""
    Qh = oracle.random_mv8(n, m, 31)
    Q = ctx.array(Qh)
    eigmi.orthonormalize_mv8(ctx, n, m, Q, eigmi.ORTHO_MGS | eigmi.ORTHO_LOOKAHEAD(L))
    passes = eigmi.orthonormalize_passes(ctx)
    got = oracle.mv_to_cols(Q.get(), n, m)
    ref = oracle.mv_to_cols(oracle.orthonormalize_mv8(Qh, n, m, "mgs"), n, m)
    print(f"look-ahead L={L} n={n} m={m}: {passes} read passes, |Q - Q_ref| = {np.abs(got - ref).max():.2e}")
    assert np.abs(got.T @ got - np.eye(m)).max() < 1e-13
    assert np.abs(got - ref).max() < 1e-12
    if L > 1:
        assert passes == -(-8 // L)


@pytest.mark.parametrize("coop", [True, False], ids=["coop", "launches"])
@pytest.mark.parametrize("L", [2, 8])
def test_mgs_lookahead_refused(ctx, L, coop):
    """A column nearly in the span of the one before it (column 3 = column 2 + 1e-2 noise: after the
    projection it keeps ~1e-4 of its squared norm, below the 1/16 gate): the look-ahead step for it is
    refused and the next pass starts there with a direct row, so the block takes one pass more than
    the well conditioned case for L = 8 (steps 0-2, then 3-7) and five for L = 2 (0-1, 2, 3-4, 5-6,
    7).  Q stays orthonormal and within the conditioning-scaled tolerance of the restatement.  By
    default the refused steps run inside the last launch between grid barriers; with
    EIG_ORTHO_NO_COOP as separate launches of the 9-launch worst case -- the same Q bit for bit."""
    n, m = 30000, 8
    X = oracle.mv_to_cols(oracle.random_mv8(n, m, 41), n, m)
    X[:, 3] = X[:, 2] + 1e-2 * X[:, 3]
    Qh = oracle.cols_to_mv(X)
    Q = ctx.array(Qh)
    flags = 0 if coop else eigmi.ORTHO_NO_COOP
    eigmi.orthonormalize_mv8(ctx, n, m, Q, eigmi.ORTHO_MGS | eigmi.ORTHO_LOOKAHEAD(L) | flags)
    passes = eigmi.orthonormalize_passes(ctx)
    Q2 = ctx.array(Qh)
    eigmi.orthonormalize_mv8(ctx, n, m, Q2, eigmi.ORTHO_MGS | eigmi.ORTHO_LOOKAHEAD(L) | (flags ^ eigmi.ORTHO_NO_COOP))
    assert np.array_equal(Q.get(), Q2.get())
    got = oracle.mv_to_cols(Q.get(), n, m)
    ref = oracle.mv_to_cols(oracle.orthonormalize_mv8(Qh, n, m, "mgs"), n, m)
    cond = np.linalg.cond(X)
    print(f"refused look-ahead L={L}: cond {cond:.1e}, {passes} read passes, |Q - Q_ref| = "
          f"{np.abs(got - ref).max():.2e}, |Q^T Q - I| = {np.abs(got.T @ got - np.eye(m)).max():.2e}")
    assert passes == {2: 5, 8: 2}[L]
    assert np.abs(got.T @ got - np.eye(m)).max() < 1e-14 * cond
    assert np.abs(got - ref).max() < 1e-14 * cond


def test_cholqr_split_half_order(ctx):
    """orthonormalize_avx2_b8 (kernels_avx2.hh:255-381) projects a later block with columns 0-3 of
    the diagonal block, then 4-7 against the updated block; _v2 (:385-622) in one 8x8 step.  The two
    orders are the same mathematics and differ by rounding only (tests/test_oracle.py shows ~5e-9 on
    nearly dependent blocks, where the Gram sums' own order moves results as much), so the device
    check is: the split variant is a different operation sequence from the single projection (not
    bitwise equal) and within 1e-12 of its restatement on well-conditioned input."""
    n, m = 3000, 24
    Qh = oracle.random_mv8(n, m, 11)
    Qs, Q1 = ctx.array(Qh), ctx.array(Qh)
    eigmi.orthonormalize_mv8(ctx, n, m, Qs, eigmi.ORTHO_CHOLQR_SPLIT)
    eigmi.orthonormalize_mv8(ctx, n, m, Q1, eigmi.ORTHO_CHOLQR)
    a, b = Qs.get(), Q1.get()
    assert not np.array_equal(a, b)
    ref = oracle.orthonormalize_mv8(Qh, n, m, "cholqr_split")
    assert np.abs(a - ref).max() < 1e-12


@pytest.mark.parametrize("n,m", [(3000, 16), (4096, 8), (513, 8)])
def test_mgs_small_vs_grid(ctx, n, m):
    """n <= 4096 on one rank: the diagonal block's MGS in one workgroup (k_mgs_small, EIG_ORTHO_ONE_WG)
    and the grid-wide passes (the default look-ahead, and variant | EIG_ORTHO_GRID) do the same per-row
    operations, so they agree to the rounding of the sums' order."""
    Qh = oracle.random_mv8(n, m, 5)
    Qa, Qb = ctx.array(Qh), ctx.array(Qh)
    eigmi.orthonormalize_mv8(ctx, n, m, Qa, eigmi.ORTHO_MGS | eigmi.ORTHO_ONE_WG)
    eigmi.orthonormalize_mv8(ctx, n, m, Qb, eigmi.ORTHO_MGS | eigmi.ORTHO_GRID)
    a, b = Qa.get(), Qb.get()
    assert np.all(np.isfinite(a)) and np.abs(a - b).max() < 1e-13


def test_orthonormalize_naive(ctx):
    n, m = 3000, 12
    X = np.random.default_rng(8).standard_normal((n, m))
    cm = np.ascontiguousarray(X.T.reshape(-1))
    Q = ctx.array(cm)
    eigmi.orthonormalize_naive(ctx, n, m, Q)
    got = Q.get().reshape(m, n).T
    ref = oracle.orthonormalize_naive(cm, n, m).reshape(m, n).T
    assert np.abs(got - ref).max() < 1e-12


@pytest.mark.parametrize("kind", ["laplace", "identity"])
def test_b_orthonormalize(ctx, kind):
    N, m = 48, 24
    B = oracle.laplace2d(N) if kind == "laplace" else oracle.laplace2d(N, "identity")
    n = B.n
    Qh = oracle.random_mv8(n, m, 77)
    MB = eigmi.Matrix.from_bcsr(ctx, B.rowptr, B.col, B.val)
    Q, norm = ctx.array(Qh), ctx.zeros(1)
    eigmi.b_orthonormalize_mv8(MB, m, Q, norm)
    refQ, refnorm = oracle.b_orthonormalize_mv8(B, Qh, n, m)
    got = oracle.mv_to_cols(Q.get(), n, m)
    Bs = B.to_scipy()
    orth = np.abs(got.T @ (Bs @ got) - np.eye(m)).max()
    diff = np.abs(got - oracle.mv_to_cols(refQ, n, m)).max()
    print(f"B-orthonormalize {kind}: |Q^T B Q - I| = {orth:.3e}, |Q - Q_ref| = {diff:.3e}")
    assert orth < 1e-10
    assert diff < 1e-12
    assert abs(norm.get(1)[0] - refnorm) <= 1e-12 * abs(refnorm)


@pytest.mark.parametrize("name", ["poisson3d_20_class", "varcoef3d_24_march", "laplace2d_64", "random_sell"])
def test_spmm_dot_gram_pair(ctx, name):
    """The StandardLargest pair (eigensolver.hh:78-85, m = 8): eig_spmm_dot_gram_mv8's product BITWISE the
    reference SpMM (kernels_cpp.hh:626-657) on every image -- the row-class box kernel, the band march,
    and the fallback (product + panel Gram) on a SELL-only matrix --, its diagonal dots and window Gram
    within the summation-order bound of the restated dot_products_diagonal_blocked / _all_blocked; then
    eig_orthonormalize_gram_mv8 from that Gram within 1e-12 of the restated orthonormalize_blocked."""
    import scipy.sparse as sp
    flags = 0
    if name == "poisson3d_20_class":
        A = oracle.poisson3d(20)
    elif name == "varcoef3d_24_march":  # (no row classes: the band march with the Gram epilogue)
        rp, c, v = eigmi.gen_matrix(eigmi.GEN_VARCOEF3D, 24)
        A = oracle.CSR(24 ** 3, rp, c, v)
    elif name == "laplace2d_64":
        A = oracle.laplace2d(64)
    else:
        n0 = 3000
        S = sp.random(n0, n0, density=6.0 / n0, random_state=8, format="csr")
        S = (S + S.T + sp.identity(n0) * 8.0).tocsr()
        S.sort_indices()
        A = oracle.CSR(n0, S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data.astype(np.float64))
        flags = eigmi.MAT_NO_BAND
    n, m = A.n, 8
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, flags=flags)
    Xh = oracle.random_mv8(n, m, 31)
    X, Y, dp, G = ctx.array(Xh), ctx.zeros(n * m), ctx.zeros(8), ctx.zeros(64)
    eigmi.spmm_dot_gram_mv8(M, m, X, Y, dp, G)
    Yh = Y.get()
    assert np.array_equal(Yh, oracle.spmm_mv8(A, Xh, m))
    Xc, Yc = oracle.mv_to_cols(Xh, n, m), oracle.mv_to_cols(Yh, n, m)
    bound_d = 4 * n * 2.3e-16 * np.einsum("ij,ij->j", np.abs(Xc), np.abs(Yc))
    assert np.all(np.abs(dp.get() - oracle.dot_diag_mv8(Xh, Yh, n, m)) <= bound_d)
    Gref = oracle.gram_mv8(Yh, Yh, n, m)
    bound_g = 4 * n * 2.3e-16 * (np.abs(Yc).T @ np.abs(Yc))
    g = G.get().reshape(8, 8)
    up = np.triu(np.ones((8, 8), bool))
    assert np.all(np.abs(g - Gref)[up] <= bound_g[up])
    eigmi.orthonormalize_gram_mv8(ctx, n, m, Y, G)
    ctx.sync()
    ref = oracle.orthonormalize_mv8(Yh, n, m)
    assert np.abs(Y.get() - ref).max() < 1e-12 * max(1.0, np.abs(ref).max())
