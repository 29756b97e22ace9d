"""Config C5: the generalised pencil K x = lambda M x of P1 on the Kuhn split, block
Lanczos k=32 with the tall-skinny panels on MFMA.

CPU: the product generator (gen.cpp kinds 6/7, row-by-row assembly) against the independent
global element assembly in oracle.p1_kuhn -- identical pattern, values to 1e-15 relative.
GPU: the panel kernels against numpy, the Chebyshev mass solve against scipy's sparse direct
solve, and the block Lanczos Ritz values against (a) the numpy restatement of the same recurrence
(oracle.block_lanczos_gen, same start block) and (b) the exact eigenvalues of (K, M) from
scipy.linalg.eigh -- the answer the reference's GeneralizedInverse / ARPACK shift-invert path
computes (eigensolver.hh:204-351, arpack_geneo_wrapper.hh:581-658).

Tolerances: panel Gram / update 1e-13 relative (summation order differs from numpy); mass solve
1e-12 relative at degree 36 (Chebyshev bound 2 rho^36 ~ 2e-15 in the D-norm); Ritz values vs the
numpy recurrence 1e-9 relative (unconverged values amplify rounding differences), converged
extreme eigenvalues vs eigh 1e-9 relative."""
import numpy as np
import pytest

import eigmi
import oracle


@pytest.mark.parametrize("N", [1, 2, 3, 6])
def test_p1_generator_matches_global_assembly(N):
    K, M = oracle.p1_kuhn(N)
    for kind, ref in ((eigmi.GEN_P1STIFF3D, K), (eigmi.GEN_P1MASS3D, M)):
        rp, c, v = eigmi.gen_matrix(kind, N)
        assert eigmi.lib.eig_gen_nnzb(kind, N) == ref.nnz
        assert np.array_equal(rp, ref.indptr) and np.array_equal(c, ref.indices)
        assert np.max(np.abs(v - ref.data)) <= 1e-15 * np.max(np.abs(ref.data))


def test_p1_known_answers():
    """K = h * (7-point Laplacian) on the shared 15-point pattern (the Kuhn split's P1 stiffness),
    M symmetric positive definite, and the Jacobi-scaled mass spectrum inside Wathen's element
    bound [1/2, 5/2] that the Chebyshev solve relies on."""
    N = 6
    K, M = oracle.p1_kuhn(N)
    L7 = oracle.poisson3d(N).to_scipy()
    assert abs(K - L7 / (N + 1)).max() <= 1e-15
    d = 1.0 / np.sqrt(M.diagonal())
    w = np.linalg.eigvalsh((M.multiply(d[:, None]).multiply(d[None, :])).toarray())
    assert 0.5 <= w[0] and w[-1] <= 2.5


def test_p1_rows_partition():
    N = 5
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_P1MASS3D, N)
    b, cnt = 40, 50
    rr, cc, vv = eigmi.gen_rows(eigmi.GEN_P1MASS3D, N, b, cnt)
    assert np.array_equal(cc[:rr[-1]], c[rp[b]:rp[b + cnt]])
    assert np.array_equal(vv[:rr[-1]], v[rp[b]:rp[b + cnt]])


def _upload(ctx, A):
    return eigmi.Matrix.from_bcsr(ctx, A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data)


@pytest.mark.gpu
@pytest.mark.parametrize("n,m1,m2", [(1000, 32, 32), (5003, 96, 32), (777, 8, 16), (20000, 160, 24),
                                     (300007, 96, 32), (4097, 48, 16), (3, 16, 16)])
def test_panel_gram(ctx, n, m1, m2):
    rng = np.random.default_rng(n)
    Q1, Q2 = rng.standard_normal((n, m1)), rng.standard_normal((n, m2))
    d1, d2, G = ctx.array(oracle.cols_to_mv(Q1)), ctx.array(oracle.cols_to_mv(Q2)), ctx.zeros(m1 * m2)
    eigmi.panel_gram_mv8(ctx, n, m1, m2, d1, d2, G)
    g = G.get().reshape(m1, m2)
    ref = Q1.T @ Q2
    assert np.max(np.abs(g - ref)) <= 1e-13 * np.max(np.abs(Q1).sum(0)[:, None] * np.abs(Q2).max())
    eigmi.panel_gram_mv8(ctx, n, m1, m2, d1, d2, G)
    assert np.array_equal(G.get().reshape(m1, m2), g), "panel Gram must be run-to-run deterministic"


@pytest.mark.gpu
@pytest.mark.parametrize("n,m1,m2,alpha,beta", [(1000, 32, 32, -1.0, 1.0), (4099, 64, 8, 1.0, 0.0),
                                                 (333, 8, 24, 0.5, -2.0)])
def test_panel_update(ctx, n, m1, m2, alpha, beta):
    rng = np.random.default_rng(m1 + m2)
    Q, S, Y = rng.standard_normal((n, m1)), rng.standard_normal((m1, m2)), rng.standard_normal((n, m2))
    dq, ds, dy = ctx.array(oracle.cols_to_mv(Q)), ctx.array(S.ravel()), ctx.array(oracle.cols_to_mv(Y))
    eigmi.panel_update_mv8(ctx, n, m1, m2, dq, ds, alpha, beta, dy)
    got = oracle.mv_to_cols(dy.get(), n, m2)
    ref = beta * Y + alpha * (Q @ S)
    assert np.max(np.abs(got - ref)) <= 1e-13 * (np.abs(Q) @ np.abs(S)).max()


@pytest.mark.gpu
def test_panel_update_in_place(ctx):
    n, m = 2000, 16
    rng = np.random.default_rng(7)
    Q, S = rng.standard_normal((n, m)), np.triu(rng.standard_normal((m, m)))
    dq, ds = ctx.array(oracle.cols_to_mv(Q)), ctx.array(S.ravel())
    eigmi.panel_update_mv8(ctx, n, m, m, dq, ds, 1.0, 0.0, dq)
    assert np.allclose(oracle.mv_to_cols(dq.get(), n, m), Q @ S, rtol=0, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("N,m", [(8, 8), (12, 32)])
def test_mass_solve(ctx, N, m):
    import scipy.sparse.linalg as sla
    _, Mh = oracle.p1_kuhn(N)
    M = _upload(ctx, Mh)
    n = N ** 3
    B = np.random.default_rng(N).standard_normal((n, m))
    dB, dX = ctx.array(oracle.cols_to_mv(B)), ctx.zeros(n * m)
    eigmi.mass_solve_mv8(M, m, 36, dB, dX)
    X = oracle.mv_to_cols(dX.get(), n, m)
    Xe = sla.spsolve(Mh.tocsc(), B)
    assert np.max(np.abs(X - Xe)) <= 1e-12 * np.max(np.abs(Xe))
    Xo = oracle.cheb_solve(Mh, B, 36)
    assert np.max(np.abs(X - Xo)) <= 1e-13 * np.max(np.abs(Xo))


@pytest.mark.gpu
def test_block_lanczos_vs_recurrence_and_eigh(ctx):
    import scipy.linalg as sl
    N, b, steps = 10, 32, 14
    Kh, Mh = oracle.p1_kuhn(N)
    n = N ** 3
    K, M = _upload(ctx, Kh), _upload(ctx, Mh)
    bl = eigmi.BlockLanczos(K, M, block=b, max_steps=steps, degree=36, seed=123)
    t = bl.step(steps)
    assert t.steps == steps and t.total_ms > 0
    T = bl.tmatrix()
    V0 = oracle.mv_to_cols(oracle.random_mv8(n, b, 123), n, b)
    Tref, _ = oracle.block_lanczos_gen(Kh, Mh, V0, steps)
    th, thr = np.linalg.eigvalsh(T), np.linalg.eigvalsh(Tref)
    assert np.max(np.abs(th - thr) / np.abs(thr)) <= 1e-9
    exact = sl.eigh(Kh.toarray(), Mh.toarray(), eigvals_only=True)
    ev, Y, res = bl.ritz(8, eigmi.WHICH_LA, want_evec=True)
    assert np.max(np.abs(ev - exact[::-1][:8]) / exact[::-1][:8]) <= 1e-9
    # the device residuals ||K y - theta M y|| are the host's on the returned vectors; relative to
    # |theta| ||M y|| they are ~ sqrt(eigenvalue error) at this Krylov dimension
    R = (Kh @ Y.T) - (Mh @ Y.T) * ev[None, :]
    host_res = np.linalg.norm(R, axis=0)
    assert np.allclose(res, host_res, rtol=1e-6, atol=0)
    assert np.all(host_res / (ev * np.linalg.norm(Mh @ Y.T, axis=0)) <= 1e-4)
    # Ritz vectors are M-orthonormal
    G = Y @ (Mh @ Y.T)
    assert np.max(np.abs(G - np.eye(8))) <= 1e-9
    bl.close()


@pytest.mark.gpu
def test_cholqr2_ill_conditioned_block(ctx):
    """ADVICE r3 (blanczos.cpp mcholqr2): when the first CholQR pass's R is ill-conditioned (a block
    whose directions run out) the second pass recomputes M (Z R0^-1) instead of reusing (M Z) R0^-1,
    so the basis stays M-orthonormal to ~eps (reuse would leave ~eps cond(R0) = 1e-10).  The
    spectrum: two eigenvalue clusters of 300 (width 1e-6) and four single eigenvalues, so the
    invariant subspace of a random 8-column start block has 8 + 8 + 4 dimensions: the block formed
    in step 1 holds 4 O(1) directions and 4 of size ~1e-6 (R0 diagonal spread ~2e6, simulated in
    numpy).  The Ritz vectors are orthonormal to 1e-12 and the Ritz values lie in the spectrum."""
    import scipy.sparse as sp
    rng = np.random.default_rng(3)
    lam = np.sort(np.concatenate([np.repeat([1.0, 2.0], 300), [3.0, 4.0, 5.0, 6.0]]) + 1e-6 * rng.random(604))
    n = lam.size
    Kh = sp.diags(lam).tocsr()
    Mh = sp.identity(n).tocsr()
    K, M = _upload(ctx, Kh), _upload(ctx, Mh)
    bl = eigmi.BlockLanczos(K, M, block=8, max_steps=2, degree=36, seed=11)
    t = bl.step(2)
    assert t.cholqr_recomputed > 0, "the ill-conditioned block did not take the recompute path"
    ev, Y, _ = bl.ritz(4, eigmi.WHICH_LA, want_evec=True)
    assert np.all((ev > 1.0 - 1e-9) & (ev < 6.0 + 1e-5))
    G = Y @ Y.T
    assert np.max(np.abs(G - np.eye(4))) <= 1e-12
    # the Ritz values are those of the projected pencil on the returned vectors
    assert np.allclose(np.sort(np.linalg.eigvalsh(Y @ (Kh @ Y.T))), np.sort(ev), rtol=1e-10, atol=0)
    bl.close()


@pytest.mark.gpu
def test_block_lanczos_smallest_full_space(ctx):
    """Small pencil (n = 216): with the Krylov space near the whole space the SMALLEST eigenvalues
    -- the ones GeneralizedInverse returns -- are exact too."""
    import scipy.linalg as sl
    N, b, steps = 6, 8, 24
    Kh, Mh = oracle.p1_kuhn(N)
    K, M = _upload(ctx, Kh), _upload(ctx, Mh)
    bl = eigmi.BlockLanczos(K, M, block=b, max_steps=steps, degree=40, seed=7)
    bl.step(steps)
    exact = sl.eigh(Kh.toarray(), Mh.toarray(), eigvals_only=True)
    ev, _, res = bl.ritz(4, eigmi.WHICH_SA)
    assert np.max(np.abs(ev - exact[:4]) / exact[:4]) <= 1e-8
    bl.close()


@pytest.mark.gpu
def test_block_lanczos_argument_errors(ctx):
    Kh, Mh = oracle.p1_kuhn(4)
    K, M = _upload(ctx, Kh), _upload(ctx, Mh)
    with pytest.raises(eigmi.EigError):
        eigmi.BlockLanczos(K, M, block=12, max_steps=2)
    with pytest.raises(eigmi.EigShapeError):
        eigmi.BlockLanczos(K, M, block=32, max_steps=2)  # (2+1)*32 > 64 rows


def _cheb_degree(lmin, lmax, eps):
    kappa = lmax / lmin
    rho = (np.sqrt(kappa) - 1) / (np.sqrt(kappa) + 1)
    return int(np.ceil(np.log(eps / 2) / np.log(rho)))


@pytest.mark.gpu
def test_shift_invert_smallest_p1(ctx):
    """C5 at the end GeneralizedInverse returns (eigensolver.hh:204-351) -- the 4
    smallest eigenvalues of the P1 pencil at N = 24 (n = 13824) through the spectral transformation
    (K - sigma M)^-1 M, sigma = 0, inner Chebyshev-Jacobi K-solve (K = L7 / (N+1), so
    spec(D^-1 K) = [2 sin^2(pi h / 2), 2 cos^2(pi h / 2)], h = 1 / (N + 1); degree for 1e-13).
    Bar: within 1e-8 (relative) of ARPACK shift-invert (scipy eigsh sigma = 0) on the same pencil;
    residuals ||K y - lambda M y|| <= 1e-5 lambda ||M y|| (the cluster 59.81 (double), 60.15: Ritz
    vectors of a multiple eigenvalue converge as the square root of its Ritz value)."""
    import scipy.sparse.linalg as ssl
    N = 24
    K, M = oracle.p1_kuhn(N)
    h = 1.0 / (N + 1)
    lmin, lmax = 2 * np.sin(np.pi * h / 2) ** 2, 2 * np.cos(np.pi * h / 2) ** 2
    deg = _cheb_degree(lmin * 0.999, lmax * 1.001, 1e-13)
    dK, dM = _upload(ctx, K), _upload(ctx, M)
    bl = eigmi.BlockLanczos(dK, dM, block=32, max_steps=8, degree=deg, lmin=lmin * 0.999, lmax=lmax * 1.001,
                            Ks=dK, sigma=0.0)
    bl.step(8)
    ev, Y, res = bl.ritz(4, eigmi.WHICH_SA, want_evec=True)
    print('SI block Lanczos N=24:', ev, 'degree', deg)
    ref = np.sort(ssl.eigsh(K, k=4, M=M, sigma=0.0, which="LM", tol=1e-14, v0=np.ones(K.shape[0]),
                            return_eigenvectors=False))
    assert np.all(np.diff(ev) >= 0)
    assert np.max(np.abs(ev - ref) / ref) <= 1e-8, (ev, ref)
    for lam, y in zip(ev, Y):
        r = K @ y - lam * (M @ y)
        assert np.linalg.norm(r) <= 1e-5 * lam * np.linalg.norm(M @ y)  # (a double eigenvalue: vectors ~ sqrt(eps_lambda))
    bl.close()


@pytest.mark.gpu
def test_block_lanczos_variable_coefficients_box_image(ctx):
    """C5's block Lanczos (b = 32) on the variable-coefficient P1 K / M (eig_gen kinds 9 / 10: a
    coefficient per tetrahedron) at 48^3 = 110,592 rows, uploaded with EIG_MAT_NO_CLASS so the K SpMM
    and the Chebyshev mass solve run on the box-image kernels that stream the matrix values
    (k_box_mv32): the block tridiagonal's eigenvalues against the numpy restatement of the same
    recurrence (oracle.block_lanczos_gen, same start block) within 1e-9 relative."""
    import scipy.sparse as sp
    N, b, steps = 48, 32, 3
    n = N ** 3
    mats = []
    for kind in (eigmi.GEN_P1STIFF3D_VAR, eigmi.GEN_P1MASS3D_VAR):
        rp, c, v = eigmi.gen_matrix(kind, N)
        mats.append((sp.csr_matrix((v, c, rp), shape=(n, n)),
                     eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=eigmi.MAT_NO_CLASS)))
    (Kh, K), (Mh, M) = mats
    assert K.kernel("spmm32") == "k_box_mv32" and M.kernel("cheb32") == "k_box_mv32_cheb"
    bl = eigmi.BlockLanczos(K, M, block=b, max_steps=steps, degree=36, seed=123)
    bl.step(steps)
    T = bl.tmatrix()
    V0 = oracle.mv_to_cols(oracle.random_mv8(n, b, 123), n, b)
    Tref, _ = oracle.block_lanczos_gen(Kh, Mh, V0, steps)
    th, thr = np.linalg.eigvalsh(T), np.linalg.eigvalsh(Tref)
    print(f"variable-coefficient block Lanczos 48^3: max rel diff {np.max(np.abs(th - thr) / np.abs(thr)):.2e}")
    assert np.max(np.abs(th - thr) / np.abs(thr)) <= 1e-9
    bl.close()
    K.close(), M.close()
