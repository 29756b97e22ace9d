"""computeGenSymShiftInvertMinMagnitude semantics (arpack_geneo_wrapper.hh:581-658)
-- the nev eigenpairs nearest sigma ("LM" on OP = (A - sigma B)^-1 B), eigenvalues sorted ascending,
B-normalised vectors -- by the device thick-restart Lanczos (eig_shift_invert_solve) on the LU
operator of SURVEY 8(f) row 1.

Parity anchor: ARPACK itself (scipy.sparse.linalg.eigsh bundles ARPACK-NG; the reference binds it
through ARPACK++), fixtures under tests/golden/ made by make_golden.py:
  * C1 2-D Dirichlet 64^2 and 3-D Poisson 16^3, B = I, sigma = 0 (c1_arpack.npz, poisson3d_16_arpack.npz);
  * the reference harness's GenEO pencil (.cc:455-512, ini [ev]): Neumann Laplacian, partition-of-
    unity B, sigma = -1e-3, nev = 4 at N = 32, and the C5 P1 pencil at N = 8 (geneo_arpack.npz).
Tolerance: eigenvalues to 1e-10 absolute (the GenEO kernel eigenvalue is 0) / 1e-11 relative;
vectors through their residual ||A x - lambda B x|| <= 1e-8 ||A|| and B-orthonormality 1e-10
(degenerate pairs make the vectors themselves non-unique)."""
import os

import numpy as np
import pytest

import eigmi
import oracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def up(ctx, A):
    return eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)


def check_vectors(As, Bs, ev, X, tol=1e-8):
    Bs = Bs if Bs is not None else np.eye(As.shape[0])
    R = As @ X.T - (Bs @ X.T) * ev[None, :]
    assert np.abs(R).max() <= tol * np.abs(As).sum(1).max(), np.abs(R).max()
    G = X @ (Bs @ X.T)
    assert np.abs(G - np.eye(len(ev))).max() <= 1e-10


METHODS = ["single", "block"]


@pytest.mark.parametrize("method", METHODS)
def test_c1_standard_smallest(ctx, method):
    d = np.load(os.path.join(GOLD, "c1_arpack.npz"))
    A = oracle.laplace2d(64)
    ev, X, restarts = eigmi.shift_invert_solve(up(ctx, A), 4, sigma=0.0, method=method)
    assert np.allclose(ev, d["sa_w"], rtol=0, atol=1e-10)
    assert np.allclose(ev, np.sort(d["analytic"])[:4], rtol=0, atol=1e-10)
    check_vectors(A.to_scipy().toarray(), None, ev, X)


@pytest.mark.parametrize("method", METHODS)
def test_poisson3d_smallest(ctx, method):
    d = np.load(os.path.join(GOLD, "poisson3d_16_arpack.npz"))
    A = oracle.poisson3d(16)
    ev, _, _ = eigmi.shift_invert_solve(up(ctx, A), 4, sigma=0.0, want_evec=False, method=method)
    assert np.allclose(ev, d["sa_w"], rtol=1e-11, atol=0)


@pytest.mark.parametrize("method", METHODS)
def test_geneo_pencil(ctx, method):
    """The reference harness's ARPACK experiment, src/dune-eigensolver.cc:508-512."""
    d = np.load(os.path.join(GOLD, "geneo_arpack.npz"))
    N, shift = int(d["geneo_N"]), float(d["geneo_shift"])
    A, B = oracle.laplace2d(N, "neumann"), oracle.laplace2d(N, "pu", overlap=3)
    ev, X, _ = eigmi.shift_invert_solve(up(ctx, A), 4, sigma=-shift, B=up(ctx, B), method=method)
    assert np.allclose(ev, d["geneo_w"], rtol=0, atol=1e-10)
    check_vectors(A.to_scipy().toarray(), B.to_scipy().toarray(), ev, X)


@pytest.mark.parametrize("method", METHODS)
def test_p1_pencil(ctx, method):
    d = np.load(os.path.join(GOLD, "geneo_arpack.npz"))
    K, M = oracle.p1_kuhn(int(d["p1_N"]))
    dK = eigmi.Matrix.from_bcsr(ctx, K.indptr.astype(np.int64), K.indices.astype(np.int32), K.data)
    dM = eigmi.Matrix.from_bcsr(ctx, M.indptr.astype(np.int64), M.indices.astype(np.int32), M.data)
    ev, X, _ = eigmi.shift_invert_solve(dK, 6, sigma=0.0, B=dM, method=method)
    assert np.allclose(ev, d["p1_w"], rtol=1e-11, atol=0)
    check_vectors(K.toarray(), M.toarray(), ev, X)


@pytest.mark.parametrize("method", METHODS)
def test_given_factors_and_interior_shift(ctx, method):
    """Factors passed in (of A - sigma I, like the wrapper's ashiftb, :599-604) give the same
    answer; a shift inside the spectrum selects the eigenvalues nearest sigma."""
    A = oracle.laplace2d(24)
    exact = np.sort(oracle.eig_laplace2d(24))
    sigma = 0.5 * (exact[30] + exact[31]) + 1e-3
    As = oracle.CSR(A.nrows, A.rowptr, A.col, A.val.copy())
    oracle.lib.orc_shift_diag(As.n, As.rowptr, As.col, As.val, -sigma)
    d = eigmi.LU.from_bcsr(None, As.rowptr, As.col, As.val).export()
    d = {k: v for k, v in d.items()}
    lu = eigmi.LU.from_factors(ctx, **d)
    dA = up(ctx, A)
    ev1, _, _ = eigmi.shift_invert_solve(dA, 6, sigma=sigma, lu=lu, want_evec=False, method=method)
    ev2, X, _ = eigmi.shift_invert_solve(dA, 6, sigma=sigma, method=method)
    nearest = np.sort(exact[np.argsort(np.abs(exact - sigma))[:6]])
    assert np.allclose(ev1, nearest, rtol=0, atol=1e-10) and np.allclose(ev2, nearest, rtol=0, atol=1e-10)
    check_vectors(A.to_scipy().toarray(), None, ev2, X)  # (negative theta: eigenvalues below sigma)


def test_block_method_arguments(ctx):
    """EIG_SI_BLOCK needs its basis (cmax + p columns) inside n; both method flags at once is an error."""
    A = oracle.laplace2d(6)
    with pytest.raises(eigmi.EigError):
        eigmi.shift_invert_solve(up(ctx, A), 4, sigma=0.0, method="block")  # n = 36 < 72 columns
    ev, _, _ = eigmi.shift_invert_solve(up(ctx, A), 4, sigma=0.0, want_evec=False)  # auto: one-vector
    assert np.allclose(ev, np.sort(oracle.eig_laplace2d(6))[:4], rtol=0, atol=1e-10)
    with pytest.raises(eigmi.EigError):  # nev = 264: the CholQR Gram (264 x 264) exceeds the tickets
        eigmi.shift_invert_solve(up(ctx, oracle.laplace2d(64)), 264, sigma=0.0, method="block")
    with pytest.raises(eigmi.EigError):
        A2 = up(ctx, A)
        A2.ctx.check(eigmi.lib.eig_shift_invert_solve_ex(A2.h, None, None, 0.0, 4, 0, 0.0, 0, 1,
                                                         eigmi._np_ptr(np.zeros(4)), None, None, 3))


@pytest.mark.parametrize("method,nev", [("auto", 60), ("block", 100)])
def test_large_nev_block(ctx, method, nev):
    """Large nev on the block method, with its Grams' partials in a buffer sized for the launch:
    nev = 60 (p = 64, a 384-column basis; EIG_SI_AUTO takes the block method) and nev = 100 (p = 104,
    624 columns: the projection Gram goes in row slices).  Eigenvalues against the analytic
    spectrum, vectors through their residual and orthonormality."""
    A = oracle.laplace2d(64)
    ev, X, _ = eigmi.shift_invert_solve(up(ctx, A), nev, sigma=0.0, method=method)
    assert np.allclose(ev, np.sort(oracle.eig_laplace2d(64))[:nev], rtol=0, atol=1e-10)
    As = A.to_scipy()
    R = (As @ X.T) - X.T * ev[None, :]
    assert np.abs(R).max() <= 1e-8 * 8.0
    assert np.abs(X @ X.T - np.eye(nev)).max() <= 1e-10


def test_argument_errors(ctx):
    A = oracle.laplace2d(4)
    with pytest.raises(eigmi.EigError):
        eigmi.shift_invert_solve(up(ctx, A), 16, sigma=0.0)  # nev >= n
    with pytest.raises(eigmi.EigShapeError):
        B = oracle.laplace2d(5, "identity")
        eigmi.shift_invert_solve(up(ctx, A), 2, sigma=0.1, B=up(ctx, B))  # sizes differ


@pytest.mark.gpu
def test_adaptive_threshold_vs_arpack(ctx, golden_dir):
    """computeGenSymShiftInvertMinMagnitudeAdaptive (arpack_geneo_wrapper.hh:661-774) on the harness
    pencil (Neumann A, PU-masked B, sigma = -1e-3) against ARPACK's 40 eigenvalues nearest sigma
    (tests/golden/geneo_adaptive_arpack.npz): nev grows 4 -> 5 -> 6 -> 7 -> 9 -> 11 -> 14 (x1.3) and
    stops when the largest returned eigenvalue reaches the threshold; every returned eigenvalue
    within 1e-10 of ARPACK's."""
    import os
    g = np.load(os.path.join(golden_dir, "geneo_adaptive_arpack.npz"))
    N, shift, w, thr = int(g["N"]), float(g["shift"]), g["w"], float(g["threshold"])
    i0, mx = int(g["initial_nev"]), int(g["max_nev"])
    # the reference loop replayed on ARPACK's eigenvalues
    nev, passes = i0, 1
    while w[nev - 1] < thr and nev < mx:
        nev = min(mx, int(nev * 1.3))
        passes += 1
    assert (nev, passes) == (14, 7)
    An, Bp = oracle.laplace2d(N, "neumann"), oracle.laplace2d(N, "pu", overlap=3)
    dA = eigmi.Matrix.from_bcsr(ctx, An.rowptr, An.col, An.val)
    dB = eigmi.Matrix.from_bcsr(ctx, Bp.rowptr, Bp.col, Bp.val)
    ev, X, p = eigmi.shift_invert_adaptive(dA, thr, i0, mx, sigma=-shift, B=dB)
    assert len(ev) == nev and p == passes
    assert ev[-1] >= thr and np.all(ev[:-1] <= ev[1:])
    assert np.max(np.abs(ev - w[:nev])) < 1e-10
    check_vectors(An.to_scipy().toarray(), Bp.to_scipy().toarray(), ev, X)
    # max_nev caps the growth; initial_nev > max_nev is the reference's "initial_nev too large"
    ev2, _, p2 = eigmi.shift_invert_adaptive(dA, 10.0, 4, 6, sigma=-shift, B=dB, want_evec=False)
    assert len(ev2) == 6 and p2 == 3 and np.max(np.abs(ev2 - w[:6])) < 1e-10
    with pytest.raises(eigmi.EigError):
        eigmi.shift_invert_adaptive(dA, 1.0, 8, 4, sigma=-shift, B=dB)
