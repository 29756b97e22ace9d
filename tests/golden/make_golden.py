"""Generate the golden fixtures under tests/golden/ (run in the build container; the outputs are
committed, this script is kept for provenance).

What pins what (DESIGN.md "Oracle"):
  * analytic spectrum of the 2-D Dirichlet 5-point Laplacian -- the reference's own known answer,
    src/dune-eigensolver.cc:437-446 (stored for N = 64, config C1);
  * ARPACK eigenpairs through scipy.sparse.linalg.eigsh (scipy 1.15.3 bundles ARPACK-NG) -- the
    reference's Krylov driver dependency (arpack_geneo_wrapper.hh:621-632), not vendored in the
    reference; C1 largest (LA) and smallest via shift-invert sigma = 0 "LM" exactly as
    computeGenSymShiftInvertMinMagnitude calls it with B = I (arpack_geneo_wrapper.hh:581-658);
  * the reference's StandardLargest run recorded in SURVEY.md section 6 / BASELINE.md section 2
    (compiled reference headers, this container): iterations and Ritz_0 at ini tol 2e-3;
  * 3x3-block BCRSMatrix::mv (no reference test exists): scipy bsr_matrix product and the
    Kronecker known answer lambda(L_Q1) * mu(C) of the C3 generator.
Matrices are rebuilt from the oracle generators (which follow dune-istl setupLaplacian).
"""
import json
import os
import sys

import numpy as np
import scipy
import scipy.linalg as sla
import scipy.sparse.linalg as ssl

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402


def c1():
    A = oracle.laplace2d(64).to_scipy()
    la_w, la_v = ssl.eigsh(A, k=4, which="LA", tol=1e-14, v0=np.ones(A.shape[0]))
    sa_w, sa_v = ssl.eigsh(A, k=4, sigma=0.0, which="LM", tol=1e-14, v0=np.ones(A.shape[0]))
    o = np.argsort(la_w)[::-1]
    la_w, la_v = la_w[o], la_v[:, o]
    o = np.argsort(sa_w)
    sa_w, sa_v = sa_w[o], sa_v[:, o]
    np.savez_compressed(os.path.join(HERE, "c1_arpack.npz"), la_w=la_w, la_v=la_v, sa_w=sa_w, sa_v=sa_v,
                        analytic=oracle.eig_laplace2d(64))


def poisson3d():
    N = 16
    A = oracle.poisson3d(N).to_scipy()
    la_w = ssl.eigsh(A, k=4, which="LA", tol=1e-14, v0=np.ones(A.shape[0]), return_eigenvectors=False)
    sa_w = ssl.eigsh(A, k=4, sigma=0.0, which="LM", tol=1e-14, v0=np.ones(A.shape[0]), return_eigenvectors=False)
    h = np.pi / (N + 1)
    s = 4 * np.sin(np.arange(1, N + 1) * h / 2) ** 2
    ana = np.sort((s[:, None, None] + s[None, :, None] + s[None, None, :]).ravel())
    np.savez_compressed(os.path.join(HERE, "poisson3d_16_arpack.npz"), la_w=np.sort(la_w)[::-1], sa_w=np.sort(sa_w),
                        analytic=ana)


def q1elast():
    N = 6
    A = oracle.q1elast(N)
    S = A.to_scipy()
    rng = np.random.default_rng(123)
    x = rng.standard_normal(S.shape[0])
    y = S @ x
    w = sla.eigvalsh(S.toarray())
    th = np.arange(1, N + 1) * np.pi / (N + 1)
    k1 = 2 - 2 * np.cos(th)
    m1 = (4 + 2 * np.cos(th)) / 6
    lam = (k1[:, None, None] * m1[None, :, None] * m1[None, None, :] + m1[:, None, None] * k1[None, :, None] *
           m1[None, None, :] + m1[:, None, None] * m1[None, :, None] * k1[None, None, :]).ravel()
    mu = np.array([2 - np.sqrt(2), 2.0, 2 + np.sqrt(2)])
    ana = np.sort((lam[:, None] * mu[None, :]).ravel())
    np.savez_compressed(os.path.join(HERE, "q1elast_6_bsr.npz"), x=x, y_bsr=y, eig_dense=w, analytic=ana)


def geneo():
    """The reference harness's generalised experiment (src/dune-eigensolver.cc:455-512, ini [ev]):
    Neumann Laplacian A, partition-of-unity-masked B (overlap 3), ARPACK shift-invert with
    sigma = -shift = -1e-3 ("LM", computeGenSymShiftInvertMinMagnitude, arpack_geneo_wrapper.hh:
    581-658), nev = 4 at N = 32; plus the C5 P1 pencil (K, M) at N = 8, sigma = 0, nev = 6."""
    N, shift = 32, 1e-3
    A = oracle.laplace2d(N, "neumann").to_scipy()
    B = oracle.laplace2d(N, "pu", overlap=3).to_scipy()
    w, v = ssl.eigsh(A, k=4, M=B, sigma=-shift, which="LM", tol=1e-14, v0=np.ones(A.shape[0]))
    o = np.argsort(w)
    K, M = oracle.p1_kuhn(8)
    pw = ssl.eigsh(K, k=6, M=M, sigma=0.0, which="LM", tol=1e-14, v0=np.ones(K.shape[0]),
                   return_eigenvectors=False)
    np.savez_compressed(os.path.join(HERE, "geneo_arpack.npz"), geneo_N=N, geneo_shift=shift, geneo_w=w[o],
                        geneo_v=v[:, o], p1_N=8, p1_w=np.sort(pw))


def geneo_adaptive():
    """computeGenSymShiftInvertMinMagnitudeAdaptive (arpack_geneo_wrapper.hh:661-774) on the harness
    pencil at N = 32: the 40 eigenvalues nearest sigma = -1e-3 from ARPACK (eigsh "LM", tol 1e-14),
    ascending, and a threshold halfway between the 11th and 12th (distinct values; the 10th and 11th are
    a double eigenvalue), so that nev = 4 grows 4 -> 5 -> 6 -> 7 -> 9 -> 11 -> 14 (x1.3, int) and stops
    at 14 with ev[13] >= threshold."""
    N, shift = 32, 1e-3
    A = oracle.laplace2d(N, "neumann").to_scipy()
    B = oracle.laplace2d(N, "pu", overlap=3).to_scipy()
    w = np.sort(ssl.eigsh(A, k=40, M=B, sigma=-shift, which="LM", tol=1e-14, v0=np.ones(A.shape[0]),
                          return_eigenvectors=False))
    thr = 0.5 * (w[10] + w[11])
    np.savez_compressed(os.path.join(HERE, "geneo_adaptive_arpack.npz"), N=N, shift=shift, w=w, threshold=thr,
                        initial_nev=4, max_nev=40)


def convdiff(N, pe=40.0):
    """Non-symmetric test operator (no reference fixture exists for the non-symmetric modes): 2-D
    Dirichlet 5-point Laplacian on an N x N grid plus a rotating convection field b = pe (-(y - 1/2),
    x - 1/2), central differences -- complex eigenvalue pairs near the bottom of the spectrum.  And
    an SPD B on the same 5-point pattern (the reference's A - sigma B needs pattern(B) within
    pattern(A), arpack_geneo_wrapper.hh:599-600): (M1 kron I + I kron M1) / 2, M1 = tridiag(1, 4, 1) / 6."""
    import scipy.sparse as sp
    h = 1.0 / (N + 1)
    L1 = sp.diags([-np.ones(N - 1), 2 * np.ones(N), -np.ones(N - 1)], [-1, 0, 1])
    D1 = sp.diags([-np.ones(N - 1), np.ones(N - 1)], [-1, 1]) * (0.5 * h)  # h^2 * d/dx (central)
    I = sp.identity(N)
    xs = (np.arange(N) + 1) * h
    X, Y = np.meshgrid(xs, xs, indexing="xy")  # row index = y, column = x: unknown = y * N + x
    bx, by = -pe * (Y - 0.5).ravel(), pe * (X - 0.5).ravel()
    A = sp.kron(I, L1) + sp.kron(L1, I) + sp.diags(bx) @ sp.kron(I, D1) + sp.diags(by) @ sp.kron(D1, I)
    M1 = sp.diags([np.ones(N - 1), 4 * np.ones(N), np.ones(N - 1)], [-1, 0, 1]) / 6.0
    B = (sp.kron(M1, I) + sp.kron(I, M1)) * 0.5
    A, B = A.tocsr(), B.tocsr()
    A.sort_indices()
    B.sort_indices()
    return A, B


def nonsym():
    """ARPACK's non-symmetric driver (scipy eigs = dnaupd/dneupd, real shift-invert mode 3,
    "LM") for the non-symmetric modes computeStdNonSymMinMagnitude / computeGenNonSymShiftInvert-
    MinMagnitude (arpack_geneo_wrapper.hh:428-578): the rotating convection-diffusion operator at
    N = 24 (n = 576) standard (sigma = 0, nev = 6) and against the SPD B (sigma = 0.1, nev = 6), and
    the harness GenEO pencil (symmetric, real spectrum) through eigs at sigma = -1e-3, nev = 4."""
    N = 24
    A, B = convdiff(N)
    w_std = ssl.eigs(A, k=6, sigma=0.0, which="LM", tol=1e-14, v0=np.ones(A.shape[0]), return_eigenvectors=False)
    w_gen = ssl.eigs(A, k=6, M=B, sigma=0.1, which="LM", tol=1e-14, v0=np.ones(A.shape[0]),
                     return_eigenvectors=False)
    Ng, shift = 32, 1e-3
    Ag = oracle.laplace2d(Ng, "neumann").to_scipy()
    Bg = oracle.laplace2d(Ng, "pu", overlap=3).to_scipy()
    w_geneo = ssl.eigs(Ag, k=4, M=Bg, sigma=-shift, which="LM", tol=1e-14, v0=np.ones(Ag.shape[0]),
                       return_eigenvectors=False)
    srt = lambda w: w[np.lexsort((w.imag, w.real))]  # noqa: E731
    np.savez_compressed(os.path.join(HERE, "nonsym_arpack.npz"), N=N, A_indptr=A.indptr, A_indices=A.indices,
                        A_data=A.data, B_indptr=B.indptr, B_indices=B.indices, B_data=B.data,
                        w_std=srt(w_std), w_gen=srt(w_gen), sigma_gen=0.1, geneo_N=Ng, geneo_shift=shift,
                        w_geneo=srt(w_geneo))


def reference_run():
    rec = {
        "source": "SURVEY.md section 6 / BASELINE.md section 2: reference headers multivector.hh + kernels_cpp.hh + "
                  "eigensolver.hh::StandardLargest compiled g++ 11.4 -O3 in the survey container",
        "StandardLargest_laplace2d_N64_nev4_seed123_tol2e-3": {"iterations": 50, "ritz0_rounded_4": 7.9037,
                                                                "exact_largest": 7.9953},
        "StandardLargest_laplace2d_N64_nev4_seed123_tol1e-12": {"iterations": 13193,
                                                                 "max_abs_err_vs_analytic_largest": 1e-9},
        "laplace2d_N64_nnz": 20224,
        "poisson3d_N128_nnz": 14581760,
        "scipy_version": scipy.__version__,
    }
    with open(os.path.join(HERE, "reference_run.json"), "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    c1()
    poisson3d()
    q1elast()
    geneo()
    geneo_adaptive()
    nonsym()
    reference_run()
    print("golden fixtures written to", HERE)
