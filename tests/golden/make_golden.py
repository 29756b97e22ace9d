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
    reference_run()
    print("golden fixtures written to", HERE)
