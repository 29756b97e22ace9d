"""CPU tests: pin the oracle (oracle/oracle.cc) against the reference's known answers and the
golden fixtures, before it is trusted as the checker of the HIP path."""
import json
import os

import numpy as np
import pytest
import scipy.linalg as sla

import oracle
from fused_ref import classic, classic_spread, shifted, top_ritz


def test_generators_match_scipy_patterns():
    A = oracle.laplace2d(64)
    assert A.nnz == 20224  # SURVEY 8(a) C1 and reference_run.json
    S = A.to_scipy().toarray()
    assert np.array_equal(S, S.T)
    assert np.all(np.diag(S) == 4.0)
    P = oracle.poisson3d(8)
    assert P.nnz == 7 * 8 ** 3 - 6 * 8 ** 2
    for r in range(P.nrows):  # ISTL rows: strictly ascending columns
        c = P.col[P.rowptr[r]:P.rowptr[r + 1]]
        assert np.all(np.diff(c) > 0)


def test_c1_analytic_known_answer(golden_dir):
    """src/dune-eigensolver.cc:437-446 spectrum == ARPACK (scipy) == dense eigh."""
    g = np.load(os.path.join(golden_dir, "c1_arpack.npz"))
    ana = oracle.eig_laplace2d(64)
    assert np.allclose(g["analytic"], ana, rtol=0, atol=1e-15)
    assert np.allclose(g["la_w"], ana[::-1][:4], rtol=0, atol=1e-12)
    assert np.allclose(g["sa_w"], ana[:4], rtol=0, atol=1e-12)
    w = sla.eigvalsh(oracle.laplace2d(16).to_scipy().toarray())
    assert np.allclose(w, oracle.eig_laplace2d(16), atol=1e-12)


def test_standard_largest_matches_recorded_reference_run(golden_dir):
    """the compiled reference stopped after 50 iterations with Ritz_0 = 7.9037."""
    rec = json.load(open(os.path.join(golden_dir, "reference_run.json")))
    r = rec["StandardLargest_laplace2d_N64_nev4_seed123_tol2e-3"]
    ev, evec, it = oracle.standard_largest(oracle.laplace2d(64), 0.0, 2e-3, 4000, 4, 123)
    assert it == r["iterations"]
    assert round(ev[0], 4) == r["ritz0_rounded_4"]
    assert evec.shape == (4, 4096)


def test_standard_largest_matches_recorded_reference_run_tol_1e12(golden_dir):
    """The second recorded reference run (eigensolver.hh:75-103 at tol 1e-12):
    13,193 iterations, Ritz values within 1e-9 of the analytic largest eigenvalues (.cc:437-446).
    The restatement reproduces the count exactly (-O2 -ffp-contract=off; the survey's reference build
    was -O3 without -march, i.e. no FMA contraction either)."""
    rec = json.load(open(os.path.join(golden_dir, "reference_run.json")))
    r = rec["StandardLargest_laplace2d_N64_nev4_seed123_tol1e-12"]
    ev, _, it = oracle.standard_largest(oracle.laplace2d(64), 0.0, 1e-12, 20000, 4, 123)
    assert it == r["iterations"]
    ana = np.sort(oracle.eig_laplace2d(64))[::-1][:4]
    assert np.abs(np.asarray(ev) - ana).max() <= r["max_abs_err_vs_analytic_largest"]


@pytest.mark.parametrize("m", [8, 16, 32])
@pytest.mark.parametrize("variant", ["mgs", "cholqr", "cholqr_split"])
def test_orthonormalize_blocked(m, variant):
    n = 1000
    Q = oracle.random_mv8(n, m, 7)
    Qo = oracle.orthonormalize_mv8(Q, n, m, variant)
    X = oracle.mv_to_cols(Qo, n, m)
    assert np.abs(X.T @ X - np.eye(m)).max() < 1e-13
    # same thin QR as numpy (unique with positive diagonal R)
    q, r = np.linalg.qr(oracle.mv_to_cols(Q, n, m))
    q = q * np.sign(np.diag(r))
    assert np.abs(q - X).max() < 1e-12


def test_cholqr_split_half_order_differs():
    """orthonormalize_avx2_b8's split-half projection (kernels_avx2.hh:255-381) and _v2's single
    8x8 projection differ by rounding: measurably (~5e-9) when a later block is nearly a combination
    of the diagonal block, and both keep orthonormality to the same level."""
    n, m = 3000, 16
    rng = np.random.default_rng(1)
    X = rng.standard_normal((n, m))
    X[:, 8:] = X[:, :8] @ rng.standard_normal((8, 8)) + 1e-7 * rng.standard_normal((n, 8))
    Q = oracle.cols_to_mv(X)
    a = oracle.mv_to_cols(oracle.orthonormalize_mv8(Q, n, m, "cholqr"), n, m)
    b = oracle.mv_to_cols(oracle.orthonormalize_mv8(Q, n, m, "cholqr_split"), n, m)
    assert 1e-10 < np.abs(a - b).max() < 1e-6
    for Y in (a, b):
        assert np.abs(Y.T @ Y - np.eye(m)).max() < 1e-6


def test_orthonormalize_naive_matches_blocked_span():
    n, m = 500, 8
    Q = oracle.random_mv8(n, m, 3)
    X = oracle.mv_to_cols(Q, n, m)
    cm = np.ascontiguousarray(X.T.reshape(-1))  # MultiVector<double,1>: column after column
    on = oracle.orthonormalize_naive(cm, n, m).reshape(m, n).T
    ob = oracle.mv_to_cols(oracle.orthonormalize_mv8(Q, n, m), n, m)
    assert np.abs(on - ob).max() < 1e-12


def test_b_orthonormalize_identity_B_equals_cholqr():
    n, m = 64 * 64, 16
    B = oracle.laplace2d(64, "identity")
    Q = oracle.random_mv8(n, m, 5)
    Qb, norm = oracle.b_orthonormalize_mv8(B, Q, n, m)
    X = oracle.mv_to_cols(Qb, n, m)
    assert np.abs(X.T @ X - np.eye(m)).max() < 1e-13
    assert norm > 0


def test_b_orthonormalize_spd_B():
    n, m = 32 * 32, 16
    B = oracle.laplace2d(32)
    Q = oracle.random_mv8(n, m, 9)
    Qb, norm = oracle.b_orthonormalize_mv8(B, Q, n, m)
    X = oracle.mv_to_cols(Qb, n, m)
    Bs = B.to_scipy()
    assert np.abs(X.T @ (Bs @ X) - np.eye(m)).max() < 1e-11


def test_spmm_and_dots_against_numpy():
    A = oracle.poisson3d(10)
    n, m = A.n, 16
    Q = oracle.random_mv8(n, m, 1)
    Y = oracle.spmm_mv8(A, Q, m)
    X = oracle.mv_to_cols(Q, n, m)
    assert np.abs(oracle.mv_to_cols(Y, n, m) - A.to_scipy() @ X).max() < 1e-12
    dp = oracle.dot_diag_mv8(Q, Y, n, m)
    assert np.allclose(dp, np.einsum("ij,ij->j", X, A.to_scipy() @ X), rtol=1e-12)
    G = oracle.gram_mv8(Q, Y, n, m)
    assert np.allclose(G, X.T @ (A.to_scipy() @ X), rtol=1e-12, atol=1e-9)


def test_bcsr_mv_matches_scipy_bsr_and_kron_known_answer(golden_dir):
    g = np.load(os.path.join(golden_dir, "q1elast_6_bsr.npz"))
    A = oracle.q1elast(6)
    y = oracle.csr_mv(A, g["x"])
    assert np.abs(y - g["y_bsr"]).max() < 1e-13
    assert np.allclose(np.sort(g["eig_dense"]), g["analytic"], atol=1e-12)


def test_lanczos_oracle_ritz_values_converge(golden_dir):
    """The restated three-term recurrence reproduces ARPACK's extremal eigenvalues (C1)."""
    A = oracle.laplace2d(64)
    u0 = oracle.random_vec(A.n, 123)
    U, alpha, beta = oracle.lanczos(A, u0, 300)
    T = np.diag(alpha) + np.diag(beta[1:-1], 1) + np.diag(beta[1:-1], -1)
    w = np.linalg.eigvalsh(T)
    g = np.load(os.path.join(golden_dir, "c1_arpack.npz"))
    assert abs(w[-1] - g["la_w"][0]) < 1e-10
    assert abs(w[0] - g["sa_w"][0]) < 1e-6


@pytest.mark.parametrize("pipe", [False, True], ids=["fused", "pipelined"])
@pytest.mark.parametrize("mat", ["c1", "p3d_20"])
def test_lanczos_fused_oracle_matches_two_reduction_form(mat, pipe, golden_dir):
    """The one-reduction recurrence (orc_lanczos_fused) is the same Krylov process: alpha/beta
    agree with orc_lanczos to rounding over 40 and 100 steps (measured <= 2e-12; two runs of
    the classic form whose start vectors differ by 1e-16 differ by as much), and its Ritz values
    converge to ARPACK's (C1)."""
    A = oracle.laplace2d(64) if mat == "c1" else oracle.poisson3d(20)
    u0 = oracle.random_vec(A.n, 123)
    for k in (40, 100):
        _, a, b = oracle.lanczos(A, u0, k)
        fa, fb = oracle.lanczos_fused(A, u0, k, pipelined=pipe)
        assert np.allclose(fa, a, rtol=1e-11, atol=0) and np.allclose(fb, b, rtol=1e-11, atol=0)
    if mat == "c1":
        fa, fb = oracle.lanczos_fused(A, u0, 300, pipelined=pipe)
        T = np.diag(fa) + np.diag(fb[1:-1], 1) + np.diag(fb[1:-1], -1)
        w = np.linalg.eigvalsh(T)
        g = np.load(os.path.join(golden_dir, "c1_arpack.npz"))
        assert abs(w[-1] - g["la_w"][0]) < 1e-10


@pytest.mark.parametrize("pipe", [False, True], ids=["fused", "pipelined"])
@pytest.mark.parametrize("mat", ["p3d_16", "c1"])
@pytest.mark.parametrize("sigma", [0.0, 1e2, 1e4, 1e6, -1e6])
def test_lanczos_fused_shifted_operator(mat, sigma, pipe):
    """the fused step's predicted norm ||t||^2 - (t.u)^2/||u||^2 cancels when
    alpha >> beta (A + sigma I, eigensolver.hh:59-66, arpack_geneo_wrapper.hh:600-601): the
    unguarded form was off by 9e-2 in beta at sigma = 1e6.  The guarded step (shift by
    trace/n, repair when the prediction keeps < 1e-2 of ||t||^2) follows the classic recurrence
    over 60 steps to 1e-12 relative, or to 4x the classic recurrence's own spread where that is
    larger (sigma = +-1e6: ~6e-10 from a 1e-16 change of u0)."""
    A0 = oracle.poisson3d(16) if mat == "p3d_16" else oracle.laplace2d(64)
    A = shifted(A0, sigma)
    u0 = oracle.random_vec(A.n, 123)
    ca, cb = classic(A, u0, 60)
    fa, fb, L = oracle.lanczos_fused(A, u0, 60, with_launches=True, pipelined=pipe)
    tol = max(1e-12, 4 * classic_spread(A, u0, 60, cb))
    if abs(sigma) <= 1e4:  # the verdict's 1e-12 (the classic spread is <= 4e-13 here)
        assert np.all(np.abs(fb - cb) <= 1e-12 * np.abs(cb))
    assert np.all(np.abs(fa - ca) <= 1e-12 * np.abs(ca))
    assert np.all(np.abs(fb - cb) <= tol * np.abs(cb))
    # the shift keeps every prediction sound: 60 steps + the forced final repair
    assert L == 61


@pytest.mark.parametrize("pipe", [False, True], ids=["fused", "pipelined"])
def test_lanczos_fused_repair_path(pipe):
    """Outlier rows (diagonal + add on 12 rows) put trace/n away from the bulk of the spectrum, so
    |alpha - mu| >> beta at some steps: those launches repair (form u_k, reduce its exact norm)
    and the recurrence still follows the classic one to its own spread.  (A 12-fold outlier makes
    Lanczos without re-orthogonalisation chaotic after ~20 steps -- the classic form's own spread
    reaches O(1) -- so the long run is compared through its converged Ritz value.)"""
    A0 = oracle.poisson3d(16)
    rows = set(range(0, A0.n, A0.n // 12))
    A = shifted(A0, 0.0, rows, 1e2)
    u0 = oracle.random_vec(A.n, 123)
    ca, cb = classic(A, u0, 16)
    fa, fb, L = oracle.lanczos_fused(A, u0, 16, with_launches=True, pipelined=pipe)
    assert L > 17, "expected repair launches"
    tol = max(1e-12, 4 * classic_spread(A, u0, 16, cb))
    assert np.all(np.abs(fa - ca) <= tol * np.abs(ca))
    assert np.all(np.abs(fb - cb) <= tol * np.abs(cb))
    A = shifted(A0, 0.0, rows, 1e5)
    ca, cb = classic(A, u0, 60)
    fa, fb, L = oracle.lanczos_fused(A, u0, 60, with_launches=True, pipelined=pipe)
    assert L > 70
    assert abs(top_ritz(fa, fb) - top_ritz(ca, cb)) <= 1e-12 * top_ritz(ca, cb)


@pytest.mark.parametrize("pipe", [False, True], ids=["fused", "pipelined"])
def test_lanczos_fused_breakdown(pipe):
    """u0 = an eigenvector: u_1 = 0 exactly, the repair finds ||u_1|| = 0 and the recurrence
    halts with beta[1] = 0 (what the classic form computes)."""
    n = 64
    rp = np.arange(n + 1, dtype=np.int64)
    A = oracle.CSR(n, rp, np.arange(n, dtype=np.int32), np.arange(1.0, n + 1.0))
    u0 = np.zeros(n)
    u0[5] = 2.0
    fa, fb, L = oracle.lanczos_fused(A, u0, 4, with_launches=True, pipelined=pipe)
    assert fb[0] == 2.0 and fa[0] == 6.0 and fb[1] == 0.0
    assert L == 3  # step 0, the repair, the halted launch


def test_flop_byte_models():
    assert oracle.lib.orc_flops_orthonormalize(10, 2) == 2 * 10 + 10 + 2 * 10 + 10 + 4 * 10
    assert oracle.lib.orc_bytes_orthonormalize_blocked(100, 16, 8) > 0
