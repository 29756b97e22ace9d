"""GPU parity of the guarded fused Lanczos step (k_spmv.hip fused_begin) on shifted
and ill-scaled operators -- VERDICT r1 "do this" #1 / ADVICE medium: the unguarded one-reduction
prediction ||t||^2 - (t.u)^2/||u||^2 lost 9e-2 of beta at A + 1e6 I.

Bar: the GPU's fused alpha/beta follow the classic two-reduction recurrence (orc_lanczos_rotating,
the reference CPU path's Lanczos step) to 1e-12 relative for |sigma| <= 1e4, and to 4x the classic
recurrence's own run-to-run spread beyond that (two classic runs whose start vectors differ by
1e-16 already differ by ~6e-10 at sigma = 1e6 after 60 steps; tests/fused_ref.py); alpha to 1e-12
relative throughout.  Both the plane-march kernel (band image) and the SELL row kernel run the
guard; repairs and the halted (breakdown) state are exercised.  The pipelined step
(EIG_LANCZOS_PIPELINED: SpMV on t_{k-1}, A u_k by the z recurrence; k_lanczos_pipe) runs the same
guard and is held to the same bars against the classic recurrence and its own restatement
(orc_lanczos_pipelined)."""

import numpy as np
import pytest

import eigmi
import oracle
from fused_ref import classic, classic_spread, shifted, top_ritz

pytestmark = pytest.mark.gpu


def upload(ctx, A, band=True):
    return eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, A.br, A.bc, flags=0 if band else eigmi.MAT_NO_BAND)


def fused_run(M, steps, batches=1, graph=False, pipe=False):
    ws = eigmi.LanczosWorkspace(M, steps, seed=123, fused=not pipe, pipelined=pipe)
    try:
        per = steps // batches
        done = 0
        while done < steps:
            k = min(per, steps - done)
            if graph:
                ws.capture(k)
                ws.replay()
            else:
                ws.step(k)
            done += k
        a, b = ws.tridiag()
        return a, b, ws.info()[1]
    finally:
        ws.close()


KERNEL = {True: "k_lanczos_fused_march", False: "k_lanczos_fused_b1"}


PIPE = pytest.mark.parametrize("pipe", [False, True], ids=["fused", "pipelined"])


@PIPE
@pytest.mark.parametrize("band", [True, False], ids=["march", "sell"])
@pytest.mark.parametrize("mat", ["p3d_16", "c1"])
@pytest.mark.parametrize("sigma", [1e2, 1e4, 1e6, -1e6])
def test_fused_shifted_operator_vs_classic(ctx, band, mat, sigma, pipe):
    A = shifted(oracle.poisson3d(16) if mat == "p3d_16" else oracle.laplace2d(64), sigma)
    M = upload(ctx, A, band)
    assert M.lanczos_kernel_info(True)[0] == KERNEL[band]
    a, b, L = fused_run(M, 60, pipe=pipe)
    u0 = oracle.random_vec(A.n, 123)
    ca, cb = classic(A, u0, 60)
    oa, ob, oL = oracle.lanczos_fused(A, u0, 60, with_launches=True, pipelined=pipe)
    assert L == oL == 61  # 60 steps + the forced final repair (no prediction failed)
    tol = max(1e-12, 4 * classic_spread(A, u0, 60, cb))
    assert np.all(np.abs(a - ca) <= 1e-12 * np.abs(ca))
    assert np.all(np.abs(b - cb) <= tol * np.abs(cb))
    assert np.all(np.abs(b - ob) <= tol * np.abs(ob))
    if abs(sigma) <= 1e4:
        assert np.all(np.abs(b - cb) <= 1e-12 * np.abs(cb))


@PIPE
@pytest.mark.parametrize("band", [True, False], ids=["march", "sell"])
def test_fused_repair_launches(ctx, band, pipe):
    """Outliers (+100 on 12 diagonal entries) make some predictions unsound: those launches
    repair, the step after each runs with c = 0 and the exact norm.  Same decisions and values as
    the oracle restatement; in batches (top-up launches after each batch) and as replayed graphs
    bitwise the one-batch run."""
    A0 = oracle.poisson3d(16)
    A = shifted(A0, 0.0, range(0, A0.n, A0.n // 12), 1e2)
    M = upload(ctx, A, band)
    a, b, L = fused_run(M, 16, pipe=pipe)
    u0 = oracle.random_vec(A.n, 123)
    ca, cb = classic(A, u0, 16)
    oa, ob, oL = oracle.lanczos_fused(A, u0, 16, with_launches=True, pipelined=pipe)
    assert L == oL and L > 17
    tol = max(1e-12, 4 * classic_spread(A, u0, 16, cb))
    assert np.all(np.abs(a - ca) <= tol * np.abs(ca)) and np.all(np.abs(b - cb) <= tol * np.abs(cb))
    assert np.all(np.abs(a - oa) <= tol * np.abs(oa)) and np.all(np.abs(b - ob) <= tol * np.abs(ob))
    for batches, graph in ((4, False), (3, True)):
        a2, b2, L2 = fused_run(M, 16, batches, graph, pipe)
        assert np.array_equal(a2, a) and np.array_equal(b2, b)
    # long run with large outliers: chaotic without re-orthogonalisation, compared through the
    # converged top Ritz value
    A = shifted(A0, 0.0, range(0, A0.n, A0.n // 12), 1e5)
    M = upload(ctx, A, band)
    a, b, L = fused_run(M, 60, pipe=pipe)
    ca, cb = classic(A, u0, 60)
    assert L > 70
    assert abs(top_ritz(a, b) - top_ritz(ca, cb)) <= 1e-12 * top_ritz(ca, cb)


@PIPE
def test_fused_breakdown_halts(ctx, pipe):
    """u0 an eigenvector of a diagonal matrix: u_1 = 0 exactly; the repair launch reduces
    ||u_1|| = 0, the recurrence halts (EIG_ERR_BREAKDOWN) with beta[1] = 0, alpha[0] exact."""
    n = 256
    rp = np.arange(n + 1, dtype=np.int64)
    M = eigmi.Matrix.from_bcsr(ctx, rp, np.arange(n, dtype=np.int32), np.arange(1.0, n + 1.0))
    u0 = eigmi.DeviceArray(ctx, n)
    e = np.zeros(n)
    e[5] = 2.0
    u0.upload(e)
    ws = eigmi.LanczosWorkspace(M, 8, u0=u0, fused=not pipe, pipelined=pipe)
    with pytest.raises(eigmi.EigError) as ei:
        ws.step(8)
    assert ei.value.code == 5  # EIG_ERR_BREAKDOWN
    a, b = ws.tridiag()
    assert len(a) == 1 and a[0] == 6.0 and b[0] == 2.0 and b[1] == 0.0
    ws.close()


def _extreme_ritz(alpha, beta, k=3):
    from scipy.linalg import eigh_tridiagonal
    w = eigh_tridiagonal(alpha, beta[1:len(alpha)], eigvals_only=True)
    return np.concatenate([w[:k], w[-k:]])


@pytest.mark.parametrize("kind,steps", [("laplace2d_64", 700), ("poisson3d_256", 500)])
def test_long_run_no_drift(ctx, kind, steps):
    """ADVICE r2 (k_spmv.hip k_lanczos_pipe): the pipelined step rebuilds A u_k from z_k = S - c z_{k-1}
    and only an occasional repair resets it, so a long run could drift where the 60-step tests do
    not look.  Past loss of orthogonality alpha / beta of any two recurrences part ways (ghost
    copies), so the check is on what Lanczos delivers: the extreme Ritz values of T_k after several
    hundred steps, fused and pipelined against the classic two-kernel recurrence and against the
    analytic extreme eigenvalues, to 1e-10 relative."""
    ana = None
    if kind == "laplace2d_64":
        A = oracle.laplace2d(64)
        ana = np.sort(oracle.eig_laplace2d(64))  # (the extremes converge within 700 steps at n = 4096)
    else:
        # 256^3: 500 steps leave the extreme Ritz values unconverged (relative gap ~4e-5), so the
        # check is the agreement of the three recurrences only
        A = oracle.CSR(256 ** 3, *eigmi.gen_matrix(eigmi.GEN_POISSON3D, 256))
    M = upload(ctx, A)
    ref = _extreme_ritz(*eigmi.lanczos_run(M, steps, seed=123)[:2])
    scale = np.abs(ref).max()
    for pipe in (False, True):
        a, b, _ = fused_run(M, steps, batches=5, pipe=pipe)
        got = _extreme_ritz(a, b)
        print(kind, "pipelined" if pipe else "fused", "max |ritz - classic| / scale =", np.abs(got - ref).max() / scale)
        assert np.abs(got - ref).max() <= 1e-10 * scale, (pipe, got, ref)
    if ana is not None:
        assert abs(ref[0] - ana[0]) <= 1e-10 * scale and abs(ref[-1] - ana[-1]) <= 1e-10 * scale, (ref, ana[[0, -1]])
    M.close()
