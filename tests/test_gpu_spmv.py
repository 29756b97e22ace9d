"""GPU parity: SpMV (BCRSMatrix::mv / multMvB, matmul_sparse_tallskinny_naive) on the HIP
SELL-64 kernels vs the oracle.  Integer-exact order is kept, so the bar is BITWISE equality."""
import numpy as np
import pytest

import eigmi
import oracle

pytestmark = pytest.mark.gpu


def upload(ctx, A):
    return eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, A.br, A.bc)


MATS = {
    "c1_dirichlet64": lambda: oracle.laplace2d(64),
    "neumann64": lambda: oracle.laplace2d(64, "neumann"),
    "pu64": lambda: oracle.laplace2d(64, "pu", 3),
    "identity32": lambda: oracle.laplace2d(32, "identity"),
    "poisson3d_16": lambda: oracle.poisson3d(16),
    "poisson3d_33_ragged": lambda: oracle.poisson3d(33),  # n = 35937, last slice partial
    "q1elast_5": lambda: oracle.q1elast(5),
    "q1elast_8": lambda: oracle.q1elast(8),
}


@pytest.mark.parametrize("name", sorted(MATS))
def test_mv_bitwise(ctx, name):
    A = MATS[name]()
    M = upload(ctx, A)
    rng = np.random.default_rng(42)
    for x in (rng.standard_normal(A.n), np.ones(A.n), np.zeros(A.n)):
        y = M.mv_host(x)
        ref = oracle.csr_mv(A, x)
        assert np.array_equal(y, ref), f"{name}: max diff {np.abs(y - ref).max()}"


def test_bcsr_golden_fixture(ctx, golden_dir):
    import os
    g = np.load(os.path.join(golden_dir, "q1elast_6_bsr.npz"))
    A = oracle.q1elast(6)
    y = upload(ctx, A).mv_host(g["x"])
    assert np.abs(y - g["y_bsr"]).max() < 1e-13


def random_bcsr(nbr, nbc, br, bc, density, seed, empty_rows=True):
    rng = np.random.default_rng(seed)
    rowptr = [0]
    cols, vals = [], []
    for r in range(nbr):
        k = rng.binomial(nbc, density)
        if empty_rows and r % 17 == 5:
            k = 0
        c = np.sort(rng.choice(nbc, size=min(k, nbc), replace=False))
        cols.extend(c.tolist())
        vals.append(rng.standard_normal(len(c) * br * bc))
        rowptr.append(len(cols))
    vals = np.concatenate(vals) if vals else np.zeros(0)
    return oracle.CSR(nbr, np.array(rowptr, np.int64), np.array(cols, np.int32), vals, br, bc)


@pytest.mark.parametrize("br", [1, 2, 3, 4])
@pytest.mark.parametrize("bc", [1, 2, 3, 4])
def test_mv_random_blocks_bitwise(ctx, br, bc):
    nbr, nbc = 300, 257
    A = random_bcsr(nbr, nbc, br, bc, 0.03, 100 * br + bc)
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, br, bc, ncols_blocks=nbc)
    x = np.random.default_rng(1).standard_normal(nbc * bc)
    y = M.mv_host(x)
    ref = np.zeros(nbr * br)
    oracle.lib.orc_bcsr_mv(nbr, br, bc, A.rowptr, A.col, A.val, x, ref)
    assert np.array_equal(y, ref)


def test_mv_long_rows(ctx):
    """Rows longer than the 8-wide prefetch (dense-ish rows, widths 1..200)."""
    A = random_bcsr(130, 400, 1, 1, 0.5, 3)
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, 1, 1, ncols_blocks=400)
    x = np.random.default_rng(2).standard_normal(400)
    ref = np.zeros(130)
    oracle.lib.orc_bcsr_mv(130, 1, 1, A.rowptr, A.col, A.val, x, ref)
    assert np.array_equal(M.mv_host(x), ref)


def test_mv_device_pointers_and_empty(ctx):
    A = oracle.poisson3d(8)
    M = upload(ctx, A)
    x = np.random.default_rng(5).standard_normal(A.n)
    dx, dy = ctx.array(x), ctx.zeros(A.n)
    M.mv(dx, dy)
    ctx.sync()
    assert np.array_equal(dy.get(), oracle.csr_mv(A, x))
    E = eigmi.Matrix.from_bcsr(ctx, np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0), 1, 1)
    assert E.info.n == 0
    assert E.mv_host(np.zeros(0)).size == 0


def test_shift_diag_matches_reference_shift(ctx):
    A = oracle.laplace2d(40)
    M = upload(ctx, A)
    M.shift_diag(0.375)
    val = A.val.copy()
    oracle.lib.orc_shift_diag(A.n, A.rowptr, A.col, val, 0.375)
    B = oracle.CSR(A.nrows, A.rowptr, A.col, val)
    x = np.random.default_rng(0).standard_normal(A.n)
    assert np.array_equal(M.mv_host(x), oracle.csr_mv(B, x))


def test_invalid_inputs_raise(ctx):
    rp = np.array([0, 2], np.int64)
    with pytest.raises(eigmi.EigError):
        eigmi.Matrix.from_bcsr(ctx, rp, np.array([1, 0], np.int32), np.ones(2), 1, 1)  # descending
    with pytest.raises(eigmi.EigShapeError):
        eigmi.Matrix.from_bcsr(ctx, np.array([0, 1], np.int64), np.array([0], np.int32), np.ones(25), 5, 5)
    with pytest.raises(eigmi.EigShapeError):
        eigmi.Matrix.from_bcsr(ctx, rp, np.array([0, 7], np.int32), np.ones(2), 1, 1)  # column out of range
