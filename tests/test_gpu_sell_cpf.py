"""Explicit-column SELL slices with the cross-slice column prefetch (EIG_TUNE_SELL_CPF, the default;
k_lanczos_fused_b1<1, MODE, true> and k_spmv_b1<1, MODE, true>): the next slice's column indices load
while this slice's gathers fly, the products and their order stay rows_dot's -- so eig_mv must be
BITWISE the reference row loop (oracle.csr_mv) with and without it, and the fused step's alpha / beta
bitwise those of the plain kernel, on a scrambled + RCM Poisson matrix (every slice explicit or mixed)
and on ragged rows wider than one 8-entry round (the later rounds' path)."""
import numpy as np
import pytest

import eigmi
import oracle

pytestmark = pytest.mark.gpu


def _ragged(n=3000, seed=7):
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    S = sp.random(n, n, density=0.006, random_state=rng, format="csr")
    S = (S + S.T + sp.diags(rng.uniform(20, 30, n))).tocsr()
    S.sort_indices()
    return S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data.copy()


def _mats():
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, 24)
    yield "poisson24_rcm", eigmi.scrambled_rcm(rp, c, v, 5)
    yield "ragged3000", _ragged()
    # a MIXED image (stencil slices beside explicit ones, whose stencil width reads -1): the
    # per-slice choice and the prefetch across a stencil slice
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, 48)
    yield "poisson48_rcm_mixed", eigmi.scrambled_rcm(rp, c, v, 123)


def _run(ctx, mat, cpf, steps=30):
    M = eigmi.Matrix.from_bcsr(ctx, *mat, flags=eigmi.MAT_NO_BAND)
    info = M.info
    print(f"  image: {info.stencil_slices} of {info.nslices} slices stencil")
    M.tune(sell_cpf=cpf)
    ws = eigmi.LanczosWorkspace(M, steps + 2, seed=9, fused=True)
    try:
        ws.step(steps)
        a, b = ws.tridiag()
        kern = M.kernel("fused")
    finally:
        ws.close()
        M.close()
    return a, b, kern


@pytest.mark.parametrize("name,mat", list(_mats()), ids=[m[0] for m in _mats()])
def test_sell_column_prefetch_bitwise(ctx, name, mat):
    a0, b0, k0 = _run(ctx, mat, 0)
    a1, b1, k1 = _run(ctx, mat, 1)
    a2, b2, _ = _run(ctx, mat, 2)  # the automatic setting (the fused step takes the prefetch)
    assert np.array_equal(a1, a2) and np.array_equal(b1, b2)
    if name.endswith("mixed"):
        M = eigmi.Matrix.from_bcsr(ctx, *mat, flags=eigmi.MAT_NO_BAND)
        assert 0 < M.info.stencil_slices < M.info.nslices
        M.close()
    print(f"{name}: kernel {k1}, {a0.size} steps")
    assert np.array_equal(a0, a1) and np.array_equal(b0, b1)
    # and the recurrence is the restatement's (tolerance: the sums' order differs; the first 12 steps,
    # before the unreorthogonalised recurrence's rounding growth on the ragged matrix's cluster)
    rp, c, v = mat
    A = oracle.CSR(rp.size - 1, rp, c, v)
    ra, rb = oracle.lanczos_fused(A, oracle.random_vec(A.n, 9), a0.size)
    assert np.allclose(a1[:12], ra[:12], rtol=1e-10, atol=0) and np.allclose(b1[:12], rb[:12], rtol=1e-10, atol=0)


@pytest.mark.parametrize("name,mat", list(_mats()), ids=[m[0] for m in _mats()])
def test_sell_column_prefetch_mv_bitwise(ctx, name, mat):
    rp, c, v = mat
    A = oracle.CSR(rp.size - 1, rp, c, v)
    xh = np.random.default_rng(3).standard_normal(A.n)
    ref = oracle.csr_mv(A, xh)
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=eigmi.MAT_NO_BAND)
    x, y = ctx.array(xh), ctx.zeros(A.n)
    try:
        for cpf in (0, 1, 2):
            M.tune(sell_cpf=cpf)
            M.mv(x, y)
            assert np.array_equal(y.get(), ref), cpf
    finally:
        M.close()
