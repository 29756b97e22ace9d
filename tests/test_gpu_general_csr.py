"""GPU parity of the general (non-banded) CSR/ELL path: 3-D Poisson under a seeded
random symmetric permutation followed by reverse Cuthill-McKee (eigmi.scrambled_rcm) has the
Poisson nnz and symmetry but no constant-offset band and (mostly) no stencil slices, so eig_mv and
the Lanczos kernels take the explicit-column SELL-64 image (k_spmv_b1 / k_lanczos_*_b1) that an
unstructured DUNE matrix imported through Matrix Market would take.

Bars: eig_mv BITWISE equal to the reference row loop (oracle.csr_mv = matmul_sparse_tallskinny_naive,
kernels_cpp.hh:596-621; BCRSMatrix::mv at arpack_geneo_wrapper.hh:275) at 64^3 and at the full
256^3; the Lanczos recurrences within 1e-12 relative of the oracle restatements (only the
reductions' summation order differs)."""
import numpy as np
import pytest

import eigmi
import oracle

pytestmark = pytest.mark.gpu


def scrambled(N, seed=123):
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
    rp, c, v = eigmi.scrambled_rcm(rp, c, v, seed)
    return oracle.CSR(rp.size - 1, rp, c, v)


@pytest.fixture(scope="module")
def s64():
    return scrambled(64)


def test_general_image_selected(ctx, s64):
    M = eigmi.Matrix.from_bcsr(ctx, s64.rowptr, s64.col, s64.val)
    assert M.info.sym_offsets == 0, "scrambled matrix must not get the band image"
    assert M.info.stencil_slices < M.info.nslices // 2
    assert M.kernel("spmv") == "k_spmv_b1" and M.kernel("fused") == "k_lanczos_fused_b1"
    M.close()


def test_general_mv_bitwise_64(ctx, s64):
    M = eigmi.Matrix.from_bcsr(ctx, s64.rowptr, s64.col, s64.val)
    rng = np.random.default_rng(7)
    for x in (rng.standard_normal(s64.n), np.ones(s64.n)):
        assert np.array_equal(M.mv_host(x), oracle.csr_mv(s64, x))
    # explicit columns everywhere (no stencil slices at all): the same bits
    Me = eigmi.Matrix.from_bcsr(ctx, s64.rowptr, s64.col, s64.val, flags=eigmi.MAT_NO_STENCIL)
    assert Me.info.stencil_slices == 0
    x = rng.standard_normal(s64.n)
    assert np.array_equal(Me.mv_host(x), oracle.csr_mv(s64, x))
    M.close()
    Me.close()


@pytest.mark.parametrize("fused", [False, True], ids=["classic", "fused"])
def test_general_lanczos_64(ctx, s64, fused):
    M = eigmi.Matrix.from_bcsr(ctx, s64.rowptr, s64.col, s64.val)
    u0 = oracle.random_vec(s64.n, 123)
    a, b, _ = eigmi.lanczos_run(M, 40, seed=123, fused=fused)
    if fused:
        ra, rb = oracle.lanczos_fused(s64, u0, 40)
    else:
        _, ra, rb = oracle.lanczos(s64, u0, 40)
    assert np.allclose(a, ra, rtol=1e-12, atol=0) and np.allclose(b[:40], rb[:40], rtol=1e-12, atol=0)
    M.close()


def test_general_mv_bitwise_256(ctx):
    """Full BASELINE size (n = 16.8 M, nnz = 117 M) on the explicit-column image."""
    A = scrambled(256)
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    assert M.info.sym_offsets == 0 and M.kernel("spmv") == "k_spmv_b1"
    x = np.random.default_rng(11).standard_normal(A.n)
    assert np.array_equal(M.mv_host(x), oracle.csr_mv(A, x))
    M.close()


def test_lanczos_auto_picks_per_image(ctx, s64):
    """EIG_LANCZOS_AUTO: the fused step on every 1x1 image -- the scrambled
    matrix too, now that k_lanczos_fused_b1 no longer spills there (408 vs 634 us at 256^3, faster
    than the two-kernel step) -- and the recurrence is bitwise the explicitly requested one."""
    M = eigmi.Matrix.from_bcsr(ctx, s64.rowptr, s64.col, s64.val)
    ws = eigmi.LanczosWorkspace(M, 30, seed=123, fused="auto")
    assert ws.variant == "fused" and ws.kernel == "k_lanczos_fused_b1"
    ws.step(30)
    a, b = ws.tridiag()
    ws.close()
    ref = eigmi.LanczosWorkspace(M, 30, seed=123, fused=True)
    ref.step(30)
    ra, rb = ref.tridiag()
    ref.close()
    assert np.array_equal(a, ra) and np.array_equal(b, rb)
    M.close()
    P = oracle.poisson3d(32)
    Mp = eigmi.Matrix.from_bcsr(ctx, P.rowptr, P.col, P.val)
    ws = eigmi.LanczosWorkspace(Mp, 30, seed=123, fused="auto")
    assert ws.variant == "fused" and ws.kernel == Mp.lanczos_kernel_info(True)[0]
    assert ws.kernel_bytes == Mp.lanczos_kernel_info(True)[1]
    ws.close()
    Mp.close()


def test_stencil_image_fused_64(ctx):
    """The fused step on the SELL stencil image (3-D Poisson 64^3 without the band image: every slice a
    stencil slice, k_lanczos_fused_b1 kStencil): 60 steps within 1e-12 of the restatement
    orc_lanczos_fused (only the three sums' order differs)."""
    A = oracle.poisson3d(64)
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, flags=eigmi.MAT_NO_BAND)
    assert M.info.stencil_slices == M.info.nslices and M.kernel("fused") == "k_lanczos_fused_b1"
    a, b, _ = eigmi.lanczos_run(M, 60, seed=123, fused=True)
    M.close()
    ra, rb = oracle.lanczos_fused(A, oracle.random_vec(A.n, 123), 60)
    assert np.max(np.abs(a - ra) / np.abs(ra)) <= 1e-12
    assert np.max(np.abs(b[1:] - rb[1:]) / np.abs(rb[1:])) <= 1e-12
