"""The value-streaming plane march (k_spmv.hip march_rows_geo2<VAL>, march variants 10 / 11): the
BCRSMatrix::mv / Lanczos step kernels on a geometric 7-point (or 5-point) band whose values are NOT
constant, so every stored value is read from the symmetric band arrays in HBM on every launch
(the reference reads every stored value per call: kernels_cpp.hh:611-617, arpack_geneo_wrapper.hh:275).

Bar: eig_mv BITWISE the reference row loop (oracle.csr_mv = matmul_sparse_tallskinny_naive,
kernels_cpp.hh:596-621); the classic and fused Lanczos alpha / beta BITWISE equal to the plain
masked march (variant 0: same rows per wave, same reduction order) at every plane-run count, and
within 1e-12 (relative) of the oracle's restated recurrences.  The matrices: eig_gen kind 8 (a hashed
conductance per grid edge), 7-point Poisson with EIG_MAT_NO_UNIFORM, and random symmetric boxes."""
import numpy as np
import pytest

import eigmi
import oracle


def varcoef(N):
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_VARCOEF3D, N)
    return oracle.CSR(N ** 3, rp, c, v)


def test_varcoef_generator_properties():
    """kind 8: the 7-point pattern of kind 4, bitwise symmetric, off-diagonals in (-1.5, -0.5],
    diagonally dominant rows (strictly on the Dirichlet faces), no two grid edges alike."""
    N = 12
    A = varcoef(N)
    P = oracle.poisson3d(N)
    assert np.array_equal(A.rowptr, P.rowptr) and np.array_equal(A.col, P.col)
    import scipy.sparse as sp
    S = sp.csr_matrix((A.val, A.col, A.rowptr), shape=(A.n, A.n))
    assert (S != S.T).nnz == 0
    r = np.repeat(np.arange(A.n), np.diff(A.rowptr))
    off = A.val[A.col != r]
    assert off.max() <= -0.5 and off.min() > -1.5
    assert len(np.unique(off)) > 0.45 * off.size  # each grid edge its own value (stored twice)
    d = A.val[A.col == r]
    rowabs = np.bincount(r, weights=np.abs(A.val)) - d
    assert np.all(d >= rowabs * (1 - 1e-15)) and np.count_nonzero(d > rowabs + 0.4) == N ** 3 - (N - 2) ** 3
    # the distributed generator produces the same rows
    rp2, c2, v2 = eigmi.gen_rows(eigmi.GEN_VARCOEF3D, N, 5 * N * N, 3 * N * N)
    lo, hi = A.rowptr[5 * N * N], A.rowptr[8 * N * N]
    assert np.array_equal(v2, A.val[lo:hi]) and np.array_equal(c2, A.col[lo:hi])


@pytest.mark.parametrize("kind,base", [(eigmi.GEN_P1STIFF3D_VAR, eigmi.GEN_P1STIFF3D),
                                       (eigmi.GEN_P1MASS3D_VAR, eigmi.GEN_P1MASS3D)])
def test_p1_varcoef_generator(kind, base):
    """kinds 9 / 10: the P1 Kuhn pattern of kinds 6 / 7, bitwise symmetric (element contributions summed
    in element order), SPD, and no longer class-constant (values vary row to row)."""
    import scipy.sparse as sp
    N = 9
    r, c, v = eigmi.gen_matrix(kind, N)
    r0, c0, v0 = eigmi.gen_matrix(base, N)
    assert np.array_equal(r, r0) and np.array_equal(c, c0)
    S = sp.csr_matrix((v, c, r), shape=(N ** 3, N ** 3))
    assert (S != S.T).nnz == 0
    assert np.linalg.eigvalsh(S.toarray()).min() > 0
    ratio = v / np.where(v0 == 0, 1, v0)
    assert ratio[v0 != 0].min() >= 0.5 - 1e-12 and ratio[v0 != 0].max() < 1.5
    assert len(np.unique(np.round(ratio[v0 != 0], 12))) > 100
    # the distributed generator produces the same rows
    r2, c2, v2 = eigmi.gen_rows(kind, N, 2 * N * N, 3 * N * N)
    assert np.array_equal(v2, v[r[2 * N * N]:r[5 * N * N]])


def _box_random(nx, ny, nz, seed):
    """Random symmetric 7-point values on an nx x ny x nz box (positive diagonal, one random value per
    grid edge)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    n = nx * ny * nz
    idx = np.arange(n)
    x, y, z = idx % nx, (idx // nx) % ny, idx // (nx * ny)
    rows, cols, vals = [idx], [idx], [6.0 + rng.random(n)]
    for step, ok in ((1, x < nx - 1), (nx, y < ny - 1), (nx * ny, z < nz - 1)):
        i = idx[ok]
        w = -0.5 - rng.random(i.size)
        rows += [i, i + step]
        cols += [i + step, i]
        vals += [w, w]
    S = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    S.sort_indices()
    return oracle.CSR(n, S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data.astype(np.float64))


MATS = {
    "varcoef64": lambda: (varcoef(64), 0),
    "poisson64_arrays": lambda: (oracle.poisson3d(64), eigmi.MAT_NO_UNIFORM),
    "box64x16x20": lambda: (_box_random(64, 16, 20, 3), 0),
    "box128x3x9": lambda: (_box_random(128, 3, 9, 4), 0),
}


@pytest.mark.gpu
@pytest.mark.parametrize("mat", list(MATS))
def test_value_march_bitwise(ctx, mat):
    A, flags = MATS[mat]()
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, flags=flags)
    info = M.info
    # automatic: the fused step on the value pack (15), eig_mv on the plain masked march (0)
    assert info.sym_geo == 1 and info.sym_uniform == 0 and info.march_variant == 15 and info.march_variant_mv == 0
    n = A.n
    assert M.lanczos_kernel_info(True) == ("k_lanczos_fused_march", 8 * 4 * n + 32 * n)
    assert eigmi.image_bytes(M, "spmv") == 8 * info.sym_arrays * n + n + 16 * n
    x = np.random.default_rng(11).standard_normal(n)
    ref = oracle.csr_mv(A, x)
    for runs in (0, 1, 2, 3, 5, 7):
        base = {}
        # 1: the plain masked march on the arrays; 9 / 10 / 12 / 13: variants 10 / 11 / 14 / 15 (the same
        # rows per wave: alpha / beta bitwise)
        for pf in (1, 9, 10, 12, 13, 15):
            M.tune(runs, march_prefetch=pf)
            assert M.info.march_variant == {1: 0, 9: 10, 10: 11, 12: 14, 13: 15, 15: 18}[pf]
            assert np.array_equal(M.mv_host(x), ref), (runs, pf)
            for fused in (False, True):
                a, b, _ = eigmi.lanczos_run(M, 25, seed=7, fused=fused)
                if pf == 1:
                    base[fused] = (a, b)
                else:
                    assert np.array_equal(a, base[fused][0]) and np.array_equal(b, base[fused][1]), (runs, pf, fused)
    M.tune(0, march_prefetch=0)
    fa, fb, _ = eigmi.lanczos_run(M, 20, seed=123, fused=True)
    qa, qb = oracle.lanczos_fused(A, oracle.random_vec(n, 123), 20)
    assert np.allclose(fa, qa, rtol=1e-12, atol=0) and np.allclose(fb, qb, rtol=1e-12, atol=0)
    ca, cb, _ = eigmi.lanczos_run(M, 20, seed=123)
    _, ra, rb = oracle.lanczos(A, oracle.random_vec(n, 123), 20)
    assert np.allclose(ca, ra, rtol=1e-12, atol=0) and np.allclose(cb, rb, rtol=1e-12, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("mat", list(MATS))
def test_value_march_two_lines(ctx, mat):
    """March variants 22 / 23 (EIG_TUNE_MARCH_PREFETCH 16 / 17: the value pack marched TWO grid lines
    per wave, the +-nx neighbours across the pair from registers): eig_mv BITWISE the reference row
    loop (each row sums what variant 15 sums, in the same order), the fused and classic recurrences
    within 1e-12 of their restatements, at several plane-run counts; a grid with an odd line count
    keeps variant 15."""
    A, flags = MATS[mat]()
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val, flags=flags)
    n = A.n
    odd = mat == "box128x3x9"
    x = np.random.default_rng(12).standard_normal(n)
    ref = oracle.csr_mv(A, x)
    U0 = oracle.random_vec(n, 123)
    qa, qb = oracle.lanczos_fused(A, U0, 20)
    _, ra, rb = oracle.lanczos(A, U0, 20)
    for runs in (0, 1, 2, 5):
        for pf in (16, 17):
            M.tune(runs, march_prefetch=pf)
            assert M.info.march_variant == (15 if odd else pf + 6), (runs, pf)
            assert np.array_equal(M.mv_host(x), ref), (runs, pf)
            fa, fb, _ = eigmi.lanczos_run(M, 20, seed=123, fused=True)
            assert np.allclose(fa, qa, rtol=1e-12, atol=0) and np.allclose(fb, qb, rtol=1e-12, atol=0), (runs, pf)
            ca, cb, _ = eigmi.lanczos_run(M, 20, seed=123)
            assert np.allclose(ca, ra, rtol=1e-12, atol=0) and np.allclose(cb, rb, rtol=1e-12, atol=0), (runs, pf)
    M.tune(0, march_prefetch=0)


@pytest.mark.gpu
def test_value_march_after_shift(ctx):
    """A += sigma I updates the band values the value marches stream (StandardLargest's shift,
    eigensolver.hh:59-66), the value pack included (built at first use, refilled in place by the
    shift): eig_mv bitwise the shifted reference matrix on every variant, and the fused step's alpha /
    beta bitwise equal across the variants (same rows per wave)."""
    A = varcoef(64)
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    assert M.info.march_variant == 15
    x = np.random.default_rng(2).standard_normal(A.n)
    M.tune(march_prefetch=13)  # eig_mv on the pack too: built now
    assert np.array_equal(M.mv_host(x), oracle.csr_mv(A, x))
    M.shift_diag(-2.375)
    val = A.val.copy()
    oracle.lib.orc_shift_diag(A.n, A.rowptr, A.col, val, -2.375)
    B = oracle.CSR(A.nrows, A.rowptr, A.col, val)
    ref = None
    for pf in (13, 9, 1, 0):
        M.tune(march_prefetch=pf)
        assert np.array_equal(M.mv_host(x), oracle.csr_mv(B, x)), pf
        a, b, _ = eigmi.lanczos_run(M, 10, seed=3, fused=True)
        if ref is None:
            ref = (a, b)
        else:
            assert np.array_equal(a, ref[0]) and np.array_equal(b, ref[1]), pf


@pytest.mark.gpu
def test_lower_only_entry_not_uniform(ctx):
    """A constant band whose one LOWER entry (its mirror not stored: a one-sided pattern) has another
    value must not be taken as a uniform band (the uniform march would use the array's constant for
    it).  Row 1000 of the 16^3 Poisson keeps (1000, 999) = -2.5 while (999, 1000) is dropped."""
    P = oracle.poisson3d(16)
    keep = np.ones(P.val.size, bool)
    r = 999
    keep[P.rowptr[r] + int(np.nonzero(P.col[P.rowptr[r]:P.rowptr[r + 1]] == 1000)[0][0])] = False
    val = P.val.copy()
    val[P.rowptr[1000] + int(np.nonzero(P.col[P.rowptr[1000]:P.rowptr[1001]] == 999)[0][0])] = -2.5
    counts = np.diff(P.rowptr) - np.add.reduceat(~keep, P.rowptr[:-1]).astype(np.int64)
    rp = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    A = oracle.CSR(P.n, rp, P.col[keep].copy(), val[keep].copy())
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    assert M.info.sym_offsets == 7 and M.info.sym_uniform == 0
    x = np.random.default_rng(5).standard_normal(A.n)
    assert np.array_equal(M.mv_host(x), oracle.csr_mv(A, x))


@pytest.fixture(scope="module")
def v256(ctx):
    N = 256
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_VARCOEF3D, N)
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v)
    return N, M, oracle.CSR(N ** 3, rp, c, v)


@pytest.mark.gpu
def test_value_march_256_bitwise(ctx, v256):
    """Configuration size (C4's grid, variable coefficients): eig_mv bitwise the oracle row loop."""
    N, M, A = v256
    assert M.info.march_variant == 22 and M.info.march_variant_mv == 0
    x = np.random.default_rng(9).standard_normal(N ** 3)
    assert np.array_equal(M.mv_host(x), oracle.csr_mv(A, x))


FULL_STEPS = 60  # fused steps compared with the restatement at 256^3 (the oracle: ~10 steps / s)


def fused_vs_oracle(M, A, steps):
    """`steps` fused GPU steps (the benchmark's kernel) against orc_lanczos_fused on the same matrix
    and start vector -- GPU against the CPU restatement, no GPU-vs-GPU step -- rtol 1e-12."""
    n = A.n
    U0 = np.zeros(n)
    oracle.lib.orc_random_vec(n, 123, U0)
    fa, fb, _ = eigmi.lanczos_run(M, steps, seed=123, fused=True)
    ra, rb = oracle.lanczos_fused(A, U0, steps)
    assert fa.size == steps and rb.size == steps + 1
    da = np.max(np.abs(fa - ra) / np.abs(ra))
    db = np.max(np.abs(fb[1:] - rb[1:]) / np.abs(rb[1:]))
    print(f"{steps} fused steps vs orc_lanczos_fused: max rel diff alpha {da:.2e}, beta {db:.2e}")
    assert np.allclose(fa, ra, rtol=1e-12, atol=0) and np.allclose(fb, rb, rtol=1e-12, atol=0)
    return U0


@pytest.mark.gpu
def test_value_march_256_lanczos(ctx, v256):
    """The benchmark step on the value-streaming image at 256^3 (kind 8, march variant 22 -- the
    2-line march, the default from EIG_MARCH_2L_MIN_ROWS rows): 60 fused steps vs orc_lanczos_fused
    and 4 classic steps vs orc_lanczos_rotating, rtol 1e-12."""
    N, M, A = v256
    n = N ** 3
    assert M.info.march_variant == 22
    U0 = fused_vs_oracle(M, A, FULL_STEPS)
    ca, cb, _ = eigmi.lanczos_run(M, 4, seed=123)
    u1, u2 = np.zeros(n), np.zeros(n)
    qa, qb = np.zeros(4), np.zeros(5)
    oracle.lib.orc_lanczos_rotating(n, A.rowptr, A.col, A.val, 4, U0, u1, u2, qa, qb)
    assert np.allclose(ca, qa, rtol=1e-12, atol=0) and np.allclose(cb, qb, rtol=1e-12, atol=0)


@pytest.fixture(scope="module")
def p256a(ctx):
    """The benchmark's exact image: 3-D Poisson 256^3 uploaded with EIG_MAT_NO_UNIFORM (every band
    value streamed from HBM on every step; bench.py --image arrays, the default)."""
    N = 256
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=eigmi.MAT_NO_UNIFORM)
    yield N, M, oracle.CSR(N ** 3, rp, c, v)
    M.close()


@pytest.mark.gpu
def test_bench_image_256_spmv_bitwise(ctx, p256a):
    """eig_mv (BCRSMatrix::mv, kernels_cpp.hh:596-621) on the benched image, bitwise the oracle row loop."""
    N, M, A = p256a
    info = M.info
    assert info.sym_uniform == 0 and info.march_variant == 22 and info.march_variant_mv == 0
    x = np.random.default_rng(21).standard_normal(N ** 3)
    assert np.array_equal(M.mv_host(x), oracle.csr_mv(A, x))


@pytest.mark.gpu
@pytest.mark.parametrize("pf", [13, 17])
def test_bench_image_256_other_variants(ctx, p256a, pf):
    """The benched image with variant 15 (one line per wave: the default below EIG_MARCH_2L_MIN_ROWS
    rows, i.e. on the ranks of the 8-GPU split) and variant 23 (2 lines, 4 waves per SIMD): eig_mv
    bitwise the oracle row loop and 60 fused steps vs orc_lanczos_fused, rtol 1e-12."""
    N, M, A = p256a
    M.tune(march_prefetch=pf)
    try:
        assert M.info.march_variant == {13: 15, 17: 23}[pf] and M.info.march_variant_mv == {13: 15, 17: 23}[pf]
        x = np.random.default_rng(22).standard_normal(N ** 3)
        assert np.array_equal(M.mv_host(x), oracle.csr_mv(A, x))
        fused_vs_oracle(M, A, FULL_STEPS)
    finally:
        M.tune(march_prefetch=0)


@pytest.mark.gpu
def test_bench_image_256_fused_steps(ctx, p256a):
    """The benched kernel (k_lanczos_fused_march<.., 15> on the Poisson 256^3 arrays image): 60 fused
    steps vs orc_lanczos_fused, rtol 1e-12 (arpack_geneo_wrapper.hh:621-632 drives the same recurrence
    through ARPACK's dsaupd)."""
    N, M, A = p256a
    assert M.lanczos_kernel_info(True) == ("k_lanczos_fused_march", 64 * N ** 3)
    fused_vs_oracle(M, A, FULL_STEPS)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,N", [(eigmi.GEN_P1STIFF3D, 64), (eigmi.GEN_P1MASS3D, 64), (eigmi.GEN_P1STIFF3D, 128),
                                    (eigmi.GEN_P1STIFF3D_VAR, 64), (eigmi.GEN_P1MASS3D_VAR, 64)])
def test_kuhn_box_march(ctx, kind, N):
    """The P1 Kuhn 15-point box march (march variants 20 / 16 / 12, config C5's K and M): eig_mv bitwise the
    reference row loop; the fused and classic recurrences within 1e-12 of their restatements and of
    the row kernels (EIG_TUNE_MARCH_PREFETCH = 1: no march) at every plane-run count.  Kinds 9 / 10
    (variable coefficients: every entry of an offset differs, so a mirrored lower value read from the
    wrong row would show) as well as the constant-coefficient kinds 6 / 7."""
    rp, c, v = eigmi.gen_matrix(kind, N)
    A = oracle.CSR(N ** 3, rp, c, v)
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v)
    info = M.info
    assert info.sym_offsets == 15 and info.march_variant == 20, (info.sym_offsets, info.march_variant)
    n = A.n
    assert M.lanczos_kernel_info(True) == ("k_lanczos_fused_march", 8 * info.sym_arrays * n + 32 * n)
    x = np.random.default_rng(13).standard_normal(n)
    ref = oracle.csr_mv(A, x)
    assert np.array_equal(M.mv_host(x), ref)
    M.tune(march_prefetch=1)  # row kernels
    assert M.info.march_variant == -1
    assert np.array_equal(M.mv_host(x), ref)
    base = {f: eigmi.lanczos_run(M, 25, seed=7, fused=f)[:2] for f in (False, True)}
    # 0: the Kuhn pack with the line exchange in LDS (variant 20, default), 13: the pack alone (16),
    # 14: the arrays (12)
    for pf in (0, 13, 14):
        M.tune(march_prefetch=pf)
        assert M.info.march_variant == {0: 20, 13: 16, 14: 12}[pf]
        for runs in (0, 1, 3, 7):
            M.tune(runs)
            assert np.array_equal(M.mv_host(x), ref), (runs, pf)
            for fused in (False, True):
                a, b, _ = eigmi.lanczos_run(M, 25, seed=7, fused=fused)
                assert np.allclose(a, base[fused][0], rtol=1e-12, atol=0) and \
                    np.allclose(b, base[fused][1], rtol=1e-12, atol=0), (runs, pf, fused)
    M.tune(0, march_prefetch=0)
    fa, fb, _ = eigmi.lanczos_run(M, 15, seed=123, fused=True)
    qa, qb = oracle.lanczos_fused(A, oracle.random_vec(n, 123), 15)
    assert np.allclose(fa, qa, rtol=1e-12, atol=0) and np.allclose(fb, qb, rtol=1e-12, atol=0)
