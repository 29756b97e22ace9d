"""the exported-LU-factor apply matmul_inverse_tallskinny_blocked
(kernels_cpp.hh:660-755) and the inverse drivers StandardInverse / GeneralizedInverse
(eigensolver.hh:116-351).

CPU (no GPU): the host factorisation (eig_lu_create_bcsr with a NULL context) against numpy --
P R A Q = L U to rounding -- and the oracle's restatement of the reference's factor apply against
numpy solves; the oracle drivers against the analytic 2-D Dirichlet spectrum (.cc:437-446).
GPU: eig_inverse_mv8 BITWISE equal to the oracle restatement on the same factors (the device keeps
the reference's per-row operation order), through both factor entry points, with do_recip 0 / 1;
the device drivers against the oracle drivers (same iteration count, eigenvalues to 1e-12
relative: only the reductions' summation order differs) and against analytic eigenvalues."""
import numpy as np
import pytest
import scipy.sparse as sp

import eigmi
import oracle


def factors(A):
    lu = eigmi.LU.from_bcsr(None, A.rowptr, A.col, A.val, A.br)
    d = lu.export()
    lu.close()
    return d


def dense(A):
    return A.to_scipy().toarray()


CASES = {
    "laplace2d_16": lambda: oracle.laplace2d(16),
    "poisson3d_8": lambda: oracle.poisson3d(8),
    "q1elast_4": lambda: oracle.q1elast(4),
    "neumann2d_12": lambda: oracle.laplace2d(12, "neumann"),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_host_lu_factorisation(name):
    A = CASES[name]()
    if name.startswith("neumann"):  # singular: factor the shifted operator as StandardInverse would
        A.val[A.col == np.repeat(np.arange(A.n), np.diff(A.rowptr))] += 0.5
    d = factors(A)
    n = A.n
    L = sp.csr_matrix((d["Lx"], d["Lj"], d["Lp"]), shape=(n, n)).toarray()
    U = sp.csc_matrix((d["Ux"], d["Ui"], d["Up"]), shape=(n, n)).toarray()
    assert np.allclose(np.diag(L), 1.0) and np.all(np.triu(L, 1) == 0) and np.all(np.tril(U, -1) == 0)
    # unit diagonal last in each L row, diagonal last in each U column (umfpacktools.hh contract)
    assert np.all(d["Lj"][d["Lp"][1:] - 1] == np.arange(n)) and np.all(d["Ui"][d["Up"][1:] - 1] == np.arange(n))
    B = (dense(A) / d["Rs"][:, None])[d["P"]][:, d["Q"]]
    assert np.abs(L @ U - B).max() <= 1e-13 * np.abs(B).max()


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_inverse_solves(name):
    A = CASES[name]()
    if name.startswith("neumann"):
        A.val[A.col == np.repeat(np.arange(A.n), np.diff(A.rowptr))] += 0.5
    f = oracle.LU(**factors(A))
    n, m = A.n, 16
    X = oracle.random_mv8(n, m, 3)
    out, _ = oracle.inverse_mv8(f, X, m)
    Xc, Oc = oracle.mv_to_cols(X, n, m), oracle.mv_to_cols(out, n, m)
    Ad = dense(A)
    assert np.abs(Ad @ Oc - Xc).max() <= 1e-10 * np.abs(Xc).max() * np.linalg.cond(Ad) / 1e3 + 1e-12


def test_oracle_standard_inverse_known_answer():
    """StandardInverse at tight tolerance: the 4 smallest eigenvalues of the 2-D Dirichlet
    Laplacian, the reference's own known answer (src/dune-eigensolver.cc:437-446)."""
    N = 16
    A = oracle.laplace2d(N)
    f = oracle.LU(**factors(A))
    ev, _, it = oracle.standard_inverse(A, f, 0.0, 1e-13, 2000, 4, 123)
    exact = np.sort(oracle.eig_laplace2d(N))[:4]
    assert np.allclose(np.sort(ev), exact, rtol=0, atol=1e-9), (ev, exact)


def test_oracle_generalized_inverse_identity_b():
    """GeneralizedInverse with B = I on A's pattern (.cc:145-156 generator) and a shift: the pencil's
    eigenvalues are A's (the returned ra subtracts the shift, :276-277)."""
    N = 12
    A, B = oracle.laplace2d(N), oracle.laplace2d(N, "identity")
    shift = 0.75
    As = oracle.CSR(A.nrows, A.rowptr, A.col, A.val + shift * B.val)
    f = oracle.LU(**factors(As))
    ev, _, it = oracle.generalized_inverse(A, B, f, shift, 0.0, 1e-14, 3000, 4, 123)
    exact = np.sort(oracle.eig_laplace2d(N))[:4]
    assert it > 10 and np.allclose(np.sort(ev), exact, rtol=0, atol=1e-9)


# ------------------------------------------------------------------------------------------- GPU
def _gpu_lu(ctx, A, via="bcsr", recip=False):
    if via == "bcsr":
        lu = eigmi.LU.from_bcsr(ctx, A.rowptr, A.col, A.val, A.br)
        d = lu.export()
        return lu, oracle.LU(**d)
    d = factors(A)
    if recip:  # the same factor in the do_recip form: rows multiplied by 1 / Rs
        d = dict(d, Rs=1.0 / d["Rs"], do_recip=1)
    lu = eigmi.LU.from_factors(ctx, **d)
    return lu, oracle.LU(**d)


class trsv_kernel:
    """eig_lu_set_solver for the duration of a block: "staged" / "csr" (bitwise kernels) or None (the
    default: the block-inverse solve where the factor has its image)."""

    def __init__(self, lu, kind):
        self.lu, self.kind = lu, kind

    def __enter__(self):
        self.lu.set_solver(self.kind)

    def __exit__(self, *a):
        self.lu.set_solver(None)


# The block-inverse solve multiplies by inv(D_b) instead of substituting: agreement with the
# reference arithmetic to rounding.  Bound: 1e-13 of the largest |entry| of the result.
BINV_RTOL = 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("name,m,via", [("laplace2d_16", 8, "bcsr"), ("poisson3d_8", 16, "factors"),
                                        ("q1elast_4", 24, "bcsr"), ("neumann2d_12", 8, "factors")])
@pytest.mark.parametrize("kernel", ["staged", None])
def test_inverse_mv8_bitwise(ctx, name, m, via, kernel):
    A = CASES[name]()
    if name.startswith("neumann"):
        A.val[A.col == np.repeat(np.arange(A.n), np.diff(A.rowptr))] += 0.5
    lu, f = _gpu_lu(ctx, A, via)
    n = A.n
    X = oracle.random_mv8(n, m, 11)
    ref_out, ref_in = oracle.inverse_mv8(f, X, m)
    din, dout = ctx.array(X), ctx.zeros(n * m)
    with trsv_kernel(lu, kernel):
        lu.inverse_mv8(m, din, dout)
    out = dout.get()
    if kernel == "staged":
        assert np.array_equal(out, ref_out), "A^-1 Q not bitwise the reference arithmetic"
    else:
        err = np.abs(out - ref_out).max() / np.abs(ref_out).max()
        print(f"{name}: block-inverse vs reference arithmetic {err:.2e}")
        assert err <= BINV_RTOL
    # Qin is scratch afterwards ("you may overwrite the input argument", kernels_cpp.hh:659); its
    # contents are not part of the contract (the reference leaves U-solve partial sums there)
    lu.close()


@pytest.mark.gpu
def test_inverse_mv8_interior_shift(ctx):
    """factors of an interior shift (laplace2d(32) - sigma I, sigma between lambda_5 and
    lambda_6) -- small U pivots.  Either the block-inverse image is refused for an ill-conditioned
    diagonal block (kBinvCond) and the default is a bitwise substitution kernel, or its result stays
    within 1e-11 of the reference arithmetic relative to max |x|."""
    A = oracle.laplace2d(32)
    N = 32
    s1 = 4 * np.sin(np.arange(1, N + 1) * np.pi / (N + 1) / 2) ** 2
    lam = np.sort((s1[:, None] + s1[None, :]).ravel())
    sigma = 0.5 * (lam[5] + lam[6]) + 1e-3
    A.val[A.col == np.repeat(np.arange(A.n), np.diff(A.rowptr))] -= sigma
    lu, f = _gpu_lu(ctx, A, "bcsr")
    X = oracle.random_mv8(A.n, 8, 4)
    ref_out, _ = oracle.inverse_mv8(f, X, 8)
    din, dout = ctx.array(X), ctx.zeros(A.n * 8)
    lu.inverse_mv8(8, din, dout)
    out = dout.get()
    used, _, _ = lu.solver_info()
    err = np.abs(out - ref_out).max() / np.abs(ref_out).max()
    print(f"interior shift: kernel {used}, vs reference arithmetic {err:.2e}")
    if used == "blockinv":
        assert err <= 1e-11
    else:
        assert np.array_equal(out, ref_out)
    with trsv_kernel(lu, "staged"):
        din = ctx.array(X)
        lu.inverse_mv8(8, din, dout)
    assert np.array_equal(dout.get(), ref_out)
    lu.close()


@pytest.mark.gpu
def test_inverse_mv8_do_recip(ctx):
    A = oracle.poisson3d(6)
    lu, f = _gpu_lu(ctx, A, "factors", recip=True)
    X = oracle.random_mv8(A.n, 8, 2)
    ref_out, _ = oracle.inverse_mv8(f, X, 8)
    din, dout = ctx.array(X), ctx.zeros(A.n * 8)
    with trsv_kernel(lu, "staged"):
        lu.inverse_mv8(8, din, dout)
    assert np.array_equal(dout.get(), ref_out)
    din = ctx.array(X)
    lu.inverse_mv8(8, din, dout)
    assert np.abs(dout.get() - ref_out).max() <= BINV_RTOL * np.abs(ref_out).max()


@pytest.mark.gpu
def test_inverse_mv8_unsorted_rows(ctx):
    """Factors whose L rows are not in ascending column order (possible from UMFPACK): the device
    sorts them, so the result equals the reference to rounding (1e-13), not bitwise."""
    A = oracle.laplace2d(12)
    d = factors(A)
    Lj, Lx = d["Lj"].copy(), d["Lx"].copy()
    for i in range(A.n):
        a, b = d["Lp"][i], d["Lp"][i + 1] - 1  # keep the unit diagonal last
        Lj[a:b], Lx[a:b] = Lj[a:b][::-1].copy(), Lx[a:b][::-1].copy()
    d2 = dict(d, Lj=Lj, Lx=Lx)
    lu = eigmi.LU.from_factors(ctx, **d2)
    X = oracle.random_mv8(A.n, 8, 4)
    ref_out, _ = oracle.inverse_mv8(oracle.LU(**d2), X, 8)
    din, dout = ctx.array(X), ctx.zeros(A.n * 8)
    lu.inverse_mv8(8, din, dout)
    assert np.abs(dout.get() - ref_out).max() <= 1e-13 * np.abs(ref_out).max()


@pytest.mark.gpu
@pytest.mark.parametrize("shift,tol,nev", [(0.0, 1e-10, 4), (0.3, 1e-8, 10)])
def test_standard_inverse_vs_oracle(ctx, shift, tol, nev):
    N = 16
    A = oracle.laplace2d(N)
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    ev, evec, it = eigmi.standard_inverse(M, shift, tol, 1000, nev, 123)
    As = oracle.CSR(A.nrows, A.rowptr, A.col, A.val.copy())
    oracle.lib.orc_shift_diag(As.n, As.rowptr, As.col, As.val, shift)
    f = oracle.LU(**factors(As))  # the device factored the same shifted matrix with the same code
    rev, revec, rit = oracle.standard_inverse(A, f, shift, tol, 1000, nev, 123)
    assert it == rit
    assert np.allclose(ev, rev, rtol=1e-12, atol=0)
    exact = np.sort(oracle.eig_laplace2d(N))[:4]
    if tol <= 1e-10:
        assert np.allclose(np.sort(ev)[:4], exact, rtol=0, atol=1e-8)


@pytest.mark.gpu
def test_generalized_inverse_vs_oracle(ctx):
    N = 12
    A, B = oracle.laplace2d(N), oracle.laplace2d(N, "identity")
    dA = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    dB = eigmi.Matrix.from_bcsr(ctx, B.rowptr, B.col, B.val)
    shift, reg = 0.75, 0.0
    ev, _, it = eigmi.generalized_inverse(dA, dB, shift, reg, 1e-12, 500, 4, 123)
    As = oracle.CSR(A.nrows, A.rowptr, A.col, A.val + shift * B.val)
    f = oracle.LU(**factors(As))
    rev, _, rit = oracle.generalized_inverse(A, B, f, shift, reg, 1e-12, 500, 4, 123)
    assert it == rit and np.allclose(ev, rev, rtol=1e-12, atol=0)
    assert np.allclose(np.sort(ev), np.sort(oracle.eig_laplace2d(N))[:4], rtol=0, atol=1e-8)


@pytest.mark.gpu
def test_generalized_inverse_pu_mass(ctx):
    """The reference harness's GenEO-type pencil (.cc:98-143): Neumann Laplacian A, partition-of-
    unity-masked B, shift + regularisation; device = oracle driver (iterations, values 1e-10)."""
    N, shift, reg = 16, 1.0, 1e-3
    A, B = oracle.laplace2d(N, "neumann"), oracle.laplace2d(N, "pu", overlap=3)
    dA = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    dB = eigmi.Matrix.from_bcsr(ctx, B.rowptr, B.col, B.val)
    ev, _, it = eigmi.generalized_inverse(dA, dB, shift, reg, 1e-8, 200, 8, 123)
    diag = A.col == np.repeat(np.arange(A.n), np.diff(A.rowptr))
    As = oracle.CSR(A.nrows, A.rowptr, A.col, A.val + shift * B.val + reg * diag)
    f = oracle.LU(**factors(As))
    rev, _, rit = oracle.generalized_inverse(A, B, f, shift, reg, 1e-8, 200, 8, 123)
    assert it == rit and np.allclose(ev, rev, rtol=1e-10, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["laplace2d_64", "laplace2d_100", "laplace2d_150", "poisson3d_12", "poisson3d_16",
                                  "poisson3d_20", "laplace2d_200"])
@pytest.mark.parametrize("kernel", ["staged", "csr", None])
def test_inverse_mv8_kernels(ctx, name, kernel):
    """The bitwise triangular-solve kernels (k_tsolve_staged: envelope factors of bandwidth <= 256;
    k_tsolve: any factor) reproduce the reference arithmetic bitwise; the default block-inverse
    solve (factors that fit the staged image) to BINV_RTOL.  poisson3d_20's RCM envelope reaches
    past 256 rows: it always takes k_tsolve.  laplace2d_100: n = 10000, a ragged last block.  The
    block-inverse chain's coupled-block counts: laplace2d_64 1, laplace2d_100 / poisson3d_12 2,
    poisson3d_16 4 (RCM bandwidth 200).  The block-inverse chain is independent of the staged image
    (coupled distances 3 and up to 8 compared with the reference arithmetic):
    laplace2d_150 3, poisson3d_20 and laplace2d_200 (the reference's ev.N, n = 40000) 5-8."""
    A = {"laplace2d_64": lambda: oracle.laplace2d(64), "laplace2d_100": lambda: oracle.laplace2d(100),
         "laplace2d_150": lambda: oracle.laplace2d(150), "laplace2d_200": lambda: oracle.laplace2d(200),
         "poisson3d_12": lambda: oracle.poisson3d(12),
         "poisson3d_16": lambda: oracle.poisson3d(16), "poisson3d_20": lambda: oracle.poisson3d(20)}[name]()
    lu, f = _gpu_lu(ctx, A, "bcsr")
    used, gl, gu = lu.solver_info()
    print(f"{name}: default kernel {used}, coupled blocks L {gl} U {gu}")
    if name in ("laplace2d_150", "laplace2d_200", "poisson3d_20"):
        assert used == "blockinv" and max(gl, gu) >= 3
    X = oracle.random_mv8(A.n, 16, 3)
    ref_out, _ = oracle.inverse_mv8(f, X, 16)
    with trsv_kernel(lu, kernel):
        din, dout = ctx.array(X), ctx.zeros(A.n * 16)
        lu.inverse_mv8(16, din, dout)
    out = dout.get()
    if kernel in (None, "blockinv_mfma"):
        err = np.abs(out - ref_out).max() / np.abs(ref_out).max()
        print(f"{name}: default solve vs reference arithmetic {err:.2e}")
        assert err <= BINV_RTOL
    else:
        assert np.array_equal(out, ref_out)
    lu.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["laplace2d_16", "poisson3d_8", "q1elast_4", "neumann2d_12", "laplace2d_100",
                                  "poisson3d_16", "tiny_5"])
def test_device_band_factors_match_host(ctx, name):
    """eig_lu_create_bcsr with a context factors on the device (k_band.hip: band LU of 64 x 64 tiles +
    the block-inverse image built from the tiles).  Its exported factors carry the host envelope LU's
    pattern, permutations and scaling exactly and its values to rounding (same no-pivoting
    elimination, different operation order): 1e-12 of the largest |entry| per factor, the same
    pattern where no entry cancels exactly.  Rows past n
    in the last block (laplace2d_100: n = 10000; tiny_5: n = 25 < 64) are identity padding."""
    A = {"laplace2d_100": lambda: oracle.laplace2d(100), "poisson3d_16": lambda: oracle.poisson3d(16),
         "tiny_5": lambda: oracle.laplace2d(5)}.get(name, CASES.get(name))()
    if name.startswith("neumann"):
        A.val[A.col == np.repeat(np.arange(A.n), np.diff(A.rowptr))] += 0.5
    host = eigmi.LU.from_bcsr(None, A.rowptr, A.col, A.val, A.br).export()
    lu = eigmi.LU.from_bcsr(ctx, A.rowptr, A.col, A.val, A.br)
    used, gl, gu = lu.solver_info()
    dev = lu.export()
    for k in ("P", "Q", "Rs"):
        assert np.array_equal(dev[k], host[k]), k
    # (entries that cancel to exactly 0.0 in one operation order may be ~1e-17 in the other -- the
    # 3 x 3 elasticity blocks have such -- so the factors are compared as matrices, not patterns)
    import scipy.sparse as sp
    n = A.n

    def mats(d):
        L = sp.csr_matrix((d["Lx"], d["Lj"], d["Lp"]), shape=(n, n))
        U = sp.csc_matrix((d["Ux"], d["Ui"], d["Up"]), shape=(n, n))
        return L, U

    (Ld, Ud), (Lh, Uh) = mats(dev), mats(host)
    assert abs(Ld - Lh).max() <= 1e-12 * abs(Lh).max()
    assert abs(Ud - Uh).max() <= 1e-12 * abs(Uh).max()
    if not name.startswith("q1elast"):
        for k in ("Lp", "Lj", "Up", "Ui"):
            assert np.array_equal(dev[k], host[k]), k
    # the solve on the device-built image vs the reference arithmetic on the exported factors
    X = oracle.random_mv8(A.n, 8, 5)
    ref_out, _ = oracle.inverse_mv8(oracle.LU(**dev), X, 8)
    din, dout = ctx.array(X), ctx.zeros(A.n * 8)
    lu.inverse_mv8(8, din, dout)
    err = np.abs(dout.get() - ref_out).max() / np.abs(ref_out).max()
    print(f"{name}: kernel {used} (coupled {gl}/{gu}), device image vs reference arithmetic {err:.2e}")
    assert used == "blockinv" and err <= BINV_RTOL
    lu.close()


@pytest.mark.gpu
def test_device_lu_rejects_factors_that_need_pivoting(ctx):
    """the device band LU does not pivot (UMFPACK, the reference's factoriser,
    does).  A matrix whose every unpivoted elimination order meets a tiny pivot (3x3 blocks with
    1e-13 on the diagonal and ones elsewhere: well conditioned, eigenvalues 2 and -1) must be
    rejected by the backward-error check (EIG_ERR_BREAKDOWN), not solved to garbage."""
    import scipy.sparse as sp
    blk = np.ones((3, 3)) - np.eye(3) + 1e-13 * np.eye(3)
    A = sp.block_diag([blk] * 200).tocsr()
    A.sort_indices()
    with pytest.raises(eigmi.EigError) as e:
        eigmi.LU.from_bcsr(ctx, A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data.copy())
    assert e.value.code in (eigmi.EIG_ERR_BREAKDOWN,), str(e.value)
    # a well-pivoted matrix of the same pattern passes the check
    good = sp.block_diag([4 * np.eye(3) - (np.ones((3, 3)) - np.eye(3))] * 200).tocsr()
    good.sort_indices()
    lu = eigmi.LU.from_bcsr(ctx, good.indptr.astype(np.int64), good.indices.astype(np.int32), good.data.copy())
    lu.close()


def _inverse_setup(ctx, A, shift):
    """The device matrix, its shifted host copy and the LU of that copy (handed to the driver AND to the
    loop below, so both apply the same factors)."""
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    As = oracle.CSR(A.nrows, A.rowptr, A.col, A.val.copy())
    oracle.lib.orc_shift_diag(As.n, As.rowptr, As.col, As.val, shift)
    lu = eigmi.LU.from_bcsr(ctx, As.rowptr, As.col, As.val)
    return M, As, lu


@pytest.mark.gpu
@pytest.mark.parametrize("maxiter,tol", [(1, 0.0), (2, 0.0), (12, 0.0), (4000, 1e-9)])
def test_standard_inverse_lookahead_loop(ctx, maxiter, tol):
    """the look-ahead StandardInverse (iteration k + 1 queued before iteration k's stopping
    test, basis ping-pong) against the reference's loop (eigensolver.hh:159-189) written with the
    device primitives: Q2 = A^-1 Q1 (:168), orthonormalize_blocked (:171), the product and its
    diagonal dots (:174-175), the absolute max|ds| test with k > 1 (:178-189).  Iterates BITWISE, the
    same iteration count, Ritz values within 1e-14 (the driver's dots are fused into its product)."""
    N, nev, shift = 20, 4, 0.2
    A = oracle.laplace2d(N)
    M, As, lu = _inverse_setup(ctx, A, shift)
    ev, evec, it = eigmi.standard_inverse(M, shift, tol, maxiter, nev, 17, lu=lu)
    n, m = A.n, 8
    Ms = eigmi.Matrix.from_bcsr(ctx, As.rowptr, As.col, As.val)  # the driver shifted M in place (:145-153)
    Q = [ctx.zeros(n * m), ctx.zeros(n * m)]
    Z, dp = ctx.zeros(n * m), ctx.zeros(m)
    eigmi.random_mv8(ctx, n, m, 17, Q[0])
    eigmi.orthonormalize_mv8(ctx, n, m, Q[0])
    s2 = np.zeros(m)
    kk, basis = 1, 0
    for k in range(1, maxiter):
        kk = k
        lu.inverse_mv8(m, Q[(k + 1) % 2], Q[k % 2])
        eigmi.orthonormalize_mv8(ctx, n, m, Q[k % 2])
        eigmi.spmm_mv8(Ms, m, Q[k % 2], Z)
        eigmi.dot_diag_mv8(ctx, n, m, Q[k % 2], Z, dp)
        s1 = dp.get() - shift
        dist = np.abs(s1 - s2).max()
        s2 = s1
        basis = k % 2
        if k > 1 and dist < tol:
            break
    q = Q[basis].get().reshape(m // 8, n, 8)
    ref_evec = np.stack([q[j // 8, :, j % 8] for j in range(nev)])
    print(f"StandardInverse maxiter {maxiter} tol {tol}: {it} iterations (reference loop {kk})")
    assert it == kk
    assert np.array_equal(evec, ref_evec)
    assert np.abs(ev - s2[:nev]).max() <= 1e-14 * max(1.0, np.abs(s2).max())
    lu.close()


@pytest.mark.gpu
@pytest.mark.parametrize("maxiter,tol", [(1, 0.0), (2, 0.0), (12, 0.0), (500, 1e-10)])
def test_generalized_inverse_lookahead_loop(ctx, maxiter, tol):
    """the look-ahead GeneralizedInverse against the reference's loop (eigensolver.hh:
    270-325) written with the device primitives: B-orthonormalise (:273), product + dots (:274-275),
    then per iteration Q2 = B Q1 (:302), Q1 = As^-1 Q2 (:303), B_orthonormalize_blocked (:304), the
    product's dots (:317) and the relative test with iter > 10 (:315-325).  Iterates BITWISE, the
    same iteration count, eigenvalues within 1e-14."""
    N, nev, shift, reg = 14, 4, 0.75, 1e-3
    A, B = oracle.laplace2d(N, "neumann"), oracle.laplace2d(N, "pu", overlap=3)
    assert np.array_equal(A.rowptr, B.rowptr) and np.array_equal(A.col, B.col)
    dA = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    dB = eigmi.Matrix.from_bcsr(ctx, B.rowptr, B.col, B.val)
    diag = A.col == np.repeat(np.arange(A.n), np.diff(A.rowptr))
    sv = A.val + shift * B.val  # the driver's host copy: v += shift b, then v += reg on the diagonal (:240-252)
    sv[diag] += reg
    lu = eigmi.LU.from_bcsr(ctx, A.rowptr, A.col, sv)
    ev, evec, it = eigmi.generalized_inverse(dA, dB, shift, reg, tol, maxiter, nev, 29, lu=lu)
    n, m = A.n, 8
    dAs = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, sv)
    Q = [ctx.zeros(n * m), ctx.zeros(n * m)]
    Z, dp, norm = ctx.zeros(n * m), ctx.zeros(m), ctx.zeros(1)
    eigmi.random_mv8(ctx, n, m, 29, Q[0])
    eigmi.b_orthonormalize_mv8(dB, m, Q[0], norm)
    eigmi.spmm_mv8(dAs, m, Q[0], Z)
    eigmi.dot_diag_mv8(ctx, n, m, Q[0], Z, dp)
    ra2 = dp.get() - shift
    it_ref, basis = 0, 0
    while it_ref < maxiter:
        it_ref += 1
        i = it_ref
        eigmi.spmm_mv8(dB, m, Q[(i + 1) % 2], Z)
        lu.inverse_mv8(m, Z, Q[i % 2])
        eigmi.b_orthonormalize_mv8(dB, m, Q[i % 2], norm)
        eigmi.spmm_mv8(dAs, m, Q[i % 2], Z)
        eigmi.dot_diag_mv8(ctx, n, m, Q[i % 2], Z, dp)
        ra1 = dp.get() - shift
        basis = i % 2
        rel = np.abs(ra1 - ra2).max() / ra1.max()
        ra2 = ra1
        if it_ref > 10 and rel < tol:
            break
    q = Q[basis].get().reshape(m // 8, n, 8)
    ref_evec = np.stack([q[j // 8, :, j % 8] for j in range(nev)])
    print(f"GeneralizedInverse maxiter {maxiter} tol {tol}: {it} iterations (reference loop {it_ref})")
    assert it == it_ref
    assert np.array_equal(evec, ref_evec)
    assert np.abs(ev - ra2[:nev]).max() <= 1e-14 * max(1.0, np.abs(ra2).max())
    lu.close()
