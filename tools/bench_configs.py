#!/usr/bin/env python3
"""Per-configuration measurements beside bench.py's headline line (BASELINE.json configs):

  C1  2-D Poisson 64x64: StandardLargest (ini defaults) and the Lanczos solver on the GPU, the
      oracle (reference CPU path) timed on the same inputs
  C2  3-D Poisson 128^3: SpMV (cache-resident: 217 MB < 256 MB MALL), Lanczos step, the b = 8
      SpMM, block Gram-Schmidt (m = 8, 32) and one StandardLargest iteration vs the CPU path
  C3  3-D Q1 elasticity 64^3, 3x3 blocks: BCSR SpMV against 76 nnzb + 4 (nb+1) + 48 nb bytes
  INV inverse iteration with exported LU factors on the harness matrices:
      matmul_inverse_tallskinny_blocked (m = 8), StandardInverse, GeneralizedInverse (GenEO pencil)
      and computeGenSymShiftInvertMinMagnitude, GPU vs the oracle / scipy ARPACK on the host
  C5  generalised K x = lambda M x, P1 on the Kuhn split (15-pt shared pattern), block Lanczos
      k = 32: block steps/s with the phase split, the fused Chebyshev SpMM kernel against
      12 nnz + 4 (n+1) + (32 m + 8) n bytes per m-column launch (EIGMI_C5_N, default 256)

One JSON line per measurement; algorithmic bytes per SURVEY 8(d); peak 8 TB/s.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import eigmi  # noqa: E402
import oracle  # noqa: E402  (CPU baseline only)

PEAK = 8000.0


def emit(**kw):
    print(json.dumps(kw), flush=True)


def wall(f, reps=1):
    t0 = time.perf_counter()
    for _ in range(reps):
        r = f()
    return (time.perf_counter() - t0) / reps, r


def c1(ctx):
    A = oracle.laplace2d(64)
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    eigmi.standard_largest(M, 0.0, 2e-3, 4000, 4, 123, want_evec=False)  # warm-up
    tg, (ev, _, it) = wall(lambda: eigmi.standard_largest(M, 0.0, 2e-3, 4000, 4, 123, want_evec=False), 3)
    tc, (rev, _, rit) = wall(lambda: oracle.standard_largest(A, 0.0, 2e-3, 4000, 4, 123), 3)
    emit(config="C1 2D Poisson 64^2", op="StandardLargest nev=4 tol=2e-3 seed=123", gpu_s=round(tg, 5),
         cpu_s=round(tc, 5), iterations=it, cpu_iterations=rit, ritz0=ev[0], max_abs_diff_vs_cpu=float(np.abs(ev - rev).max()))
    tl, (ev, _, res) = wall(lambda: eigmi.lanczos_solve(M, 4, 300, eigmi.WHICH_LA, want_evec=False))
    emit(config="C1 2D Poisson 64^2", op="Lanczos solve LA nev=4 ncv=300 (full re-orth)", gpu_s=round(tl, 5),
         eigenvalues=list(ev), max_residual=float(res.max()))


def c2(ctx):
    """Config C2 (3-D Poisson 128^3).  The band values are read from HBM (EIG_MAT_NO_UNIFORM, as the
    benchmark's image) unless EIGMI_C2_UNIFORM=1 (the constant-coefficient shortcut)."""
    N = 128
    n = N ** 3
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
    nnz = int(rp[-1])
    uni = os.environ.get("EIGMI_C2_UNIFORM", "0") == "1"
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=0 if uni else eigmi.MAT_NO_UNIFORM)
    image = "stencil-only (values in the kernel arguments)" if uni else "value-streaming (band values read)"

    def emit(**kw):  # every C2 line names its image
        globals()["emit"](image=image, **kw)
    x = ctx.array(np.random.default_rng(0).standard_normal(n))
    y = ctx.zeros(n)
    M.mv_timed(x, y, 10)
    ms = M.mv_timed(x, y, 200)
    # algorithmic bytes of the image the kernel streams (band image: 8 B per band slot + the row
    # mask), the survey's CSR count beside it
    b = eigmi.image_bytes(M, "spmv")
    csr = eigmi.bytes_spmv(n, nnz)
    gbs = b / (ms * 1e-3) / 1e9
    A = oracle.CSR(n, rp, c, v)
    xh = x.get()
    tc, _ = wall(lambda: oracle.csr_mv(A, xh), 3)
    emit(config="C2 3D Poisson 128^3", op=f"SpMV (cache-resident: {b / 2**20:.0f} MiB < 256 MiB MALL)",
         us=round(ms * 1e3, 2), algorithmic_bytes=b, GBs=round(gbs, 1), frac=round(gbs / PEAK, 4),
         csr_bytes=csr, csr_equiv_GBs=round(csr / (ms * 1e-3) / 1e9, 1), cpu_us=round(tc * 1e6, 1),
         cpu_GBs=round(csr / tc / 1e9, 2))
    ws = eigmi.LanczosWorkspace(M, 210, seed=123)
    ws.step(10)
    t = ws.step(200, timed="detail")
    k1_name, k1_bytes = M.lanczos_kernel_info(False)
    emit(config="C2 3D Poisson 128^3", op="Lanczos step (classic: K1 + update)",
         it_per_s=round(200 / (t.total_ms * 1e-3), 1), k1=k1_name,
         k1_us=round(t.spmv_ms / 200 * 1e3, 2), k2_us=round(t.update_ms / 200 * 1e3, 2),
         step_frac=round((k1_bytes + 24 * n) / (t.total_ms / 200 * 1e-3) / 1e9 / PEAK, 4))
    ws.close()
    ws = eigmi.LanczosWorkspace(M, 210, seed=123, fused=True)
    ws.step(10)
    t = ws.step(200, timed=True)
    kf_name, kf_bytes = M.lanczos_kernel_info(True)
    emit(config="C2 3D Poisson 128^3", op="Lanczos step (fused, bench default)",
         it_per_s=round(200 / (t.total_ms * 1e-3), 1), kernel=kf_name, kernel_us=round(t.spmv_ms / 200 * 1e3, 2),
         kernel_frac=round(kf_bytes / (t.spmv_ms / 200 * 1e-3) / 1e9 / PEAK, 4))
    ws.close()
    for m in (8, 32):
        Qh = oracle.random_mv8(n, m, 1)
        Q, Y = ctx.array(Qh), ctx.zeros(n * m)
        eigmi.spmm_mv8(M, m, Q, Y)
        ctx.sync()

        def spmm_batch(reps=20):
            # kernel throughput: back-to-back launches, one synchronisation (a synchronisation per call
            # adds ~12 us of host round trip to a 47 us kernel)
            t0 = time.perf_counter()
            for _ in range(reps):
                eigmi.spmm_mv8(M, m, Q, Y)
            ctx.sync()
            return (time.perf_counter() - t0) / reps
        tg = min(spmm_batch() for _ in range(3))
        sb = eigmi.image_bytes(M, "spmm", m)
        emit(config="C2 3D Poisson 128^3", op=f"SpMM b=8 m={m}", us=round(tg * 1e6, 1), algorithmic_bytes=sb,
             GBs=round(sb / tg / 1e9, 1), frac=round(sb / tg / 1e9 / PEAK, 4),
             csr_equiv_GBs=round((12 * nnz + 4 * (n + 1) + 128 * n * (m // 8)) / tg / 1e9, 1))
        Q.upload(Qh)
        eigmi.orthonormalize_mv8(ctx, n, m, Q)
        ctx.sync()

        def ortho():
            Q.upload(Qh)
            ctx.sync()
            t0 = time.perf_counter()
            eigmi.orthonormalize_mv8(ctx, n, m, Q)
            ctx.sync()
            return time.perf_counter() - t0
        tg = min(ortho() for _ in range(3))
        tc, _ = wall(lambda: oracle.orthonormalize_mv8(Qh, n, m))
        ob = eigmi.lib.eig_bytes_orthonormalize_blocked(n, m, 8)
        of = eigmi.lib.eig_flops_orthonormalize(n, m)
        emit(config="C2 3D Poisson 128^3", op=f"orthonormalize_blocked (MGS) m={m}", gpu_ms=round(tg * 1e3, 3),
             cpu_ms=round(tc * 1e3, 1), model_bytes=ob, model_GBs=round(ob / tg / 1e9, 1),
             model_GFLOPs=round(of / tg / 1e9, 1), speedup=round(tc / tg, 1))
    # one StandardLargest iteration at m = 8, timed as the driver runs it (eigensolver.hh:78-96 with
    # the :78 product reused from the previous iteration's :84, SURVEY Appendix A.6: orthonormalize_blocked,
    # ONE SpMM, diagonal dots copied to the host for the stopping test) and in the reference's order
    # (two SpMMs); differencing whole solves of different lengths drowned the 10-iteration difference
    # in the host generation of the random start block
    m = 8
    Q1, Q2, dp = ctx.array(oracle.random_mv8(n, m, 1)), ctx.zeros(n * m), ctx.zeros(m)
    eigmi.orthonormalize_mv8(ctx, n, m, Q1)

    def iteration_two_spmm():
        eigmi.spmm_mv8(M, m, Q1, Q2)
        eigmi.orthonormalize_mv8(ctx, n, m, Q2)
        eigmi.spmm_mv8(M, m, Q2, Q1)
        eigmi.dot_diag_mv8(ctx, n, m, Q2, Q1, dp)
        dp.get()
    iteration_two_spmm()
    ctx.sync()
    tg2, _ = wall(iteration_two_spmm, 20)
    state = [Q1, Q2]
    eigmi.spmm_mv8(M, m, Q1, Q2)

    def iteration():
        q1, q2 = state  # q2 = A q1 (the previous iteration's second product)
        eigmi.orthonormalize_mv8(ctx, n, m, q2)
        eigmi.spmm_mv8(M, m, q2, q1)
        eigmi.dot_diag_mv8(ctx, n, m, q2, q1, dp)
        dp.get()
        state.reverse()  # the swap: Q1 <- the orthonormal block, Q2 <- its product
    iteration()
    ctx.sync()
    tg, _ = wall(iteration, 20)
    # the driver itself (one-iteration look-ahead, no host round trip between iterations): the
    # difference of 212- and 12-iteration solves (tol 0 runs to maxiter), best of 3 each
    k0, k1 = 12, 212
    ta = min(wall(lambda: eigmi.standard_largest(M, 0.0, 0.0, k0, 8, 123, want_evec=False))[0] for _ in range(3))
    tb = min(wall(lambda: eigmi.standard_largest(M, 0.0, 0.0, k1, 8, 123, want_evec=False))[0] for _ in range(3))
    td = (tb - ta) / (k1 - k0)
    tc1, _ = wall(lambda: oracle.standard_largest(A, 0.0, 0.0, 2, 8, 123))
    tc2, _ = wall(lambda: oracle.standard_largest(A, 0.0, 0.0, 3, 8, 123))
    emit(config="C2 3D Poisson 128^3", op="StandardLargest iteration m=8", gpu_ms_per_iter=round(td * 1e3, 3),
         gpu_ms_per_iter_synced=round(tg * 1e3, 3), gpu_ms_per_iter_two_spmm_synced=round(tg2 * 1e3, 3),
         cpu_ms_per_iter=round((tc2 - tc1) * 1e3, 1), speedup=round((tc2 - tc1) / td, 1),
         note="gpu_ms_per_iter: the driver (one SpMM per iteration, look-ahead); *_synced: python loops of "
              "the same primitives with a host round trip per iteration, with one or with the reference's two SpMMs; "
              "the CPU restatement runs the reference's two")


def gram(ctx):
    """a6 panel Gram G = Q1^T Q2 (k_gram_mv8) and a9 orthonormalize_blocked at C2 size (n = 128^3):
    per call, 50 back-to-back calls between two synchronisations; algorithmic bytes 8 n (m1 + m2)."""
    n = int(os.environ.get("EIGMI_GRAM_N", str(128 ** 3)))
    reps = 50
    for m1, m2 in ((8, 8), (8, 16), (8, 24), (32, 32)):
        Q1, Q2, G = ctx.array(oracle.random_mv8(n, m1, 1)), ctx.array(oracle.random_mv8(n, m2, 2)), ctx.zeros(m1 * m2)
        eigmi.gram_mv8(ctx, n, m1, m2, Q1, Q2, G)
        ctx.sync()
        def batch():
            t0 = time.perf_counter()
            for _ in range(reps):
                eigmi.gram_mv8(ctx, n, m1, m2, Q1, Q2, G)
            ctx.sync()
            return (time.perf_counter() - t0) / reps
        tg = min(batch() for _ in range(3))
        b = 8 * n * (m1 + m2)
        emit(config=f"gram n={n}", op=f"gram_mv8 m1={m1} m2={m2}", us=round(tg * 1e6, 2), algorithmic_bytes=b,
             GBs=round(b / tg / 1e9, 1), frac=round(b / tg / 1e9 / PEAK, 4))
        Q1.free(), Q2.free(), G.free()
    # block Lanczos panel products at C5 size (n = 256^3, eig_panel_gram_mv8: V^T (M Z) of CGS, k = 32)
    nc5 = int(os.environ.get("EIGMI_GRAM_N5", str(256 ** 3)))
    for m1, m2 in ((32, 32), (96, 32), (256, 32)):
        Q1, Q2, G = ctx.zeros(nc5 * m1), ctx.zeros(nc5 * m2), ctx.zeros(m1 * m2)
        # (timing only: a constant byte pattern, 0x3F3F... = 4.8e-4 per entry, instead of host random numbers)
        eigmi.lib.eig_memset(ctx.h, Q1.ptr, 0x3F, nc5 * m1 * 8)
        eigmi.lib.eig_memset(ctx.h, Q2.ptr, 0x3F, nc5 * m2 * 8)
        eigmi.panel_gram_mv8(ctx, nc5, m1, m2, Q1, Q2, G)
        ctx.sync()

        def batch5():
            t0 = time.perf_counter()
            for _ in range(5):
                eigmi.panel_gram_mv8(ctx, nc5, m1, m2, Q1, Q2, G)
            ctx.sync()
            return (time.perf_counter() - t0) / 5
        tg = min(batch5() for _ in range(3))
        b = 8 * nc5 * (m1 + m2)
        emit(config=f"panel gram n={nc5}", op=f"panel_gram_mv8 m1={m1} m2={m2}", us=round(tg * 1e6, 2),
             algorithmic_bytes=b, GBs=round(b / tg / 1e9, 1), frac=round(b / tg / 1e9 / PEAK, 4))
        Q1.free(), Q2.free(), G.free()
    for m in (8, 32):
        Qh = oracle.random_mv8(n, m, 1)
        Q = ctx.array(Qh)

        def ortho():
            Q.upload(Qh)
            ctx.sync()
            t0 = time.perf_counter()
            eigmi.orthonormalize_mv8(ctx, n, m, Q)
            ctx.sync()
            return time.perf_counter() - t0
        ortho()
        tg = min(ortho() for _ in range(5))
        ob = eigmi.lib.eig_bytes_orthonormalize_blocked(n, m, 8)
        emit(config=f"gram n={n}", op=f"orthonormalize_blocked (MGS) m={m}", gpu_ms=round(tg * 1e3, 3),
             model_bytes=ob, model_GBs=round(ob / tg / 1e9, 1))
        Q.free()


def ortho(ctx):
    """a9 orthonormalize_blocked at C2 size (n = 128^3), m = 8 / 32, best of 5 calls, against the
    reference's byte model (kernels_cpp.hh:157-175): the Gram look-ahead MGS with windows L = 8, 4, 2
    (EIG_ORTHO_LOOKAHEAD; read passes reported) and the stepwise replay (L = 1; EIGMI_MGS_INPLACE=1
    times the in-place passes there)."""
    n = 128 ** 3
    step_tag = ("in-place passes" if os.environ.get("EIGMI_MGS_INPLACE") else
                "one cooperative launch, grid barriers" if os.environ.get("EIGMI_MGS_COOP") else
                f"read-only replay passes, grid <= {os.environ.get('EIGMI_MGS_GRID', '512')}")
    for m in (8, 32):
        Qh = oracle.random_mv8(n, m, 1)
        Q = ctx.array(Qh)
        for L in (8, 4, 2, 1):
            var = eigmi.ORTHO_MGS | eigmi.ORTHO_LOOKAHEAD(L)

            def once():
                Q.upload(Qh)
                ctx.sync()
                t0 = time.perf_counter()
                eigmi.orthonormalize_mv8(ctx, n, m, Q, var)
                ctx.sync()
                return time.perf_counter() - t0
            once()
            tg = min(once() for _ in range(5))
            passes = eigmi.orthonormalize_passes(ctx) if L > 1 else 8
            tag = f"Gram look-ahead L={L}, {passes} read passes" if L > 1 else step_tag
            ob = eigmi.lib.eig_bytes_orthonormalize_blocked(n, m, 8)
            emit(config="C2 128^3", op=f"orthonormalize_blocked (MGS, {tag}) m={m}", gpu_ms=round(tg * 1e3, 4),
                 model_bytes=ob, model_GBs=round(ob / tg / 1e9, 1), model_frac=round(ob / tg / 1e9 / PEAK, 4))
        Q.free()


def c3(ctx):
    N = 64
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_Q1ELAST3D, N)
    nb = N ** 3
    nnzb = int(rp[-1])
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, 3, 3)
    x = ctx.array(np.random.default_rng(0).standard_normal(3 * nb))
    y = ctx.zeros(3 * nb)
    M.mv_timed(x, y, 5)
    ms = M.mv_timed(x, y, 100)
    b = 76 * nnzb + 4 * (nb + 1) + 48 * nb
    gbs = b / (ms * 1e-3) / 1e9
    A = oracle.CSR(nb, rp, c, v, 3, 3)
    xh = x.get()
    tc, _ = wall(lambda: oracle.csr_mv(A, xh))
    emit(config="C3 Q1 elasticity 64^3 3x3 BCSR", op="BCSR SpMV", us=round(ms * 1e3, 2), nnzb=nnzb,
         algorithmic_bytes=b, GBs=round(gbs, 1), frac=round(gbs / PEAK, 4), cpu_us=round(tc * 1e6, 1),
         cpu_GBs=round(b / tc / 1e9, 2))


def inv(ctx):
    import scipy.sparse.linalg as ssl
    N = int(os.environ.get("EIGMI_INV_N", "64"))
    A = oracle.laplace2d(N)
    n = A.n
    lu = eigmi.LU.from_bcsr(ctx, A.rowptr, A.col, A.val)
    f = oracle.LU(**lu.export())
    lnz, unz = f.Lp[-1], f.Up[-1]
    X = oracle.random_mv8(n, 8, 1)
    din, dout = ctx.array(X), ctx.zeros(n * 8)
    lu.inverse_mv8(8, din, dout)
    ctx.sync()
    reps = 20
    tg, _ = wall(lambda: (lu.inverse_mv8(8, din, dout), ctx.sync()), reps)
    tc, _ = wall(lambda: oracle.inverse_mv8(f, X, 8), 3)
    emit(config=f"INV 2D Dirichlet {N}^2", op="matmul_inverse_tallskinny_blocked m=8 (RCM envelope factors)",
         lnz=int(lnz), unz=int(unz), gpu_us=round(tg * 1e6, 1), cpu_us=round(tc * 1e6, 1), speedup=round(tc / tg, 2),
         note="triangular solves are a row dependency chain: latency-bound, no bandwidth roofline")
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    eigmi.standard_inverse(M, 0.0, 1e-10, 2000, 8, 123, want_evec=False)
    tg, (ev, _, it) = wall(lambda: eigmi.standard_inverse(M, 0.0, 1e-10, 2000, 8, 123, want_evec=False))
    tc, (rev, _, rit) = wall(lambda: oracle.standard_inverse(A, f, 0.0, 1e-10, 2000, 8, 123))
    emit(config=f"INV 2D Dirichlet {N}^2", op="StandardInverse nev=8 tol=1e-10", gpu_s=round(tg, 4), cpu_s=round(tc, 4),
         iterations=it, cpu_iterations=rit, speedup=round(tc / tg, 2), max_rel_diff=float(np.max(np.abs(ev - rev) / np.abs(rev))),
         note="gpu_s includes the factorization (host RCM + device band LU + block-inverse image); cpu_s is the "
              "iteration with the factors given")
    # the same driver with the factors given on both sides (eigensolver.hh:156 factors inside the
    # driver; the factorisation is host work on both sides, so this row times the iteration alone)
    eigmi.standard_inverse(M, 0.0, 1e-10, 2000, 8, 123, lu=lu, want_evec=False)
    tg, (ev, _, it) = wall(lambda: eigmi.standard_inverse(M, 0.0, 1e-10, 2000, 8, 123, lu=lu, want_evec=False), 3)
    emit(config=f"INV 2D Dirichlet {N}^2", op="StandardInverse nev=8 tol=1e-10, factors given", gpu_s=round(tg, 4),
         cpu_s=round(tc, 4), iterations=it, cpu_iterations=rit, speedup=round(tc / tg, 2),
         max_rel_diff=float(np.max(np.abs(ev - rev) / np.abs(rev))))
    shift, reg = 1e-3, 0.0
    An, Bp = oracle.laplace2d(N, "neumann"), oracle.laplace2d(N, "pu", overlap=3)
    dA = eigmi.Matrix.from_bcsr(ctx, An.rowptr, An.col, An.val)
    dB = eigmi.Matrix.from_bcsr(ctx, Bp.rowptr, Bp.col, Bp.val)
    tg, (ev, _, it) = wall(lambda: eigmi.generalized_inverse(dA, dB, shift, reg, 1e-8, 4000, 8, 123, want_evec=False))
    As = oracle.CSR(An.nrows, An.rowptr, An.col, An.val + shift * Bp.val)
    fs = oracle.LU(**eigmi.LU.from_bcsr(None, As.rowptr, As.col, As.val).export())
    tc, (rev, _, rit) = wall(lambda: oracle.generalized_inverse(An, Bp, fs, shift, reg, 1e-8, 4000, 8, 123))
    emit(config=f"INV GenEO pencil {N}^2 (.cc:455-512)", op="GeneralizedInverse nev=8 tol=1e-8", gpu_s=round(tg, 4),
         cpu_s=round(tc, 4), iterations=it, cpu_iterations=rit, speedup=round(tc / tg, 2),
         note="gpu_s includes the shifted copy and the factorization (device band LU); cpu_s is the iteration with "
              "the factors given")
    lus = eigmi.LU.from_bcsr(ctx, As.rowptr, As.col, As.val)
    eigmi.generalized_inverse(dA, dB, shift, reg, 1e-8, 4000, 8, 123, lu=lus, want_evec=False)
    tg, (ev, _, it) = wall(lambda: eigmi.generalized_inverse(dA, dB, shift, reg, 1e-8, 4000, 8, 123, lu=lus,
                                                             want_evec=False), 3)
    emit(config=f"INV GenEO pencil {N}^2 (.cc:455-512)", op="GeneralizedInverse nev=8 tol=1e-8, factors given",
         gpu_s=round(tg, 4), cpu_s=round(tc, 4), iterations=it, cpu_iterations=rit, speedup=round(tc / tg, 2),
         max_diff_rel_to_largest=float(np.max(np.abs(ev - rev)) / np.max(np.abs(rev))))  # (the pencil has lambda = 0)
    As_, Bs_ = An.to_scipy(), Bp.to_scipy()
    tc, w = wall(lambda: ssl.eigsh(As_, k=8, M=Bs_, sigma=-shift, which="LM", tol=1e-10, return_eigenvectors=False))
    for method in ("block", "single"):
        tg, (ev, _, r) = wall(lambda: eigmi.shift_invert_solve(dA, 8, sigma=-shift, B=dB, tol=1e-10, want_evec=False,
                                                               method=method))
        emit(config=f"INV GenEO pencil {N}^2 (.cc:455-512)", op="computeGenSymShiftInvertMinMagnitude nev=8 tol=1e-10",
             method=method, gpu_s=round(tg, 4), scipy_arpack_cpu_s=round(tc, 4), restarts=r, speedup=round(tc / tg, 2),
             max_abs_diff_vs_arpack=float(np.max(np.abs(np.sort(ev) - np.sort(w)))),
             note="both sides include the factorisation (here: host RCM + device band LU + block-inverse image; "
                  "scipy: SuperLU)")


def c5_var():
    """EIGMI_C5_VAR=1: the variable-coefficient P1 K / M (eig_gen kinds 9 / 10, a coefficient per
    tetrahedron) uploaded with EIG_MAT_NO_CLASS -- every launch streams its box image."""
    return os.environ.get("EIGMI_C5_VAR", "0") == "1"


def c5_mats(ctx, N):
    var = c5_var()
    fl = eigmi.MAT_NO_CLASS if var else 0
    rk, ck, vk = eigmi.gen_matrix(eigmi.GEN_P1STIFF3D_VAR if var else eigmi.GEN_P1STIFF3D, N)
    K = eigmi.Matrix.from_bcsr(ctx, rk, ck, vk, flags=fl)
    del rk, ck, vk
    rm, cm, vm = eigmi.gen_matrix(eigmi.GEN_P1MASS3D_VAR if var else eigmi.GEN_P1MASS3D, N)
    nnz = int(rm[-1])
    M = eigmi.Matrix.from_bcsr(ctx, rm, cm, vm, flags=fl)
    return K, M, nnz


def c5(ctx):
    N = int(os.environ.get("EIGMI_C5_N", "256"))
    steps, warm, b, degree = 3, 1, 32, 36
    n = N ** 3
    t0 = time.perf_counter()
    K, M, nnz = c5_mats(ctx, N)
    bl = eigmi.BlockLanczos(K, M, block=b, max_steps=steps + warm, degree=degree, seed=123)
    setup_s = time.perf_counter() - t0
    bl.step(warm)
    t = bl.step(steps)
    ev, _, res = bl.ritz(4, eigmi.WHICH_LA, want_resid=False)
    cols = b // (t.cheb_launches // (steps * (degree - 1)))  # columns per launch
    # per launch, SURVEY 8(d) CSR count: matrix + (gather x_k, read x_{k-1}, read b, write x_{k+1}) per
    # column + dinv; and the bytes of the image the launch streams: the row-class kernel reads no
    # matrix data (class table in LDS, 1 / a_rr included), the box-image kernel one array per offset
    csr_bytes = 12 * nnz + 4 * (n + 1) + 32 * cols * n + 8 * n
    kname = M.kernel("cheb32")
    info = M.info
    if kname == "k_boxc_mv8_cheb":
        cheb_bytes = 32 * cols * n
    elif kname == "k_box_mv32_cheb":
        cheb_bytes = (8 * (2 * info.sym_arrays - 1) + info.sym_mask_bytes + 8) * n + 32 * cols * n
    else:
        cheb_bytes = csr_bytes
    cheb_us = t.cheb_ms / t.cheb_launches * 1e3
    emit(config=f"C5 P1 Kuhn K/M {N}^3, block Lanczos k={b}" + (" (variable coefficients, box image)" if c5_var() else ""),
         op=f"block step (Chebyshev degree {degree}, CGS2, CholQR2)",
         block_steps_per_s=round(steps / (t.total_ms * 1e-3), 3), ms_per_step=round(t.total_ms / steps, 2),
         kspmm_ms=round(t.kspmm_ms / steps, 2), cheb_ms=round(t.cheb_ms / steps, 2),
         orth_ms=round(t.orth_ms / steps, 2), norm_ms=round(t.norm_ms / steps, 2),
         cheb_kernel=kname, cheb_kernel_us=round(cheb_us, 1), cheb_bytes_per_launch=cheb_bytes,
         cheb_GBs=round(cheb_bytes / (cheb_us * 1e-6) / 1e9, 1),
         cheb_frac=round(cheb_bytes / (cheb_us * 1e-6) / 1e9 / PEAK, 4),
         cheb_csr_bytes=csr_bytes, cheb_csr_equiv_GBs=round(csr_bytes / (cheb_us * 1e-6) / 1e9, 1),
         nnz=nnz, setup_s=round(setup_s, 1),
         top_ritz=[float(x) for x in ev], steps_taken=steps + warm)
    bl.close()


def boxk(ctx):
    """Row-class box kernels alone at 256^3, m = 32 (the C5 / multigrid fine-level launches): the
    SpMM Y = K X (k_boxc_mv8<kBoxStore>, 2 vector streams = 16 m n bytes) and the mass solve's
    Chebyshev step (kBoxCheb, 4 streams = 32 m n bytes) from the difference of two solve degrees."""
    N = int(os.environ.get("EIGMI_C5_N", "256"))
    var = os.environ.get("EIGMI_BOXK_VAR", "0") == "1"
    b, n, reps = 32, N ** 3, 20

    def load(kind):
        # variable coefficients: a coefficient per tetrahedron (eig_gen kinds 9 / 10; the rows leave
        # their geometric class, so the box-image kernel runs; the pattern stays the same)
        r, c, v = eigmi.gen_matrix(kind, N)
        return eigmi.Matrix.from_bcsr(ctx, r, c, v, flags=eigmi.MAT_NO_CLASS if var else 0)
    K = load(eigmi.GEN_P1STIFF3D_VAR if var else eigmi.GEN_P1STIFF3D)
    M = load(eigmi.GEN_P1MASS3D_VAR if var else eigmi.GEN_P1MASS3D)
    X, Y = ctx.zeros(n * b), ctx.zeros(n * b)
    ctx.check(eigmi.lib.eig_fill_normal(ctx.h, n * b, 5, X.ptr))
    # box-image kernels (EIG_TUNE_BOX_COLS): 32 = k_box_mv32, 16 = k_box_mv16p (EIGMI_BOX_COLS list)
    # (a value 33 = 32 columns with the XCD-contiguous tile map, EIG_TUNE_BOX_MAP)
    cols_list = [int(c) for c in os.environ.get("EIGMI_BOX_COLS", "0").split(",")]
    tag = f"{N}^3 m={b}" + (" (variable coefficients)" if var else "")
    for cols in cols_list:
        K.tune(box_cols=min(cols, 32), box_map=int(cols == 33))
        M.tune(box_cols=min(cols, 32), box_map=int(cols == 33))
        eigmi.spmm_mv8(K, b, X, Y)
        ctx.sync()

        def spmm():
            for _ in range(reps):
                eigmi.spmm_mv8(K, b, X, Y)
            ctx.sync()
        ts, _ = wall(spmm)
        ts /= reps
        emit(config=f"P1 K {tag}", op="SpMM (kBoxStore)", kernel=K.kernel("spmm32"), box_map=int(cols == 33), us=round(ts * 1e6, 1),
             bytes=16 * b * n, frac=round(16 * b * n / ts / 1e9 / PEAK, 4))
        d0, d1 = 2, 22
        eigmi.mass_solve_mv8(M, b, d0, X, Y)
        ctx.sync()
        t0, _ = wall(lambda: (eigmi.mass_solve_mv8(M, b, d0, X, Y), ctx.sync()), 5)
        t1, _ = wall(lambda: (eigmi.mass_solve_mv8(M, b, d1, X, Y), ctx.sync()), 5)
        tc = (t1 - t0) / (d1 - d0)
        # vectors only for the row-class kernels; the box image adds its nd value arrays (+ D^-1 for
        # the Chebyshev step) per row
        img_s = 0 if K.kernel("spmm32") == "k_boxc_mv8" else 15 * 8 * n
        img_c = 0 if M.kernel("cheb32") == "k_boxc_mv8_cheb" else 15 * 8 * n + 8 * n
        emit(config=f"P1 K {tag}", op="SpMM bytes incl. image", kernel=K.kernel("spmm32"),
             bytes=16 * b * n + img_s, frac=round((16 * b * n + img_s) / ts / 1e9 / PEAK, 4))
        emit(config=f"P1 M {tag}", op="Chebyshev step (kBoxCheb)", kernel=M.kernel("cheb32"), box_map=int(cols == 33), us=round(tc * 1e6, 1),
             bytes=32 * b * n + img_c, frac=round((32 * b * n + img_c) / tc / 1e9 / PEAK, 4))
    X.free(), Y.free()
    K.close(), M.close()


def c5si(ctx):
    """C5 at the end GeneralizedInverse returns (eigensolver.hh:204-351): the smallest eigenvalues
    of the P1 pencil by block Lanczos on K^-1 M (sigma = 0) with the K solve by multigrid
    (eig_blanczos_create_si_mg).  The iteration count is picked at setup so that the solve's
    residual is <= 1e-12 on a random block; the line reports setup, the solve and the block step."""
    N = int(os.environ.get("EIGMI_C5_N", "256"))
    steps, warm, b = 2, 1, 32
    n = N ** 3
    t0 = time.perf_counter()
    K, M, _ = c5_mats(ctx, N)
    t1 = time.perf_counter()
    mg = eigmi.Multigrid(K, (N, N, N), max_cols=b, smooth_degree=2, smooth_ratio=5.0)
    mg_setup = time.perf_counter() - t1
    B, X = ctx.zeros(n * b), ctx.zeros(n * b)
    ctx.check(eigmi.lib.eig_fill_normal(ctx.h, n * b, 7, B.ptr))
    hist = {}
    cycles = None
    for c in (4, 8, 12, 14, 16, 18, 20):
        t2 = time.perf_counter()
        hist[c] = mg.solve(b, B, X, c, resid=True)
        hist[f"{c}_s"] = round(time.perf_counter() - t2, 4)
        if hist[c] <= 1e-12:
            cycles = c
            break
    cycles = cycles or 20
    B.free(), X.free()
    bl = eigmi.BlockLanczos(K, M, block=b, max_steps=steps + warm, Ks=K, sigma=0.0, mg=mg, cycles=cycles, seed=123)
    setup_s = time.perf_counter() - t0
    bl.step(warm)
    t = bl.step(steps)
    ev, _, _ = bl.ritz(4, eigmi.WHICH_SA, want_resid=False)
    h = 1.0 / (N + 1)
    emit(config=f"C5 P1 Kuhn K/M {N}^3, block Lanczos k={b}, smallest end (K^-1 M, multigrid K solve)" +
         (" (variable coefficients, box image)" if c5_var() else ""),
         op="block step (multigrid solve, CGS2, CholQR2)", block_steps_per_s=round(steps / (t.total_ms * 1e-3), 3),
         ms_per_step=round(t.total_ms / steps, 2), solve_ms=round(t.cheb_ms / steps, 2),
         kspmm_ms=round(t.kspmm_ms / steps, 2), orth_ms=round(t.orth_ms / steps, 2), norm_ms=round(t.norm_ms / steps, 2),
         mg=mg.info(), mg_setup_s=round(mg_setup, 2), cycles=cycles, solve_resid_history=hist,
         setup_s=round(setup_s, 1), smallest_ritz=[float(x) for x in ev], steps_taken=steps + warm,
         note=f"Ritz values after {steps + warm} block steps (Krylov dim {(steps + warm) * b}); the continuum "
              f"lowest eigenvalue of -Laplace on the unit cube is 3 pi^2 = {3 * np.pi ** 2:.4f} (h = {h:.5f})")
    bl.close()
    mg.close()


if __name__ == "__main__":
    ctx = eigmi.Context(0)
    which = sys.argv[1:] or ["c1", "c2", "c3", "inv"]
    for w in which:
        globals()[w](ctx)
