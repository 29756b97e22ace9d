"""Sweep of the box kernels' z segments per tile column (eig_mat_tune EIG_TUNE_BOX_SEGS): SpMM
Y = A X at m = 8 / 32 on the C2 Poisson (128^3) and the P1 stiffness (256^3), and the mass solve's
Chebyshev step at 256^3, per segment count (0 = the automatic choice).  One JSON line per point.
    python tools/box_segs.py [N_poisson] [N_p1]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dune-eigensolver_amd"))
import eigmi  # noqa: E402

PEAK = 8000.0


def main():
    Np = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    Nk = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    ctx = eigmi.Context(0)
    var = os.environ.get("EIGMI_BOXSEG_VAR", "0") == "1"
    cases = ((eigmi.GEN_POISSON3D, Np, (8, 32), "Poisson"), (eigmi.GEN_P1STIFF3D, Nk, (32,), "P1 K"))
    if var:
        # variable coefficients (a random positive diagonal term per row): the box-image kernel
        cases = ((eigmi.GEN_P1STIFF3D, Nk, (32,), "P1 K var"), (eigmi.GEN_P1MASS3D, Nk, (32,), "P1 M var"))
    for kind, N, ms, name in cases:
        n = N ** 3
        r, c, v = eigmi.gen_matrix(kind, N)
        if var:
            import numpy as np
            rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(r))
            diag = np.nonzero(c == rows)[0]
            v[diag] *= 1.0 + 0.01 * np.random.default_rng(1).random(n)
            del rows, diag
        A = eigmi.Matrix.from_bcsr(ctx, r, c, v)
        del r, c, v
        for m in ms:
            X, Y = ctx.zeros(n * m), ctx.zeros(n * m)
            ctx.check(eigmi.lib.eig_fill_normal(ctx.h, n * m, 5, X.ptr))
            for segs in (0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32):
                if segs > N:
                    continue
                A.tune(box_segs=segs)
                reps = 20 if n * m < 1e8 else 10

                def run():
                    for _ in range(reps):
                        eigmi.spmm_mv8(A, m, X, Y)
                    ctx.sync()
                run()
                best = 1e30
                for _ in range(3):
                    t = time.perf_counter()
                    run()
                    best = min(best, (time.perf_counter() - t) / reps)
                by = 16 * m * n
                print(json.dumps({"matrix": f"{name} {N}^3", "op": f"SpMM m={m}", "box_segs": segs,
                                  "kernel": A.kernel("spmm32"), "us": round(best * 1e6, 1),
                                  "frac": round(by / best / 1e9 / PEAK, 4)}), flush=True)
            A.tune(box_segs=0)
            X.free(), Y.free()
        A.close()
    if var:
        return
    # Chebyshev step of the mass solve, 256^3, m = 32 (difference of two solve degrees)
    N = Nk
    n, m = N ** 3, 32
    r, c, v = eigmi.gen_matrix(eigmi.GEN_P1MASS3D, N)
    M = eigmi.Matrix.from_bcsr(ctx, r, c, v)
    del r, c, v
    X, Y = ctx.zeros(n * m), ctx.zeros(n * m)
    ctx.check(eigmi.lib.eig_fill_normal(ctx.h, n * m, 5, X.ptr))
    for segs in (0, 1, 2, 4, 8, 16, 0):
        M.tune(box_segs=segs)
        res = []
        for d in (12, 32):
            eigmi.mass_solve_mv8(M, m, d, X, Y)
            ctx.sync()
            best = 1e30
            for _ in range(3):
                t = time.perf_counter()
                eigmi.mass_solve_mv8(M, m, d, X, Y)
                ctx.sync()
                best = min(best, time.perf_counter() - t)
            res.append(best)
        tc = (res[1] - res[0]) / 20
        print(json.dumps({"matrix": f"P1 M {N}^3", "op": "Chebyshev step m=32", "box_segs": segs,
                          "kernel": M.kernel("cheb32"), "us": round(tc * 1e6, 1),
                          "frac": round(32 * m * n / tc / 1e9 / PEAK, 4)}), flush=True)
    X.free(), Y.free()
    M.close()


if __name__ == "__main__":
    main()
