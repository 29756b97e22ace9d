"""The mass solve's Chebyshev step of config C5 (variable-coefficient P1 M, eig_gen kind 10, m = 32,
the box kernel k_box_mv32_cheb) per z-segment count of the box kernels (eig_mat_tune
EIG_TUNE_BOX_SEGS; 0 = automatic): the step time as the difference of two solve degrees.

    python tools/cheb_segs.py [N]        (default 256)
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dune-eigensolver_amd"))
import eigmi  # noqa: E402

PEAK = 8000.0


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ctx = eigmi.Context(0)
    n, m = N ** 3, 32
    r, c, v = eigmi.gen_matrix(eigmi.GEN_P1MASS3D_VAR, N)
    M = eigmi.Matrix.from_bcsr(ctx, r, c, v)
    del r, c, v
    X, Y = ctx.zeros(n * m), ctx.zeros(n * m)
    ctx.check(eigmi.lib.eig_fill_normal(ctx.h, n * m, 5, X.ptr))
    for segs in (0, 1, 2, 3, 4, 6, 8, 0):
        M.tune(box_segs=segs)
        res = []
        for d in (6, 16):
            eigmi.mass_solve_mv8(M, m, d, X, Y)
            ctx.sync()
            best = 1e30
            for _ in range(2):
                t = time.perf_counter()
                eigmi.mass_solve_mv8(M, m, d, X, Y)
                ctx.sync()
                best = min(best, time.perf_counter() - t)
            res.append(best)
        tc = (res[1] - res[0]) / 10
        print(json.dumps({"matrix": f"P1 M var {N}^3", "op": "Chebyshev step m=32", "box_segs": segs,
                          "kernel": M.kernel("cheb32"), "us": round(tc * 1e6, 1)}), flush=True)
    X.free(), Y.free()
    M.close()
    ctx.close()


if __name__ == "__main__":
    main()
