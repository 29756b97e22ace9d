"""Plane runs per column (eig_mat_tune EIG_TUNE_MARCH_RUNS) for the 8-column SpMM and the SpMM + dots
(+ window Gram) product of StandardLargest on the 3-D Poisson value image (EIG_MAT_NO_UNIFORM), at
128^3 (C2) and 256^3: kernel time per call from back-to-back launches.  One JSON line per point.

    python tools/spmm_runs.py [N ...]        (default 128 256)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import eigmi  # noqa: E402


def timed(ctx, f, reps=20):
    f()
    ctx.sync()
    best = float("inf")
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        ctx.sync()
        best = min(best, (time.perf_counter() - t0) / reps)
    return best


def main():
    Ns = [int(a) for a in sys.argv[1:]] or [128, 256]
    ctx = eigmi.Context(0)
    for N in Ns:
        n = N ** 3
        rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
        M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=eigmi.MAT_NO_UNIFORM)
        del rp, c, v
        m = 8
        Q = ctx.array(np.random.default_rng(1).standard_normal(n * m))
        Y = ctx.zeros(n * m)
        dp, G = ctx.zeros(m), ctx.zeros(64)
        for runs in (0, 1, 2, 3, 4, 8, 16):
            if runs > N:
                continue
            M.tune(march_runs=runs)
            t1 = timed(ctx, lambda: eigmi.spmm_mv8(M, m, Q, Y))
            t2 = timed(ctx, lambda: eigmi.spmm_dot_gram_mv8(M, m, Q, Y, dp, G))
            print(json.dumps({"N": N, "runs": runs, "spmm_us": round(t1 * 1e6, 2), "spmm_dot_gram_us": round(t2 * 1e6, 2),
                              "kernel": M.kernel("spmm8")}), flush=True)
        M.tune(march_runs=0)
        for a in (Q, Y, dp, G):
            a.free()
        M.close()
    ctx.close()


if __name__ == "__main__":
    main()
