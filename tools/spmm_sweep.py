#!/usr/bin/env python3
"""Sweep the window-layout SpMM / fused Chebyshev kernel mappings (EIGMI_MV8_KERNEL = rows | quad |
quad2; grp | grp2; one column block: rows1 | grp1) on the C2 Poisson (7-pt, stencil image) and C5 P1 mass (15-pt, explicit columns) matrices.
Each mapping runs in its own child process (the choice is read once per process).  Prints one
JSON line per (mapping, matrix, op) with the average launch-sequence time and algorithmic GB/s:
  SpMM m columns:  12 nnz + 4 (n+1) + 16 m n        Chebyshev step: 12 nnz + 4 (n+1) + 32 m n + 8 n
(matrix streamed once per 32 / 16 columns for quad / rows+quad2: the formulas count it once)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(kind, N, m):
    sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
    import numpy as np
    import eigmi
    ctx = eigmi.Context(0)
    out = []
    for gen in (eigmi.GEN_POISSON3D, eigmi.GEN_P1MASS3D):
        rp, c, v = eigmi.gen_matrix(gen, N)
        A = eigmi.Matrix.from_bcsr(ctx, rp, c, v)
        n, nnz = N ** 3, int(rp[-1])
        X = ctx.array(np.random.default_rng(0).standard_normal(n * m))
        Y = ctx.zeros(n * m)
        B = ctx.array(np.random.default_rng(1).standard_normal(n * m))
        import ctypes
        for op in ("spmm", "cheb"):
            def run():
                if op == "spmm":
                    eigmi.spmm_mv8(A, m, X, Y)
                else:
                    eigmi.mass_solve_mv8(A, m, 6, B, Y, lmin=0.5, lmax=2.5 if gen == eigmi.GEN_P1MASS3D else 12.0)
            run()
            ctx.sync()
            import time
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                run()
            ctx.sync()
            dt = (time.perf_counter() - t0) / reps
            if op == "spmm":
                per = dt
                b = 12 * nnz + 4 * (n + 1) + 16 * m * n
            else:
                per = dt / 5  # 5 fused steps per solve (degree 6); init / memset folded in
                b = 12 * nnz + 4 * (n + 1) + 32 * m * n + 8 * n
            out.append({"kernel": kind, "matrix": "P1 mass 15pt" if gen == eigmi.GEN_P1MASS3D else "Poisson 7pt",
                        "N": N, "m": m, "op": op, "us": round(per * 1e6, 1), "GBs": round(b / per / 1e9, 1)})
        A.close()
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
        sys.exit(0)
    N = int(os.environ.get("SWEEP_N", "160"))
    # SWEEP_CASES="quad:2048 quad:1024 quad2:4096" -- mapping[:workgroups in flight (EIGMI_MV8_GX)]
    # single-block (m = 8) mappings: rows1 / grp1 (EIGMI_MV8_KERNEL1); SWEEP_M="8 32"
    cases = os.environ.get("SWEEP_CASES", "rows quad quad2").split()
    for m in [int(x) for x in os.environ.get("SWEEP_M", "32").split()]:
        for case in cases:
            kind, _, gx = case.partition(":")
            env = dict(os.environ, EIGMI_MV8_KERNEL=kind)
            k1 = {"rows1": "rows", "grp1": "grp"}.get(kind)
            if k1:
                env["EIGMI_MV8_KERNEL1"] = k1
            if gx:
                env["EIGMI_MV8_GX"] = gx
            r = subprocess.run([sys.executable, __file__, "child", case, str(N), str(m)], env=env, timeout=600)
            if r.returncode != 0:
                sys.exit(r.returncode)
