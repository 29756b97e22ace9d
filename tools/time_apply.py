#!/usr/bin/env python3
"""Block-inverse solve (eig_inverse_mv8) time per application vs the number of columns m, on the
factors of the GenEO pencil A + shift B at N^2 (the operator the shift-invert drivers apply)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import eigmi  # noqa: E402
import oracle  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ctx = eigmi.Context(0)
shift = 1e-3
An, Bp = oracle.laplace2d(N, "neumann"), oracle.laplace2d(N, "pu", overlap=3)
As = oracle.CSR(An.nrows, An.rowptr, An.col, An.val + shift * Bp.val)
t0 = time.perf_counter()
lu = eigmi.LU.from_bcsr(ctx, As.rowptr, As.col, As.val)
print(f"N={N}: LU.from_bcsr {1e3 * (time.perf_counter() - t0):.1f} ms; solver {lu.solver_info()}")
n = An.nrows
for m in (8, 16, 32, 64):
    X = np.random.default_rng(1).standard_normal(n * m)
    din, dout = ctx.array(X), ctx.zeros(n * m)
    lu.inverse_mv8(m, din, dout)
    ctx.sync()
    best = 1e9
    for _ in range(5):
        din.upload(X)
        ctx.sync()
        t0 = time.perf_counter()
        lu.inverse_mv8(m, din, dout)
        ctx.sync()
        best = min(best, time.perf_counter() - t0)
    print(f"m={m}: {best * 1e3:.3f} ms per application")
