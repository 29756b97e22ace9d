#!/usr/bin/env python3
"""Run-to-run determinism of the inverse-iteration pieces (round 6 diagnostic): the driver twice, the
LU apply and orthonormalize_blocked repeated on the same input -- bitwise or not."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import eigmi  # noqa: E402
import oracle  # noqa: E402

ctx = eigmi.Context(0)
N, shift = 20, 0.2
A = oracle.laplace2d(N)
As = oracle.CSR(A.nrows, A.rowptr, A.col, A.val.copy())
oracle.lib.orc_shift_diag(As.n, As.rowptr, As.col, As.val, shift)
lu = eigmi.LU.from_bcsr(ctx, As.rowptr, As.col, As.val)
print("solver", lu.solver_info())
runs = []
for r in range(3):
    M = eigmi.Matrix.from_bcsr(ctx, A.rowptr, A.col, A.val)
    ev, evec, it = eigmi.standard_inverse(M, shift, 1e-9, 4000, 4, 17, lu=lu)
    runs.append((ev, evec, it))
    M.close()
print("driver runs: iterations", [r[2] for r in runs], "evec bitwise equal",
      [bool(np.array_equal(runs[0][1], r[1])) for r in runs[1:]])
n, m = A.n, 8
X = ctx.array(oracle.random_mv8(n, m, 3))
Y0, Y = ctx.zeros(n * m), ctx.zeros(n * m)
lu.inverse_mv8(m, X, Y0)
ref = Y0.get()
same = 0
for i in range(200):
    lu.inverse_mv8(m, X, Y)
    same += bool(np.array_equal(Y.get(), ref))
print("LU apply bitwise repeats:", same, "/ 200")
Q = ctx.zeros(n * m)
Qh = oracle.random_mv8(n, m, 4)
Q.upload(Qh)
eigmi.orthonormalize_mv8(ctx, n, m, Q)
qref = Q.get()
same = 0
for i in range(200):
    Q.upload(Qh)
    eigmi.orthonormalize_mv8(ctx, n, m, Q)
    same += bool(np.array_equal(Q.get(), qref))
print("orthonormalize bitwise repeats:", same, "/ 200")
