#!/usr/bin/env python3
"""Kernel-level profile target for the shift-invert driver (computeGenSymShiftInvertMinMagnitude,
block method) on the GenEO pencil at N^2: run under `rocprofv3 --kernel-trace --stats`.
    python3 tools/si_profile.py 200"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import eigmi  # noqa: E402
import oracle  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ctx = eigmi.Context(0)
shift = 1e-3
An, Bp = oracle.laplace2d(N, "neumann"), oracle.laplace2d(N, "pu", overlap=3)
dA = eigmi.Matrix.from_bcsr(ctx, An.rowptr, An.col, An.val)
dB = eigmi.Matrix.from_bcsr(ctx, Bp.rowptr, Bp.col, Bp.val)
As = oracle.CSR(An.nrows, An.rowptr, An.col, An.val + shift * Bp.val)
lus = eigmi.LU.from_bcsr(ctx, As.rowptr, As.col, As.val)
for rep in range(3):
    t0 = time.perf_counter()
    eigmi.shift_invert_solve(dA, 8, sigma=-shift, B=dB, tol=1e-10, lu=lus, want_evec=False, method="block")
    t1 = time.perf_counter()
    eigmi.shift_invert_solve(dA, 8, sigma=-shift, B=dB, tol=1e-10, want_evec=False, method="block")
    t2 = time.perf_counter()
    print(f"N={N} factors given {1e3 * (t1 - t0):.1f} ms, incl. factorisation {1e3 * (t2 - t1):.1f} ms", flush=True)
