#!/usr/bin/env python3
"""One GenEO shift-invert solve (nev = 8, block method, factorisation included) after a warm-up:
the command profiled by tools/gpu_si_prof.sh."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import eigmi  # noqa: E402
import oracle  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
method = sys.argv[2] if len(sys.argv) > 2 else "block"
ctx = eigmi.Context(0)
shift = 1e-3
An, Bp = oracle.laplace2d(N, "neumann"), oracle.laplace2d(N, "pu", overlap=3)
dA = eigmi.Matrix.from_bcsr(ctx, An.rowptr, An.col, An.val)
dB = eigmi.Matrix.from_bcsr(ctx, Bp.rowptr, Bp.col, Bp.val)
for rep in range(2):
    t0 = time.perf_counter()
    ev, _, r = eigmi.shift_invert_solve(dA, 8, sigma=-shift, B=dB, tol=1e-10, want_evec=False, method=method)
    print(f"N={N} {method}: {1e3 * (time.perf_counter() - t0):.1f} ms, restarts {r}")
