#!/usr/bin/env python3
"""Where the inverse drivers' wall time goes at 64^2: host-only factorisation vs the device
factor upload (staged + block-inverse images), and the shift-invert solve with / without the
factors given."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import eigmi  # noqa: E402
import oracle  # noqa: E402


def t(f, reps=3):
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        r = f()
        best = min(best, time.perf_counter() - t0)
    return best, r


ctx = eigmi.Context(0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
A = oracle.laplace2d(N)
th, _ = t(lambda: eigmi.LU.from_bcsr(None, A.rowptr, A.col, A.val))
td, lu = t(lambda: eigmi.LU.from_bcsr(ctx, A.rowptr, A.col, A.val))
print(f"host LU {th*1e3:.1f} ms, device LU (factor + images + upload) {td*1e3:.1f} ms")
shift = 1e-3
An, Bp = oracle.laplace2d(N, "neumann"), oracle.laplace2d(N, "pu", overlap=3)
dA = eigmi.Matrix.from_bcsr(ctx, An.rowptr, An.col, An.val)
dB = eigmi.Matrix.from_bcsr(ctx, Bp.rowptr, Bp.col, Bp.val)
As = oracle.CSR(An.nrows, An.rowptr, An.col, An.val + shift * Bp.val)
lus = eigmi.LU.from_bcsr(ctx, As.rowptr, As.col, As.val)
for method in ("single", "block"):
    ts, (ev, _, r) = t(lambda: eigmi.shift_invert_solve(dA, 8, sigma=-shift, B=dB, tol=1e-10, want_evec=False,
                                                        method=method))
    tg, _ = t(lambda: eigmi.shift_invert_solve(dA, 8, sigma=-shift, B=dB, tol=1e-10, lu=lus, want_evec=False,
                                               method=method))
    tv, _ = t(lambda: eigmi.shift_invert_solve(dA, 8, sigma=-shift, B=dB, tol=1e-10, lu=lus, method=method))
    print(f"shift-invert {method}: {ts*1e3:.1f} ms incl. factorisation, {tg*1e3:.1f} ms with the factors given, "
          f"{tv*1e3:.1f} ms with vectors; restarts {r}; ev {ev[:3]}")
if len(sys.argv) <= 2:
    for kind in ("staged", "csr"):
        lus.set_solver(kind)
        tk, _ = t(lambda: eigmi.shift_invert_solve(dA, 8, sigma=-shift, B=dB, tol=1e-10, lu=lus, want_evec=False,
                                                   method="single"))
        print(f"shift-invert single with factors, solver {kind}: {tk*1e3:.1f} ms")
import scipy.sparse.linalg as ssl  # noqa: E402
As_, Bs_ = An.to_scipy(), Bp.to_scipy()
tc, w = t(lambda: ssl.eigsh(As_, k=8, M=Bs_, sigma=-shift, which="LM", tol=1e-10, return_eigenvectors=False))
print(f"scipy ARPACK + SuperLU: {tc*1e3:.1f} ms; ev {np.sort(w)[:3]}")
