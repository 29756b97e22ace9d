#!/usr/bin/env python3
"""A/B of the device band LU's panel kernels (k_band_panel2 default vs EIGMI_BAND_PANEL=1): run once
per setting with an output prefix; the second call with --compare checks the exported factors are
bitwise identical and prints the factorisation times.
    EIGMI_BAND_PANEL=1 python3 tools/band_panel_ab.py /tmp/p1 && python3 tools/band_panel_ab.py /tmp/p2 --compare /tmp/p1"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import eigmi  # noqa: E402
import oracle  # noqa: E402

out = sys.argv[1]
cmp = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--compare" else None
ctx = eigmi.Context(0)
cases = {"laplace2d_64": oracle.laplace2d(64), "laplace2d_200": oracle.laplace2d(200),
         "poisson3d_16": oracle.poisson3d(16), "q1elast_4": oracle.q1elast(4), "laplace2d_5": oracle.laplace2d(5)}
ok = True
for name, A in cases.items():
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        lu = eigmi.LU.from_bcsr(ctx, A.rowptr, A.col, A.val, A.br)
        ctx.sync()
        best = min(best, time.perf_counter() - t0)
        ex = lu.export()
        lu.close()
    np.savez(f"{out}_{name}.npz", **{k: np.asarray(v) for k, v in ex.items()})
    line = f"{name}: LU create {best * 1e3:.2f} ms"
    if cmp:
        ref = np.load(f"{cmp}_{name}.npz")
        same = all(np.array_equal(ref[k], np.asarray(ex[k])) for k in ref.files)
        ok = ok and same
        line += f", factors bitwise equal to the other panel kernel: {same}"
    print(line, flush=True)
if cmp and not ok:
    sys.exit(1)
