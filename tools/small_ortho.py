#!/usr/bin/env python3
"""orthonormalize_blocked (MGS) on small blocks (C1's n = 4096 and around): the one-workgroup
k_mgs_small (EIG_ORTHO_ONE_WG) against the default grid look-ahead path, us per call over back-to-back calls."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import numpy as np  # noqa: E402

import eigmi  # noqa: E402

ctx = eigmi.Context(0)
reps = 200
for n in [int(x) for x in (sys.argv[1:] or ["512", "1024", "2048", "4096"])]:
    m = 8
    Q = ctx.zeros(n * m)
    for name, var in (("small", eigmi.ORTHO_MGS | eigmi.ORTHO_ONE_WG), ("grid", eigmi.ORTHO_MGS)):
        eigmi.random_mv8(ctx, n, m, 1, Q)
        eigmi.orthonormalize_mv8(ctx, n, m, Q, var)
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            eigmi.orthonormalize_mv8(ctx, n, m, Q, var)
        ctx.sync()
        us = (time.perf_counter() - t0) / reps * 1e6
        print(json.dumps({"n": n, "m": m, "path": name, "us_per_call": round(us, 2)}), flush=True)
