#!/usr/bin/env python3
"""Lanczos with full DGKS re-orthogonalisation (eig_lanczos_solve) at N^3: wall time per step and
the re-orthogonalisation share.  Run under rocprofv3 --kernel-trace --stats for per-kernel times.
    python tools/reorth_bench.py --N 256 --ncv 64"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import numpy as np  # noqa: E402

import eigmi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--ncv", type=int, default=64)
    ap.add_argument("--nev", type=int, default=4)
    args = ap.parse_args()
    ctx = eigmi.Context(0)
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, args.N)
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v)
    eigmi.lanczos_solve(M, args.nev, 16, want_evec=False)  # warm-up
    ctx.sync()
    t0 = time.perf_counter()
    ev, _, res = eigmi.lanczos_solve(M, args.nev, args.ncv, want_evec=False)
    ctx.sync()
    dt = time.perf_counter() - t0
    n = args.N ** 3
    k = args.ncv
    # DGKS bytes: 2 passes x (V^T t over j+1 columns + t -= V c) = 2 x 2 x 8 n (j+1), summed over j
    reorth_bytes = sum(4 * 8 * n * (j + 1) for j in range(k))
    print(json.dumps({"N": args.N, "ncv": k, "seconds": round(dt, 4), "ms_per_step": round(dt / k * 1e3, 3),
                      "reorth_model_GB": round(reorth_bytes / 1e9, 2),
                      "reorth_model_GBs_if_all_time": round(reorth_bytes / dt / 1e9, 1),
                      "ritz": [float(x) for x in ev]}), flush=True)
    M.close()
    ctx.close()


if __name__ == "__main__":
    main()
