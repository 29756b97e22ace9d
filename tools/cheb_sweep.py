#!/usr/bin/env python3
"""Per-launch time of the fused Chebyshev mass-solve step (config C5's dominant kernel) on the P1
Kuhn mass matrix, m columns: eig_mass_solve_mv8 at degree d_hi and d_lo, (t_hi - t_lo) / (d_hi - d_lo)
= one Chebyshev launch.  Variants are environment settings read at launch (SWEEP="k=v,k=v;...").
Algorithmic bytes per launch: 12 nnz + 4 (n+1) + (32 m + 8) n (tools/bench_configs.py c5).

    python tools/cheb_sweep.py --N 256 --m 32
"""
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
    ap.add_argument("--m", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dlo", type=int, default=2)
    ap.add_argument("--dhi", type=int, default=34)
    args = ap.parse_args()
    ctx = eigmi.Context(0)
    N, m = args.N, args.m
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_P1MASS3D, N)
    n = rp.size - 1
    nnz = int(rp[-1])
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v)
    B = ctx.array(np.random.default_rng(1).standard_normal(n * m))
    X = ctx.zeros(n * m)
    variants = [dict(kv.split("=") for kv in s.split(",") if kv) for s in os.environ.get("SWEEP", "").split(";")]
    res = {i: [] for i in range(len(variants))}
    for _ in range(args.rounds):
        for i, var in enumerate(variants):
            for k in [k for k in os.environ if k.startswith("EIGMI_EXP_")]:
                os.environ.pop(k, None)
            os.environ.update(var)
            ts = {}
            for d in (args.dlo, args.dhi):
                eigmi.mass_solve_mv8(M, m, d, B, X)
                ctx.sync()
                t0 = time.perf_counter()
                eigmi.mass_solve_mv8(M, m, d, B, X)
                ts[d] = time.perf_counter() - t0
            res[i].append((ts[args.dhi] - ts[args.dlo]) / (args.dhi - args.dlo))
    byt = 12 * nnz + 4 * (n + 1) + (32 * m + 8) * n  # SURVEY 8(d) CSR count (the row-class kernel: 32 m n)
    for i, var in enumerate(variants):
        t = float(np.median(res[i]))
        print(json.dumps({"variant": var, "N": N, "m": m, "kernel": M.kernel("cheb8"), "launch_ms": round(t * 1e3, 3),
                          "launch_ms_min": round(min(res[i]) * 1e3, 3), "alg_bytes": byt,
                          "GBs": round(byt / t / 1e9, 1), "frac": round(byt / t / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
