#!/usr/bin/env python3
"""A/B of SpMV image variants on one GPU, interleaved rounds in ONE process (guide rule 24).

For each variant (EIGMI_SELL_R = rows per lane) the 256^3 Poisson matrix is uploaded once; then
rounds alternate between variants: a batch of Lanczos steps (kernel events) and a batch of plain
eig_mv launches.  Prints one JSON line per variant (median / min over rounds)."""
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
    ap.add_argument("--variants", default="1e,1s,2e,2s")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    ctx = eigmi.Context(0)
    N = args.N
    n = N ** 3
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
    nnz = int(rp[-1])
    mats = {}
    pipe = {}
    for var in args.variants.split(","):  # "<R><s|e>[:p<0|1|2>]": rows per lane, stencil on/off, K1 kernel
        img, _, pm = var.partition(":")
        os.environ["EIGMI_SELL_R"] = img[0]
        os.environ["EIGMI_STENCIL"] = "0" if img.endswith("e") else "1"
        mats[var] = eigmi.Matrix.from_bcsr(ctx, rp, c, v)
        pipe[var] = pm[1:] if pm else "0"
    x = ctx.array(np.random.default_rng(0).standard_normal(n))
    y = ctx.zeros(n)
    res = {R: {"k1_us": [], "k2_us": [], "step_us": [], "mv_us": []} for R in mats}
    for _ in range(args.rounds):
        for R, M in mats.items():
            os.environ["EIGMI_K1_PIPE"] = pipe[R]
            ws = eigmi.LanczosWorkspace(M, args.steps + 2, seed=123)
            ws.step(2)
            t = ws.step(args.steps, timed="detail")
            res[R]["k1_us"].append(t.spmv_ms / args.steps * 1e3)
            res[R]["k2_us"].append(t.update_ms / args.steps * 1e3)
            res[R]["step_us"].append(t.total_ms / args.steps * 1e3)
            ws.close()
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                M.mv(x, y)
            ctx.sync()
            res[R]["mv_us"].append((time.perf_counter() - t0) / args.steps * 1e6)
    k1b = eigmi.bytes_lanczos_k1(n, nnz)
    mvb = eigmi.bytes_spmv(n, nnz)
    for R, d in res.items():
        med = {k: float(np.median(v)) for k, v in d.items()}
        out = {"R": R, **{k: round(val, 2) for k, val in med.items()},
               "k1_min_us": round(min(d["k1_us"]), 2),
               "k1_GBs": round(k1b / (med["k1_us"] * 1e-6) / 1e9, 1),
               "mv_GBs": round(mvb / (med["mv_us"] * 1e-6) / 1e9, 1),
               "it_per_s": round(1e6 / med["step_us"], 1),
               "nnz_padded": mats[R].info.nnzb_padded, "stencil_slices": mats[R].info.stencil_slices}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
