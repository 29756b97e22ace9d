#!/usr/bin/env python3
"""A/B of Lanczos step / SpMV kernel images on one GPU, interleaved rounds in ONE process.

Variant spec "<fused|pipelined|classic|mv>[:<image>][@<runs>][#<pf>][^<lines>][~<transport>]" (runs: plane runs per
column of the march kernels, pf: the geometric march variant, eig_mat_tune; default automatic;
transport, with --comm self: the one-rank allreduce of every step -- rccl, mailbox, or step = the
fused step's sums exchanged inside the step kernel, EIG_AR_MAILBOX_STEP) with image one of
    band     (default) symmetric band image, plane march where the band allows it
    arrays   band image with the values streamed from the band arrays (EIG_MAT_NO_UNIFORM)
    gather   band image, every offset through its own gather (EIG_MAT_BAND_GATHER)
    nomarch  band image, row kernels (EIG_MAT_NO_MARCH)
    sell     SELL-64 / stencil-slice image (EIG_MAT_NO_BAND)
    explicit SELL-64 with explicit column indices only (EIG_MAT_NO_BAND | EIG_MAT_NO_STENCIL)
Each image is uploaded once (eig_mat_create_bcsr_ex flags) and shared by its variants.  One JSON
line per variant: median / min over rounds of the step time and of the dominant kernel's time.

    python tools/lanczos_sweep.py --variants fused,fused:sell,classic,mv,mv:explicit
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import numpy as np  # noqa: E402

import eigmi  # noqa: E402

IMAGES = {"band": 0, "arrays": eigmi.MAT_NO_UNIFORM, "gather": eigmi.MAT_BAND_GATHER, "nomarch": eigmi.MAT_NO_MARCH, "sell": eigmi.MAT_NO_BAND,
          "explicit": eigmi.MAT_NO_BAND | eigmi.MAT_NO_STENCIL}


def parse(spec):
    """"op[:image][@runs][#pf][%cache][^lines][~transport]" -> (op, image flags, plane runs per column
    (0 = automatic), geometric march variant (eig_mat_tune EIG_TUNE_MARCH_PREFETCH; 0 = automatic),
    cache bits, lines per workgroup of the value march (EIG_TUNE_MARCH_LINES; 0 = default))."""
    spec = spec.partition("~")[0]
    spec, _, lines = spec.partition("^")
    spec, _, cache = spec.partition("%")
    spec, _, pf = spec.partition("#")
    spec, _, runs = spec.partition("@")
    parts = spec.split(":")
    return (parts[0], IMAGES[parts[1] if len(parts) > 1 else "band"], int(runs or 0), int(pf or 0), int(cache or 0),
            int(lines or 0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--variants", default="fused,fused:sell,classic,mv")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--slab", type=int, default=0, help="N x N x slab box instead of the N^3 cube")
    ap.add_argument("--matrix", choices=["poisson", "varcoef", "p1k", "p1m"], default="poisson",
                    help="7-point Poisson (eig_gen kind 4), the variable-coefficient 7-point (kind 8), or the P1 "
                         "Kuhn stiffness / mass (kinds 6 / 7, config C5's 15-point K and M)")
    ap.add_argument("--comm", choices=["none", "self"], default="none",
                    help="self: a one-rank RCCL communicator + mailbox with EIG_COMM_ALWAYS, so every step's "
                         "allreduce runs through the transport named by the variant's ~suffix (default rccl)")
    args = ap.parse_args()
    ctx = eigmi.Context(0)
    if args.comm == "self":
        ctx.comm_init(1, 0, eigmi.Context.unique_id(), mailbox=True, always=True)
        assert ctx.comm_info()["allreduce"] == "xgmi-mailbox", ctx.comm_info()
    N = args.N
    if args.slab:
        # one rank's share of an 8-way row partition: a standalone N x N x slab 7-point box
        # (Dirichlet on all faces; no halo), to time the per-GPU compute of the strong-scaling runs
        import scipy.sparse as sp

        def lap1(k):
            return sp.diags([-np.ones(k - 1), np.zeros(k), -np.ones(k - 1)], [-1, 0, 1])
        Ix, Iz = sp.identity(N), sp.identity(args.slab)
        A = (sp.kron(Iz, sp.kron(Ix, lap1(N))) + sp.kron(Iz, sp.kron(lap1(N), Ix)) +
             sp.kron(lap1(args.slab), sp.kron(Ix, Ix))).tocsr()
        A.setdiag(6.0)
        if args.matrix == "varcoef":
            # a random conductance per grid edge (symmetric), diagonal 6 + U(0, 1): no uniform band
            rng = np.random.default_rng(5)
            U = sp.triu(A, k=1).tocoo()
            U.data = -0.5 - rng.random(U.nnz)
            A = (U + U.T + sp.diags(6.0 + rng.random(A.shape[0]))).tocsr()
        A.sort_indices()
        rp, c, v = A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data.astype(np.float64)
        n = A.shape[0]
    else:
        n = N ** 3
        rp, c, v = eigmi.gen_matrix({"poisson": eigmi.GEN_POISSON3D, "varcoef": eigmi.GEN_VARCOEF3D,
                                     "p1k": eigmi.GEN_P1STIFF3D, "p1m": eigmi.GEN_P1MASS3D}[args.matrix], N)
    nnz = int(rp[-1])
    specs = args.variants.split(",")
    mats = {}
    for spec in specs:
        fl = parse(spec)[1]
        if fl not in mats:
            mats[fl] = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=fl)
    res = {s: {"k_us": [], "step_us": [], "step_us_events": []} for s in specs}
    xy = None
    for _ in range(args.rounds):
        for spec in specs:
            op, fl, runs, pf, cache, lines = parse(spec)
            M = mats[fl]
            M.tune(runs, march_prefetch=pf, cache=cache, march_lines=lines)
            if args.comm == "self":
                tr = spec.partition("~")[2] or "rccl"
                ctx.select_allreduce({"step": "mailbox-step"}.get(tr, tr))
            if op == "mv":  # plain eig_mv (BCRSMatrix::mv) launches
                if xy is None:
                    xy = (ctx.array(np.random.default_rng(0).standard_normal(n)), ctx.zeros(n))
                ms = M.mv_timed(xy[0], xy[1], args.steps)
                res[spec]["k_us"].append(ms * 1e3)
                res[spec]["step_us"].append(ms * 1e3)
                continue
            ws = eigmi.LanczosWorkspace(M, 2 * args.steps + 2, seed=123, fused=op == "fused",
                                        pipelined=op == "pipelined")
            ws.step(2)
            # kernel times from per-launch events; the step time from a second batch with the two
            # region events only (per-launch event packets lengthen every step by a few us)
            t = ws.step(args.steps, timed=True)
            t2 = ws.step(args.steps)
            res[spec]["k_us"].append(t.spmv_ms / args.steps * 1e3)
            res[spec]["step_us_events"].append(t.total_ms / args.steps * 1e3)
            res[spec]["step_us"].append(t2.total_ms / args.steps * 1e3)
            ws.close()
    for spec in specs:
        op, fl, runs, pf, cache, lines = parse(spec)
        M = mats[fl]
        M.tune(runs, march_prefetch=pf, cache=cache, march_lines=lines)
        kb = (eigmi.bytes_spmv(n, nnz) if op == "mv" else
              eigmi.bytes_spmv(n, nnz) + 56 * n if op == "pipelined" else
              eigmi.bytes_lanczos_fused(n, nnz) if op == "fused" else eigmi.bytes_lanczos_k1(n, nnz))
        r = res[spec]
        km = float(np.median(r["k_us"]))
        sm = float(np.median(r["step_us"]))
        info = M.info
        ib = eigmi.image_bytes(M, "spmv") + (16 * n if op == "fused" else 0)  # bytes the image streams
        print(json.dumps({"variant": spec, "matrix": args.matrix, "march_variant": info.march_variant,
                          "comm": args.comm,
                          "image_bytes": ib if op in ("mv", "fused") else None,
                          "image_frac": round(ib / (float(np.median(res[spec]["k_us"])) * 1e3) / 8000, 4)
                          if op in ("mv", "fused") else None,
                          "kernel": M.kernel({"mv": "spmv", "fused": "fused", "pipelined": "spmv",
                                                             "classic": "k1"}[op]),
                          "kernel_us_med": round(km, 2), "kernel_us_min": round(min(r["k_us"]), 2),
                          "kernel_csr_GBs": round(kb / km / 1e3, 1), "step_us_med": round(sm, 2),
                          "step_us_med_with_events": round(float(np.median(r["step_us_events"])), 2)
                          if r["step_us_events"] else None,
                          "steps_per_s": round(1e6 / sm, 1),
                          "step_frac_survey_bytes": round(eigmi.bytes_lanczos_step(n, nnz) / sm / 1e3 / 8000, 4)}),
              flush=True)
    for M in mats.values():
        M.close()
    ctx.close()


if __name__ == "__main__":
    main()
