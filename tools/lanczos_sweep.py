#!/usr/bin/env python3
"""A/B of Lanczos step variants on one GPU, interleaved rounds in ONE process (guide rule 24).

Variant spec "<fused|classic>[:swz0|swz1][:w4|w5|w6|w8][:nt0|nt1][:sym0|sym1|sym2][:march0|1|2|3][:mnt0|mnt1][:wg0|wg1][:seg<k>][:m7|m8]": step form, XCD-aware chunk
order (EIGMI_XCD_SWIZZLE), register budget of the fused kernel (EIGMI_FUSED_WAVES), nontemporal
stores of the step vectors (EIGMI_NT_STORE), symmetric band image or SELL image (EIGMI_SYM), plane marching
(EIGMI_MARCH).  The environment is
read at every launch, so all variants share one matrix upload.  One JSON line per variant:
median / min over rounds of the step time and of the dominant kernel's time.

    python tools/lanczos_sweep.py --variants classic:swz0,classic:swz1,fused:swz1:w5
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import numpy as np  # noqa: E402

import eigmi  # noqa: E402


def parse(spec):
    parts = spec.split(":")
    env = {"EIGMI_XCD_SWIZZLE": "0", "EIGMI_FUSED_WAVES": "8", "EIGMI_NT_STORE": "0", "EIGMI_SYM": "2", "EIGMI_MARCH": "d", "EIGMI_MARCH_NT": "1",
           "EIGMI_MARCH_WG": "0", "EIGMI_MARCH_SEG": "0", "EIGMI_MARCH_W7": "1"}
    for p in parts[1:]:
        if p in ("m7", "m8"):
            env["EIGMI_MARCH_W7"] = "1" if p == "m7" else "0"
        elif p.startswith("wg"):
            env["EIGMI_MARCH_WG"] = p[2:]
        elif p.startswith("seg"):
            env["EIGMI_MARCH_SEG"] = p[3:]
        elif p.startswith("mnt"):
            env["EIGMI_MARCH_NT"] = p[3:]
        elif p.startswith("march"):
            env["EIGMI_MARCH"] = p[5:]
        elif p.startswith("sym"):
            env["EIGMI_SYM"] = p[3:]
        elif p.startswith("nt"):
            env["EIGMI_NT_STORE"] = p[2:]
        elif p.startswith("swz"):
            env["EIGMI_XCD_SWIZZLE"] = p[3:]
        elif p.startswith("w"):
            env["EIGMI_FUSED_WAVES"] = p[1:]
    return parts[0] == "fused", env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--variants", default="classic:swz0,classic:swz1,fused:swz0,fused:swz1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--slab", type=int, default=0, help="N x N x slab box instead of the N^3 cube")
    args = ap.parse_args()
    ctx = eigmi.Context(0)
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
        A.sort_indices()
        rp, c, v = A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data.astype(np.float64)
        n = A.shape[0]
    else:
        n = N ** 3
        rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
    nnz = int(rp[-1])
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v)
    specs = args.variants.split(",")
    res = {s: {"k_us": [], "step_us": []} for s in specs}
    xy = None
    for _ in range(args.rounds):
        for spec in specs:
            fused, env = parse(spec)
            os.environ.update(env)
            if spec.startswith("mv"):  # plain eig_mv (BCRSMatrix::mv) launches
                if xy is None:
                    xy = (ctx.array(np.random.default_rng(0).standard_normal(n)), ctx.zeros(n))
                ms = M.mv_timed(xy[0], xy[1], args.steps)
                res[spec]["k_us"].append(ms * 1e3)
                res[spec]["step_us"].append(ms * 1e3)
                continue
            ws = eigmi.LanczosWorkspace(M, args.steps + 2, seed=123, fused=fused)
            ws.step(2)
            t = ws.step(args.steps, timed=True)
            res[spec]["k_us"].append(t.spmv_ms / args.steps * 1e3)
            res[spec]["step_us"].append(t.total_ms / args.steps * 1e3)
            ws.close()
    for spec in specs:
        fused, _ = parse(spec)
        kb = (eigmi.bytes_spmv(n, nnz) if spec.startswith("mv") else
              eigmi.bytes_lanczos_fused(n, nnz) if fused else eigmi.bytes_lanczos_k1(n, nnz))
        r = res[spec]
        km = float(np.median(r["k_us"]))
        sm = float(np.median(r["step_us"]))
        print(json.dumps({"variant": spec, "kernel_us_med": round(km, 2), "kernel_us_min": round(min(r["k_us"]), 2),
                          "kernel_GBs": round(kb / km / 1e3, 1), "step_us_med": round(sm, 2),
                          "steps_per_s": round(1e6 / sm, 1),
                          "step_frac_survey_bytes": round(eigmi.bytes_lanczos_step(n, nnz) / sm / 1e3 / 8000, 4)}),
              flush=True)
    M.close()
    ctx.close()


if __name__ == "__main__":
    main()
