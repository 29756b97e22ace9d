#!/usr/bin/env python3
"""The general (non-banded) CSR/ELL path at scale: 3-D Poisson N^3 under a seeded
random symmetric permutation followed by reverse Cuthill-McKee (eigmi.scrambled_rcm) -- same nnz
and symmetry, but no constant-offset band (no symmetric band image) and no per-slice stencil (every
SELL slice keeps explicit column indices).  Times eig_mv (BCRSMatrix::mv, arpack_geneo_wrapper.hh:
269-279 / kernels_cpp.hh:596-621) and the Lanczos step kernels on that image against SURVEY 8(d)'s
CSR bytes: SpMV 12 nnz + 4 (n+1) + 16 n, fused step 12 nnz + 4 (n+1) + 32 n, K1 + 24 n.
One JSON line per measurement.

    python tools/csr_general.py [--N 256] [--reps 20]
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

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--seed", type=int, default=123)
    args = ap.parse_args()
    N = args.N
    t0 = time.perf_counter()
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
    rp, c, v = eigmi.scrambled_rcm(rp, c, v, args.seed)
    t_reorder = time.perf_counter() - t0
    n, nnz = rp.size - 1, int(rp[-1])
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
    bw = int(np.abs(c - rows).max())
    ctx = eigmi.Context(0)
    t0 = time.perf_counter()
    M = eigmi.Matrix.from_bcsr(ctx, rp, c, v)
    t_up = time.perf_counter() - t0
    info = M.info
    base = {"config": f"3-D Poisson {N}^3, scrambled + RCM (seed {args.seed})", "n": n, "nnz": nnz, "bandwidth": bw,
            "stencil_slices": int(info.stencil_slices), "nslices": int(info.nslices),
            "band_image": int(info.sym_offsets), "padded_fill": round(info.nnzb_padded / nnz, 4),
            "reorder_s": round(t_reorder, 1), "upload_s": round(t_up, 1)}
    x = ctx.array(np.random.default_rng(0).standard_normal(n))
    y = ctx.zeros(n)
    for cpf in (0, 1, 0, 1):
        M.tune(sell_cpf=cpf)  # EIG_TUNE_SELL_CPF: explicit slices' cross-slice column prefetch
        M.mv_timed(x, y, 3)
        ms = min(M.mv_timed(x, y, args.reps) for _ in range(3))
        b = eigmi.bytes_spmv(n, nnz)
        print(json.dumps(dict(base, op="eig_mv" + (" +col-prefetch" if cpf else ""), kernel=M.kernel("spmv"),
                              us=round(ms * 1e3, 2), csr_bytes=b, GBs=round(b / ms / 1e6, 1),
                              frac=round(b / ms / 1e6 / PEAK, 4))), flush=True)
    ref_ab = None
    for fused, cpf in ((True, 0), (True, 1), (True, 0), (True, 1), (False, 0)):
        M.tune(sell_cpf=cpf)  # EIG_TUNE_SELL_CPF: explicit slices' cross-slice column prefetch (fused step)
        ws = eigmi.LanczosWorkspace(M, args.steps + 4, seed=123, fused=fused)
        ws.step(2)
        t = ws.step(args.steps, timed=True)
        k_us = t.spmv_ms / max(1, t.spmv_launches) * 1e3
        kb = eigmi.bytes_lanczos_fused(n, nnz) if fused else eigmi.bytes_lanczos_k1(n, nnz)
        step_us = t.total_ms / args.steps * 1e3
        # results first, timing second: a fused variant must reproduce the plain fused kernel bitwise
        ab = ws.tridiag()
        if fused and ref_ab is None:
            ref_ab = ab
        same = bool(np.array_equal(ab[0], ref_ab[0]) and np.array_equal(ab[1], ref_ab[1])) if fused else None
        print(json.dumps(dict(base, op="lanczos " + ("fused" if fused else "classic") + (" +col-prefetch" if cpf else ""),
                              alpha_beta_bitwise_vs_plain=same,
                              kernel=M.kernel("fused" if fused else "k1"), kernel_us=round(k_us, 2), csr_bytes=kb,
                              GBs=round(kb / k_us / 1e3, 1), frac=round(kb / k_us / 1e3 / PEAK, 4),
                              step_us=round(step_us, 2), steps_per_s=round(1e6 / step_us, 1))), flush=True)
        ws.close()
    M.close()
    ctx.close()


if __name__ == "__main__":
    main()
