#!/usr/bin/env python3
"""The fused Lanczos step on images other than the bench's 7-point band march: the SELL stencil
image of the 3-D Poisson matrix (EIG_MAT_NO_BAND: the kernel the distributed boundary slices and
non-band stencil matrices run, k_lanczos_fused_b1 in stencil mode) and the P1 Kuhn stiffness band
(15 offsets: the general band march, several offsets per far span).  Kernel and step time per
launch, one JSON line per matrix.

    python tools/stencil_fused.py [--N 256] [--steps 40]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import eigmi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    ctx = eigmi.Context(0)
    for label, kind, flags in (("3-D Poisson, SELL stencil image", eigmi.GEN_POISSON3D, eigmi.MAT_NO_BAND),
                               ("P1 Kuhn K, band image (general march)", eigmi.GEN_P1STIFF3D, 0)):
        rp, c, v = eigmi.gen_matrix(kind, a.N)
        M = eigmi.Matrix.from_bcsr(ctx, rp, c, v, flags=flags)
        del rp, c, v
        best = None
        for _ in range(3):
            ws = eigmi.LanczosWorkspace(M, a.steps + 4, seed=123, fused=True)
            ws.step(2)
            t = ws.step(a.steps, timed=True)
            k_us = t.spmv_ms / max(1, t.spmv_launches) * 1e3
            s_us = t.total_ms / a.steps * 1e3
            best = (k_us, s_us) if best is None or k_us < best[0] else best
            ws.close()
        name, nbytes = M.lanczos_kernel_info(True)
        print(json.dumps({"config": f"{label} {a.N}^3", "kernel": name, "kernel_us": round(best[0], 2),
                          "step_us": round(best[1], 2), "bytes": nbytes,
                          "frac": round(nbytes / (best[0] * 1e-6) / 8e12, 4)}), flush=True)
        M.close()

if __name__ == "__main__":
    main()
