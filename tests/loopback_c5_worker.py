"""Config C5's block Lanczos at C5's size, row-partitioned over P virtual ranks on ONE GPU
(tests/test_loopback_c5.py runs this as a child process).

The variable-coefficient P1 Kuhn pencil K x = lambda M x at N^3 (eig_gen kinds 9 / 10, one coefficient
per tetrahedron, EIG_MAT_NO_CLASS: every launch streams the box image, as tools/bench_configs.py c5
and tests/test_gpu_c5_size.py) is split into P z-slabs of N/P planes, one virtual rank (host thread +
context) per slab over the in-process loopback hub (eig_loopback_create).  Each rank runs BLOCK x STEPS
block Lanczos steps (eigensolver.hh:283-325 work: SpMM with K, the Chebyshev-Jacobi mass solve, CGS2 +
CholQR2 in the M-inner product, kernels_cpp.hh:356-591) with the halo exchanged and the Gram blocks
allreduced over the hub.  Checked against the one-rank run of the same pencil in this process:
  * the block-tridiagonal T within 1e-10 of max |T| (the same recurrence, other reduction orders),
  * the NEV largest Ritz values within 1e-10 relative, their device residuals within 1e-7 relative.
One JSON line per P on stdout (the first line is the one-rank run).

    python tests/loopback_c5_worker.py N STEPS P [P ...] [--const]

--const: the constant-coefficient P1 pencil (eig_gen kinds 6 / 7) with its row classes, so every rank
runs the row-class kernels (k_boxc_mv8: the class table in LDS, no matrix stream) on its slab.
"""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import eigmi  # noqa: E402

BLOCK, NEV = 32, 8
CONST = "--const" in sys.argv
KIND_K, KIND_M = ((eigmi.GEN_P1STIFF3D, eigmi.GEN_P1MASS3D) if CONST else
                  (eigmi.GEN_P1STIFF3D_VAR, eigmi.GEN_P1MASS3D_VAR))
FLAGS = 0 if CONST else eigmi.MAT_NO_CLASS


def solve(K, M, steps):
    bl = eigmi.BlockLanczos(K, M, block=BLOCK, max_steps=steps, degree=36, seed=123)
    try:
        bl.step(steps)
        T = bl.tmatrix()
        ev, _, res = bl.ritz(NEV, eigmi.WHICH_LA)
    finally:
        bl.close()
    return T, ev, res


def rank_run(hub, r, P, N, steps, out):
    n = N ** 3
    D = N * N
    p0, p1 = N * r // P, N * (r + 1) // P
    b, cnt = p0 * D, (p1 - p0) * D
    ctx = eigmi.Context(0)
    res = {"rank": r, "row_begin": b, "rows": cnt}
    K = M = None
    try:
        ctx.comm_init_loopback(hub, r)
        rk, ck, vk = eigmi.gen_rows(KIND_K, N, b, cnt)
        K = eigmi.Matrix.from_rows(ctx, n, b, rk, ck, vk, flags=FLAGS)
        del rk, ck, vk
        rm, cm, vm = eigmi.gen_rows(KIND_M, N, b, cnt)
        M = eigmi.Matrix.from_rows(ctx, n, b, rm, cm, vm, flags=FLAGS)
        del rm, cm, vm
        res.update(spmm=K.kernel("spmm32"), cheb=M.kernel("cheb32"), halo=int(K.info.halo_recv))
        t0 = time.time()
        res["T"], res["ev"], res["res"] = solve(K, M, steps)
        res["solve_s"] = round(time.time() - t0, 2)
    except Exception as e:  # reported to the parent; the other ranks' barriers then time out loudly
        res["error"] = repr(e)
    finally:
        for A in (K, M):
            if A is not None:
                A.close()
        ctx.close()
    out[r] = res


def main():
    N, steps = int(sys.argv[1]), int(sys.argv[2])
    Ps = [int(p) for p in sys.argv[3:] if not p.startswith("--")]
    n = N ** 3
    t0 = time.time()
    ctx = eigmi.Context(0)
    rk, ck, vk = eigmi.gen_matrix(KIND_K, N)
    K = eigmi.Matrix.from_bcsr(ctx, rk, ck, vk, flags=FLAGS)
    del rk, ck, vk
    rm, cm, vm = eigmi.gen_matrix(KIND_M, N)
    M = eigmi.Matrix.from_bcsr(ctx, rm, cm, vm, flags=FLAGS)
    del rm, cm, vm
    kinfo = (K.kernel("spmm32"), M.kernel("cheb32"))
    T1, ev1, res1 = solve(K, M, steps)
    K.close()
    M.close()
    ctx.close()
    print(json.dumps({"P": 1, "N": N, "const": CONST, "n": n, "steps": steps, "spmm": kinfo[0], "cheb": kinfo[1],
                      "ev": ev1.tolist(), "res": res1.tolist(), "seconds": round(time.time() - t0, 1)}), flush=True)
    tmax = float(np.abs(T1).max())
    for P in Ps:
        t1 = time.time()
        hub = eigmi.loopback_create(P)
        out = [None] * P
        th = [threading.Thread(target=rank_run, args=(hub, r, P, N, steps, out)) for r in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        eigmi.loopback_destroy(hub)
        line = {"P": P, "N": N, "steps": steps, "ranks": []}
        for res in out:
            rec = {k: res.get(k) for k in ("rank", "row_begin", "rows", "spmm", "cheb", "halo", "solve_s", "error")}
            if res.get("error") is None:
                T, ev, rs = res["T"], res["ev"], res["res"]
                rec["T_shape_ok"] = bool(T.shape == T1.shape)
                rec["T_rel"] = float(np.abs(T - T1).max() / tmax) if T.shape == T1.shape else None
                rec["ev_rel"] = float(np.max(np.abs(ev - ev1) / np.abs(ev1)))
                rec["res_rel"] = float(np.max(np.abs(rs - res1) / np.abs(res1)))
                rec["ev"] = ev.tolist()
            line["ranks"].append(rec)
        line["seconds"] = round(time.time() - t1, 1)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
