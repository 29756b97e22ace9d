"""Config C4's row partition at C4's size on ONE GPU (tests/test_loopback_c4.py runs this as a child
process, so GPU_MAX_HW_QUEUES can be set before the HIP runtime starts).

The 3-D Poisson matrix at N^3 (the benchmark's image: EIG_MAT_NO_UNIFORM, every band value streamed)
is split into P z-slabs of N/P planes, one virtual rank (host thread + context) per slab over the
in-process loopback hub (eig_loopback_create).  Every rank runs the step kernel the benchmark times
on its slab (k_lanczos_fused_march: the value march, variant 15 or the 2-line 22 by rank size) with
  * the loopback halo (device copies) and the loopback allreduce, split launches (interior march +
    boundary slices) and whole launches (EIG_TUNE_HALO = 1),
  * the in-kernel allreduce (EIG_AR_MAILBOX_STEP, csrc/xch_dev.h: the last workgroup of a launch
    publishes the three sums into every peer's mailbox and gathers theirs), split and whole launches.
Checked here against the CPU restatement on the GLOBAL matrix (oracle/oracle.cc, the checker only):
  * distributed eig_mv BITWISE oracle.csr_mv (matmul_sparse_tallskinny_naive, kernels_cpp.hh:596-621),
  * STEPS fused steps vs orc_lanczos_fused, rtol 1e-12 (one halo exchange + one fused
    3-value allreduce per step).
One JSON line per P on stdout.

    python tests/loopback_c4_worker.py N STEPS P [P ...]
"""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import eigmi  # noqa: E402
import oracle  # noqa: E402


def rank_run(hub, r, P, N, steps, x, out):
    n = N ** 3
    D = N * N
    p0, p1 = N * r // P, N * (r + 1) // P
    b, cnt = p0 * D, (p1 - p0) * D
    ctx = eigmi.Context(0)
    res = {"rank": r, "row_begin": b, "rows": cnt}
    try:
        ctx.comm_init_loopback(hub, r)
        rp, c, v = eigmi.gen_rows(eigmi.GEN_POISSON3D, N, b, cnt)
        M = eigmi.Matrix.from_rows(ctx, n, b, rp, c, v, flags=eigmi.MAT_NO_UNIFORM)
        del rp, c, v
        info = M.info
        res.update(variant=int(info.march_variant), uniform=int(info.sym_uniform),
                   halo=int(info.halo_recv), kernel=M.lanczos_kernel_info(True)[0])
        xv = M.window_vector(x[b:b + cnt])
        yv = M.window_vector()
        M.mv(xv, yv)
        res["y"] = M.owned(yv)
        xv.free()
        yv.free()
        runs = {}
        for ar in ("loopback", "mailbox-step"):
            if ar == "mailbox-step":
                ctx.comm_loopback_mailbox()
                ctx.select_allreduce("mailbox-step")
            for halo in ("split", "whole"):
                M.tune(halo_whole=int(halo == "whole"))
                a, be, _ = eigmi.lanczos_run(M, steps, seed=123, fused=True)
                runs[f"{ar}/{halo}"] = (a, be)
        ci = ctx.comm_info()
        res.update(runs=runs, allreduce=ci["allreduce"], mailbox_errors=ci["mailbox_errors"])
        M.close()
    except Exception as e:  # reported to the parent; the other ranks' barriers then time out loudly
        res["error"] = repr(e)
    finally:
        ctx.close()
    out[r] = res


def main():
    N, steps = int(sys.argv[1]), int(sys.argv[2])
    Ps = [int(p) for p in sys.argv[3:]]
    n = N ** 3
    t0 = time.time()
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, N)
    A = oracle.CSR(n, rp, c, v)
    x = np.random.default_rng(21).standard_normal(n)
    y_ref = oracle.csr_mv(A, x)
    ra, rb = oracle.lanczos_fused(A, oracle.random_vec(n, 123), steps)
    del A, rp, c, v
    t_oracle = time.time() - t0
    for P in Ps:
        t1 = time.time()
        hub = eigmi.loopback_create(P)
        out = [None] * P
        th = [threading.Thread(target=rank_run, args=(hub, r, P, N, steps, x, out)) for r in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        eigmi.loopback_destroy(hub)
        line = {"P": P, "N": N, "steps": steps, "oracle_s": round(t_oracle, 1), "ranks": []}
        for res in out:
            r = res["rank"]
            rec = {k: res.get(k) for k in ("rank", "row_begin", "rows", "variant", "uniform", "halo", "kernel",
                                            "allreduce", "mailbox_errors", "error")}
            if "y" in res:
                b, cnt = res["row_begin"], res["rows"]
                rec["mv_bitwise"] = bool(np.array_equal(res["y"], y_ref[b:b + cnt]))
            rel = {}
            for key, (a, be) in res.get("runs", {}).items():
                da = float(np.max(np.abs(a - ra) / np.abs(ra)))
                db = float(np.max(np.abs(be[1:] - rb[1:]) / np.abs(rb[1:])))
                rel[key] = [da, db]
            rec["rel"] = rel
            line["ranks"].append(rec)
        line["seconds"] = round(time.time() - t1, 1)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
