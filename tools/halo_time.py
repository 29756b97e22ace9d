"""Time the halo mailbox (k_comm.hip k_halo_push / k_halo_pull) between P mailbox-only processes on one
GPU: each rank owns a z-slab of the N^3 variable-coefficient 7-point matrix and runs `reps` eig_mv
calls and `steps` fused Lanczos steps (mailbox-step allreduce) under split and whole halo launches.
The ranks share one GPU, so per-step times include the other ranks' kernels; the exchange kernels'
own durations come from a kernel trace of this command (rocprofv3 --kernel-trace --stats).

    python tools/halo_time.py [N] [P] [reps] [steps]      (defaults 256 2 20 40)
One JSON line per rank on stdout.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def rank_main(rank, P, wd, N, reps, steps):
    import eigmi
    from mailbox_step_worker import publish, wait_for
    ctx = eigmi.Context(0)
    publish(wd, f"h{rank}.bin", ctx.ipc_handle(P, rank))
    paths = [os.path.join(wd, f"h{r}.bin") for r in range(P)]
    wait_for(paths)
    ctx.ipc_open(b"".join(open(p, "rb").read() for p in paths))
    n, D = N ** 3, N * N
    p0, p1 = N * rank // P, N * (rank + 1) // P
    b, cnt = p0 * D, (p1 - p0) * D
    rp, c, v = eigmi.gen_rows(eigmi.GEN_VARCOEF3D, N, b, cnt)
    M = eigmi.Matrix.from_rows(ctx, n, b, rp, c, v)
    del rp, c, v
    out = {"rank": rank, "P": P, "N": N, "rows": cnt, "halo_rows": int(M.info.halo_recv),
           "march_variant": int(M.info.march_variant)}
    xv, yv = M.window_vector(np.ones(cnt)), M.window_vector()
    ctx.select_allreduce("mailbox-step")
    for halo in ("split", "whole"):
        M.tune(halo_whole=int(halo == "whole"))
        M.mv(xv, yv)
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            M.mv(xv, yv)
        ctx.sync()
        out[f"mv_us_{halo}"] = round((time.perf_counter() - t0) / reps * 1e6, 1)
        ws = eigmi.LanczosWorkspace(M, steps + 6, seed=123, fused=True)
        ws.step(4)
        ctx.sync()
        t0 = time.perf_counter()
        ws.step(steps)
        ctx.sync()
        out[f"step_us_{halo}"] = round((time.perf_counter() - t0) / steps * 1e6, 1)
        ws.close()
    out["mailbox_errors"] = ctx.comm_info()["mailbox_errors"]
    out["halo_groups"] = ctx.comm_counters()["halo_groups"]
    xv.free()
    yv.free()
    M.close()
    ctx.close()
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--rank":
        rank_main(*[int(a) if i != 2 else a for i, a in enumerate(sys.argv[2:8])])
        return
    N, P, reps, steps = [int(a) for a in (sys.argv[1:] + ["256", "2", "20", "40"][len(sys.argv) - 1:])][:4]
    with tempfile.TemporaryDirectory() as wd:
        procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rank", str(r), str(P), wd, str(N),
                                   str(reps), str(steps)]) for r in range(P)]
        rc = 0
        for p in procs:
            try:
                rc |= p.wait(timeout=300)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
    sys.exit(rc)


if __name__ == "__main__":
    main()
