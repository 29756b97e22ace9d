"""One rank of tests/test_mailbox_step_gpu.py: the fused Lanczos step with its three sums exchanged
INSIDE the step kernel (EIG_AR_MAILBOX_STEP, csrc/xch_dev.h) between real processes on one GPU,
attached through eig_comm_ipc_handle / _open (the IPC mappings eig_comm_init_ex sets up between GPUs).

The global matrix is block diagonal -- rank r owns one random symmetric 7-point box (block(r)) -- so
the row partition has no halo (mailbox-only ranks have no RCCL for one) while every step's dots
still need all ranks' sums.

    python tests/mailbox_step_worker.py RANK NRANKS WORKDIR MODE
MODE "run": the recurrence under "mailbox" (one allreduce launch per step) and "mailbox-step"
(eager batches and a hipGraph replay, then the exact final beta), saved to r<RANK>.npz.
MODE "stall": rank 0 steps while rank 1 never does (it waits for rank 0's "done" file): rank 0's
in-kernel exchange must time out and the step call return EIG_ERR_RCCL, without a hang.
MODE "stall_tridiag": both ranks step, then only rank 0 calls tridiag(): the forced final repair's
exchange times out and tridiag() returns EIG_ERR_RCCL (not a NaN beta with EIG_OK).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import eigmi  # noqa: E402

NX, NY = 64, 4  # plane of 256 rows (a multiple of 64: the plane march applies)
STEPS = (6, 20, 8)  # eager, captured, eager


def block(r):
    """Rank r's diagonal block: a random symmetric 7-point box NX x NY x (5 + r), diagonally dominant."""
    import scipy.sparse as sp
    nz = 5 + r
    rng = np.random.default_rng(100 + r)
    n = NX * NY * nz
    idx = np.arange(n)
    x, y, z = idx % NX, (idx // NX) % NY, idx // (NX * NY)
    rows, cols, vals = [idx], [idx], [6.0 + rng.random(n)]
    for step, ok in ((1, x < NX - 1), (NX, y < NY - 1), (NX * NY, z < nz - 1)):
        i = idx[ok]
        w = -0.5 - rng.random(i.size)
        rows += [i, i + step]
        cols += [i + step, i]
        vals += [w, w]
    S = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    S.sort_indices()
    return S


def global_matrix(P):
    import scipy.sparse as sp
    G = sp.block_diag([block(r) for r in range(P)], format="csr")
    G.sort_indices()
    return G


def wait_for(paths, timeout=120.0):
    t0 = time.time()
    while not all(os.path.exists(p) for p in paths):
        if time.time() - t0 > timeout:
            raise TimeoutError(f"peers did not publish {paths}")
        time.sleep(0.01)


def publish(wd, name, data=b"1"):
    tmp = os.path.join(wd, name + ".tmp")
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, os.path.join(wd, name))


def main(rank, P, wd, mode):
    ctx = eigmi.Context(0)
    publish(wd, f"h{rank}.bin", ctx.ipc_handle(P, rank))
    paths = [os.path.join(wd, f"h{r}.bin") for r in range(P)]
    wait_for(paths)
    ctx.ipc_open(b"".join(open(p, "rb").read() for p in paths))
    sizes = [NX * NY * (5 + r) for r in range(P)]
    n = sum(sizes)
    b = sum(sizes[:rank])
    S = block(rank)
    rp = S.indptr.astype(np.int64)
    c = (S.indices + b).astype(np.int32)  # global columns
    M = eigmi.Matrix.from_rows(ctx, n, b, rp, c, S.data)
    out = {"nranks": ctx.comm_info()["nranks"], "march_variant": M.info.march_variant,
           "halo": int(M.info.halo_recv + M.info.halo_send)}
    if mode == "stall":
        ctx.select_allreduce("mailbox-step")
        ws = eigmi.LanczosWorkspace(M, 40, seed=123, fused=True)
        if rank == 0:
            t0 = time.perf_counter()
            try:
                ws.step(5)
                out["code"] = 0
            except eigmi.EigError as e:
                out["code"] = e.code
                out["msg"] = str(e)
            out["seconds"] = time.perf_counter() - t0
            out["errors"] = ctx.comm_info()["mailbox_errors"]
            publish(wd, "done")
        else:
            wait_for([os.path.join(wd, "done")], timeout=200.0)
        np.savez(os.path.join(wd, f"r{rank}.npz"), **out)
        # (no close of ws / M: rank 0's poisoned exchange has nothing left to run; the process ends)
        return
    if mode == "stall_tridiag":
        # both ranks take 5 steps together; then only rank 0 asks for T: its forced final repair
        # launch exchanges the sums in-kernel with a peer that never launches it
        ctx.select_allreduce("mailbox-step")
        ws = eigmi.LanczosWorkspace(M, 40, seed=123, fused=True)
        ws.step(5)
        if rank == 0:
            t0 = time.perf_counter()
            try:
                ws.tridiag()
                out["code"] = 0
            except eigmi.EigError as e:
                out["code"] = e.code
                out["msg"] = str(e)
            out["seconds"] = time.perf_counter() - t0
            out["errors"] = ctx.comm_info()["mailbox_errors"]
            publish(wd, "done")
        else:
            wait_for([os.path.join(wd, "done")], timeout=200.0)
        np.savez(os.path.join(wd, f"r{rank}.npz"), **out)
        return
    for tr in ("mailbox", "mailbox-step"):
        ctx.select_allreduce(tr)
        assert ctx.comm_info()["allreduce"] == {"mailbox": "xgmi-mailbox", "mailbox-step": "xgmi-mailbox-step"}[tr]
        ws = eigmi.LanczosWorkspace(M, sum(STEPS) + 2, seed=123, fused=True)
        ws.step(STEPS[0])
        out[f"captured_{tr}"] = ws.capture(STEPS[1])
        ws.replay()
        ws.step(STEPS[2])
        a, bb = ws.tridiag()
        k, L = ws.info()
        ws.close()
        out[f"alpha_{tr}"], out[f"beta_{tr}"], out[f"launches_{tr}"] = a, bb, L
    # pipelined workspaces keep the mailbox allreduce launch on the reduction stream under the step mode
    ws = eigmi.LanczosWorkspace(M, 22, seed=123, pipelined=True)
    ws.step(20)
    out["alpha_pipe"], out["beta_pipe"] = ws.tridiag()
    ws.close()
    out["errors"] = ctx.comm_info()["mailbox_errors"]
    np.savez(os.path.join(wd, f"r{rank}.npz"), **out)
    M.close()
    ctx.close()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4])
