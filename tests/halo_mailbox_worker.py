"""One rank of tests/test_halo_mailbox_gpu.py: a row partition WITH a halo between real processes on
one GPU, every exchange over the xGMI mailbox (eig_comm_ipc_handle / _open, no RCCL): the ghost rows
through the halo mailbox (k_comm.hip k_halo_push / k_halo_pull), the sums through the mailbox
allreduce launch or inside the step kernel (EIG_AR_MAILBOX_STEP).

The global matrices are eig_gen's 3-D boxes split into z-slabs (rank r owns planes N r / P ..
N (r + 1) / P), so every interface carries a full plane of ghosts:
  * the variable-coefficient 7-point matrix (the value march, variant 15) and the same rows in the
    SELL image (EIG_MAT_NO_BAND: interior / boundary slices), eig_mv and fused Lanczos steps under
    split and whole halo launches, eager and captured into a hipGraph;
  * the classic two-reduction step and the pipelined step;
  * generalised block Lanczos (config C5) on the variable-coefficient P1 K / M pencil, block 16: the
    exchanges of 8-column blocks (width 8).

    python tests/halo_mailbox_worker.py RANK NRANKS WORKDIR MODE
With P = 3 the run starts on a matrix that couples ranks 0 and 1 only (rank 2 owns a separate block:
it takes no part in that matrix's exchanges), so the exchange counters are per pair of ranks -- the
z-slab matrices after it would otherwise wait for numbers rank 2 never published.

MODE "run": everything above, saved to r<RANK>.npz (with the rank's serial block Lanczos Ritz values,
computed on a second context without a transport).
MODE "stall": rank 0 calls eig_mv while rank 1 never exchanges (it waits for rank 0's "done" file):
rank 0's pull must time out within seconds, the ghosts read NaN and the error word is set.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import eigmi  # noqa: E402
from mailbox_step_worker import publish, wait_for  # noqa: E402

N = 64       # the 7-point boxes: 64^3 (grid lines of 64 rows: the value march applies)
NB = 16      # the P1 pencil: 16^3
STEPS = 40
BLOCK, BSTEPS, BNEV = 16, 5, 4


def box7(nz, seed, nx=64, ny=4):
    """A random symmetric diagonally dominant 7-point box nx x ny x nz (scipy CSR)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    n = nx * ny * nz
    idx = np.arange(n)
    x, y, z = idx % nx, (idx // nx) % ny, idx // (nx * ny)
    rows, cols, vals = [idx], [idx], [6.0 + rng.random(n)]
    for step, ok in ((1, x < nx - 1), (nx, y < ny - 1), (nx * ny, z < nz - 1)):
        i = idx[ok]
        w = -0.5 - rng.random(i.size)
        rows += [i, i + step]
        cols += [i + step, i]
        vals += [w, w]
    S = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    S.sort_indices()
    return S


def partial_matrix():
    """Ranks 0 and 1 split a 64 x 4 x 12 box (6 planes each, coupled), rank 2 owns a 64 x 4 x 6 box."""
    import scipy.sparse as sp
    G = sp.block_diag([box7(12, 7), box7(6, 8)], format="csr")
    G.sort_indices()
    return G, [0, 6 * 256, 12 * 256, 18 * 256]


def slab(n_planes, D, P, r):
    p0, p1 = n_planes * r // P, n_planes * (r + 1) // P
    return p0 * D, (p1 - p0) * D


def block_ritz(ctx, Nb, b, cnt, dist):
    n = Nb ** 3
    mats = []
    for kind in (eigmi.GEN_P1STIFF3D_VAR, eigmi.GEN_P1MASS3D_VAR):
        rp, c, v = eigmi.gen_rows(kind, Nb, b, cnt)
        mats.append(eigmi.Matrix.from_rows(ctx, n, b, rp, c, v) if dist else
                    eigmi.Matrix.from_bcsr(ctx, rp, c, v))
    bl = eigmi.BlockLanczos(mats[0], mats[1], block=BLOCK, max_steps=BSTEPS, degree=36, lmin=0.5, lmax=2.5, seed=123)
    bl.step(BSTEPS)
    ev, _, _ = bl.ritz(BNEV, which=eigmi.WHICH_LA, want_resid=False)
    bl.close()
    for m in mats:
        m.close()
    return ev


def main(rank, P, wd, mode):
    ctx = eigmi.Context(0)
    publish(wd, f"h{rank}.bin", ctx.ipc_handle(P, rank))
    paths = [os.path.join(wd, f"h{r}.bin") for r in range(P)]
    wait_for(paths)
    ctx.ipc_open(b"".join(open(p, "rb").read() for p in paths))
    n, D = N ** 3, N * N
    b, cnt = slab(N, D, P, rank)
    x = np.random.default_rng(21).standard_normal(n)
    rp, c, v = eigmi.gen_rows(eigmi.GEN_VARCOEF3D, N, b, cnt)
    M = eigmi.Matrix.from_rows(ctx, n, b, rp, c, v)
    out = {"nranks": ctx.comm_info()["nranks"], "row_begin": b, "rows": cnt, "march_variant": M.info.march_variant,
           "halo_recv": int(M.info.halo_recv), "halo_send": int(M.info.halo_send)}
    if mode == "stall":
        if rank == 0:
            xv, yv = M.window_vector(x[b:b + cnt]), M.window_vector()
            t0 = time.perf_counter()
            M.mv(xv, yv)
            y = M.owned(yv)
            out["seconds"] = time.perf_counter() - t0
            out["nan_rows"] = int(np.isnan(y).sum())
            out["errors"] = ctx.comm_info()["mailbox_errors"]
            publish(wd, "done")
        else:
            wait_for([os.path.join(wd, "done")], timeout=200.0)
        np.savez(os.path.join(wd, f"r{rank}.npz"), **out)
        return
    if P == 3:
        # first a matrix whose exchanges involve ranks 0 and 1 only
        G, cuts = partial_matrix()
        gb, ge = cuts[rank], cuts[rank + 1]
        Gr = G[gb:ge]
        Q = eigmi.Matrix.from_rows(ctx, G.shape[0], gb, Gr.indptr.astype(np.int64), Gr.indices.astype(np.int32),
                                   Gr.data)
        out["partial_halo"] = int(Q.info.halo_recv)
        xq = np.random.default_rng(5).standard_normal(G.shape[0])
        qx, qy = Q.window_vector(xq[gb:ge]), Q.window_vector()
        Q.mv(qx, qy)
        out["partial_y"] = Q.owned(qy)
        qx.free()
        qy.free()
        ctx.select_allreduce("mailbox")
        out["partial_a"], out["partial_b"], _ = eigmi.lanczos_run(Q, 20, seed=123, fused=True)
        Q.close()
    # eig_mv: the window vector's ghosts through the halo mailbox, interior planes overlapped
    xv, yv = M.window_vector(x[b:b + cnt]), M.window_vector()
    M.mv(xv, yv)
    out["y"] = M.owned(yv)
    xv.free()
    yv.free()
    S = eigmi.Matrix.from_rows(ctx, n, b, rp, c, v, flags=eigmi.MAT_NO_BAND)
    out["sell_kernel"] = S.lanczos_kernel_info(True)[0]
    for name, A in (("march", M), ("sell", S)):
        for tr in ("mailbox", "mailbox-step"):
            ctx.select_allreduce(tr)
            for halo in ("split", "whole"):
                A.tune(halo_whole=int(halo == "whole"))
                a, be, _ = eigmi.lanczos_run(A, STEPS, seed=123, fused=True)
                out[f"a_{name}_{tr}_{halo}"], out[f"b_{name}_{tr}_{halo}"] = a, be
            A.tune(halo_whole=0)
            # captured: the halo mailbox's sequence number lives on the device, so replays exchange anew
            ws = eigmi.LanczosWorkspace(A, STEPS + 2, seed=123, fused=True)
            ws.step(6)
            out[f"captured_{name}_{tr}"] = ws.capture(STEPS - 12)
            ws.replay()
            ws.step(6)
            a, be = ws.tridiag()
            ws.close()
            out[f"a_{name}_{tr}_graph"], out[f"b_{name}_{tr}_graph"] = a, be
    ctx.select_allreduce("mailbox")
    a, be, _ = eigmi.lanczos_run(M, 20, seed=123)
    out["a_classic"], out["b_classic"] = a, be
    a, be, _ = eigmi.lanczos_run(M, 20, seed=123, pipelined=True)
    out["a_pipe"], out["b_pipe"] = a, be
    S.close()
    M.close()
    # C5's block Lanczos on the P1 pencil, distributed, and the same on one rank for comparison
    bb, bcnt = slab(NB, NB * NB, P, rank)
    out["ritz_dist"] = block_ritz(ctx, NB, bb, bcnt, True)
    out["counters"] = np.array(list(ctx.comm_counters().values()))
    out["errors"] = ctx.comm_info()["mailbox_errors"]
    serial = eigmi.Context(0)
    out["ritz_serial"] = block_ritz(serial, NB, 0, NB ** 3, False)
    serial.close()
    np.savez(os.path.join(wd, f"r{rank}.npz"), **out)
    ctx.close()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4])
