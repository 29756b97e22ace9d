"""CPU (gloo) tests of the N > 1 path: the row partition, the window / halo plan computed by
libeigmi's own host code (eig_plan_window, eig_plan_halo -- the functions
eig_mat_create_bcsr_dist uses), and the distributed Lanczos recurrence (halo exchange before the
SpMV, one allreduce after each fused kernel) reproduce the serial oracle.

Each rank runs the per-rank arithmetic with the oracle's CSR SpMV on its window-local rows, and
exchanges halos / dots with gloo send / recv / all_reduce exactly where the device path issues
ncclSend / ncclRecv / ncclAllReduce (drivers.cpp: lanczos_step)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, N, steps, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import eigmi
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = N ** 3
        b, cnt = eigmi.row_partition(n, world, rank, align=N * N)
        rp, c, v = eigmi.gen_rows(eigmi.GEN_POISSON3D, N, b, cnt)
        wb, wlen, own, cmin, cmax = eigmi.plan_window(b, cnt, rp, c)
        mine = torch.tensor([b, cnt, cmin, cmax], dtype=torch.int64)
        allr = [torch.zeros(4, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allr, mine)
        ranks = torch.stack(allr).numpy()
        recvs, sends = eigmi.plan_halo(world, rank, ranks, wb)
        cl = (c[:rp[-1]] - wb).astype(np.int32)  # window-local columns, as build_sell stores them
        assert cl.min() >= 0 and cl.max() < wlen

        def halo(x):
            reqs = []
            bufs = []
            for peer, off, count in sends:
                reqs.append(dist.isend(torch.from_numpy(x[off:off + count].copy()), peer))
            for peer, off, count in recvs:
                t = torch.zeros(count, dtype=torch.float64)
                bufs.append((off, count, t))
                reqs.append(dist.irecv(t, peer))
            for r in reqs:
                r.wait()
            for off, count, t in bufs:
                x[off:off + count] = t.numpy()

        def allreduce(val):
            t = torch.tensor([val], dtype=torch.float64)
            dist.all_reduce(t)
            return float(t.item())

        full0 = oracle.random_vec(n, 123)
        U = [np.zeros(wlen) for _ in range(3)]
        U[0][own:own + cnt] = full0[b:b + cnt]
        nsum = [allreduce(float(np.dot(U[0][own:own + cnt], U[0][own:own + cnt])))]
        alpha, beta = [], []
        for j in range(steps):
            u, up, t = U[j % 3], U[(j + 2) % 3], U[(j + 1) % 3]
            halo(u)
            bj = np.sqrt(nsum[j])
            sig = 1.0 / bj
            gam = bj * (1.0 / np.sqrt(nsum[j - 1])) if j > 0 else 0.0
            acc = np.zeros(cnt)
            oracle.lib.orc_csr_mv(cnt, rp, cl, v, u, acc)
            tl = acc * sig
            if j > 0:
                tl = tl - gam * up[own:own + cnt]
            t[own:own + cnt] = tl
            d = allreduce(float(np.dot(tl, u[own:own + cnt])))
            a = sig * d
            t[own:own + cnt] = tl - (a * sig) * u[own:own + cnt]
            nsum.append(allreduce(float(np.dot(t[own:own + cnt], t[own:own + cnt]))))
            alpha.append(a)
            beta.append(bj)
        beta.append(np.sqrt(nsum[steps]))
        q.put((rank, np.array(alpha), np.array(beta), [(p, cnt_) for p, _, cnt_ in recvs]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_lanczos_matches_serial_oracle(world):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    N, steps = 12, 25
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = oracle.poisson3d(N)
    _, ra, rb = oracle.lanczos(A, oracle.random_vec(A.n, 123), steps)
    for rank, alpha, beta, recv in res:
        assert np.allclose(alpha, ra, rtol=1e-12), rank
        assert np.allclose(beta, rb, rtol=1e-12), rank
        peers = sorted(p for p, _ in recv)
        assert peers == [x for x in (rank - 1, rank + 1) if 0 <= x < world]
        assert all(c == N * N for _, c in recv)  # one z-plane per neighbour
