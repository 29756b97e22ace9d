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


def _pipelined(rank, cnt, own, wlen, rp, cl, v, b, full0, steps, halo, oracle):
    """Per-rank pipelined one-reduction recurrence (orc_lanczos_pipelined / k_lanczos_pipe,
    DESIGN.md 6): launch L computes S = A t_{k-1} after the halo of T while launch L-1's three sums
    are still being allreduced (gloo async_op, waited only before the row update); the row update
    applies the scalars (fused_begin's modes: step, repair, post) and issues its own allreduce.
    Returns alpha[steps], beta[steps + 1] (final beta exact: the forced repair)."""
    import torch
    import torch.distributed as dist
    STEP, POST, HALT, REPAIR = 0, 1, 2, 3
    diag = 0.0
    for i in range(cnt):
        for p in range(rp[i], rp[i + 1]):
            if cl[p] == own + i:
                diag += v[p]
    mu2 = torch.tensor([diag, float(cnt)], dtype=torch.float64)
    dist.all_reduce(mu2)
    mu = float(mu2[0] / mu2[1])
    T = np.zeros(wlen)
    T[own:own + cnt] = full0[b:b + cnt]
    U, Z = np.zeros(cnt), np.zeros(cnt)
    t0 = torch.tensor([float(np.dot(T[own:own + cnt], T[own:own + cnt]))], dtype=torch.float64)
    dist.all_reduce(t0)
    nsum = [0.0] * (steps + 2)
    nsum[0] = float(t0.item())
    alpha, beta = np.zeros(steps), np.zeros(steps + 1)
    beta[0] = np.sqrt(nsum[0])
    st = {"j": 0, "mode": STEP, "red": np.zeros(3), "aux": (0.0, 0.0), "pend": None}

    def launch(force):
        halo(T)
        S = np.zeros(cnt)
        oracle.lib.orc_csr_mv(cnt, rp, cl, v, T, S)
        if st["pend"] is not None:  # launch L-1's allreduce completes only now
            st["pend"][0].wait()
            st["red"] = st["pend"][1].numpy().copy()
            st["pend"] = None
        j, mode, (d, q, m) = st["j"], st["mode"], st["red"]
        c = ap = bk = gam = rn = rm = 0.0
        nt = 1.0
        if mode == POST:
            rn, rm = st["aux"]
            nt = m
            act = HALT if not m > 0.0 else POST
            if act == POST:
                bk = np.sqrt(m) * rn / rm
                gam = bk / rm
        elif j == 0:
            nt, act = nsum[0], STEP
        else:
            rn, rm = np.sqrt(nsum[j - 1]), np.sqrt(m)
            c = d / m
            ap = c * rn + mu
            nt = q - c * d
            if force or not nt > 1e-2 * q:
                act = REPAIR
            else:
                bk = np.sqrt(nt) * rn / rm
                gam = bk / rm
                act = STEP
        sig = 1.0 / np.sqrt(nt)
        t = T[own:own + cnt]
        if act == HALT:
            st["mode"] = HALT
            return
        if act == REPAIR:
            alpha[j - 1] = ap
            st["aux"] = (rn, rm)
            u = t - c * U
            T[own:own + cnt] = u
            sums = [0.0, 0.0, float(np.dot(u, u))]
            st["mode"] = POST
        else:
            if act == POST:
                nsum[j], beta[j] = nt, bk
            elif j > 0:
                nsum[j], alpha[j - 1], beta[j] = nt, ap, bk
            u = t - c * U
            z = S - c * Z
            tn = (z - mu * u) * sig
            if j > 0:
                tn = tn - gam * U
            T[own:own + cnt] = tn
            U[:], Z[:] = u, z
            sums = [float(np.dot(tn, u)), float(np.dot(tn, tn)), float(np.dot(u, u))]
            st["j"], st["mode"] = j + 1, STEP
        r = torch.tensor(sums, dtype=torch.float64)
        st["pend"] = (dist.all_reduce(r, async_op=True), r)

    while st["j"] < steps and st["mode"] != HALT:
        launch(False)
    if st["mode"] == STEP and st["j"] > 0:
        launch(True)
    st["pend"][0].wait()
    m = float(st["pend"][1][2])
    rn, rm = st["aux"]
    beta[st["j"]] = np.sqrt(m) * rn / rm
    return alpha, beta


def _worker(rank, world, port, N, steps, q, variant="classic"):
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
        if variant == "pipelined":
            alpha, beta = _pipelined(rank, cnt, own, wlen, rp, cl, v, b, full0, steps, halo, oracle)
            q.put((rank, alpha, beta, [(p, cnt_) for p, _, cnt_ in recvs]))
            return
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


@pytest.mark.parametrize("variant", ["classic", "pipelined"])
@pytest.mark.parametrize("world", [2, 3])
def test_distributed_lanczos_matches_serial_oracle(world, variant):
    """classic: two allreduces per step, vs orc_lanczos.  pipelined: the allreduce of launch L
    overlaps launch L+1's halo + SpMV (async gloo), vs the serial restatement orc_lanczos_pipelined
    (1e-12) and the classic recurrence (1e-11, the fused/classic spread of test_oracle)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    N, steps = 12, 25
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, steps, q, variant)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = oracle.poisson3d(N)
    u0 = oracle.random_vec(A.n, 123)
    _, ra, rb = oracle.lanczos(A, u0, steps)
    if variant == "pipelined":
        pa, pb = oracle.lanczos_fused(A, u0, steps, pipelined=True)
    for rank, alpha, beta, recv in res:
        if variant == "pipelined":
            assert np.allclose(alpha, pa, rtol=1e-12, atol=0), rank
            assert np.allclose(beta, pb, rtol=1e-12, atol=0), rank
            assert np.allclose(alpha, ra, rtol=1e-11, atol=0) and np.allclose(beta, rb, rtol=1e-11, atol=0), rank
        else:
            assert np.allclose(alpha, ra, rtol=1e-12), rank
            assert np.allclose(beta, rb, rtol=1e-12), rank
        peers = sorted(p for p, _ in recv)
        assert peers == [x for x in (rank - 1, rank + 1) if 0 <= x < world]
        assert all(c == N * N for _, c in recv)  # one z-plane per neighbour
