"""The halo exchange over the xGMI mailbox between processes on one GPU (halo and
the in-kernel exchange had run together only on the in-process loopback transport).  P = 2, 3
mailbox-only ranks (eig_comm_ipc_open, no RCCL), each owning a z-slab of the global matrix, so every
interface carries a full plane of ghost rows; tests/halo_mailbox_worker.py runs one rank.

Against the CPU restatement on the GLOBAL matrix (oracle/oracle.cc, the checker only):
  * eig_mv BITWISE oracle.csr_mv (kernels_cpp.hh:596-621);
  * fused steps within rtol 1e-12 of orc_lanczos_fused on the value march and on the SELL image,
    split and whole halo launches, the mailbox allreduce launch and the in-kernel exchange, eager and
    replayed from a hipGraph -- the in-kernel exchange BITWISE the allreduce launch (both sum the
    slots in rank order), BITWISE the same runs over the in-process loopback transport (device-copy
    halo, host allreduce), and every rank holding the same coefficients;
  * the classic and pipelined steps within 1e-12 of their restatements;
  * C5's block Lanczos (P1 K / M, block 16, exchanges of 8-column blocks) within 1e-10 of the
    single-rank run.
A peer that never exchanges: the pull times out within seconds, the ghosts read NaN and the mailbox's
error word is set (no hang).  The reference has no distribution (src/dune-eigensolver.cc:742-748):
SURVEY 8(e)."""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

import eigmi
import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import halo_mailbox_worker as W  # noqa: E402


def _spawn(P, wd, mode):
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "halo_mailbox_worker.py"), str(r), str(P),
                               wd, mode], stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(P)]
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(out.decode(errors="replace"))
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-3000:]}"
    return [np.load(os.path.join(wd, f"r{r}.npz")) for r in range(P)]


def _loopback_runs(P):
    """The same slabs and fused runs over the in-process loopback transport (device copies for the halo,
    a host sum in rank order for the allreduce): {(name, halo): (alpha, beta)} of every rank."""
    n, D = W.N ** 3, W.N * W.N
    hub = eigmi.loopback_create(P)
    out = [None] * P

    def rank(r):
        c = eigmi.Context(0)
        res = {}
        try:
            c.comm_init_loopback(hub, r)
            b, cnt = W.slab(W.N, D, P, r)
            rp, col, v = eigmi.gen_rows(eigmi.GEN_VARCOEF3D, W.N, b, cnt)
            for name, flags in (("march", 0), ("sell", eigmi.MAT_NO_BAND)):
                A = eigmi.Matrix.from_rows(c, n, b, rp, col, v, flags=flags)
                for halo in ("split", "whole"):
                    A.tune(halo_whole=int(halo == "whole"))
                    a, be, _ = eigmi.lanczos_run(A, W.STEPS, seed=123, fused=True)
                    res[(name, halo)] = (a, be)
                A.close()
        except Exception as e:  # noqa: BLE001 -- reported below
            res["error"] = repr(e)
        finally:
            c.close()
        out[r] = res
    th = [threading.Thread(target=rank, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    eigmi.loopback_destroy(hub)
    return out


def _rel(a, ref):
    return float(np.max(np.abs(a - ref) / np.abs(ref)))


@pytest.mark.parametrize("P", [2, 3])
def test_halo_mailbox_processes(tmp_path, P):
    res = _spawn(P, str(tmp_path), "run")
    n = W.N ** 3
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_VARCOEF3D, W.N)
    A = oracle.CSR(n, rp, c, v)
    x = np.random.default_rng(21).standard_normal(n)
    y_ref = oracle.csr_mv(A, x)
    u0 = oracle.random_vec(n, 123)
    ra, rb = oracle.lanczos_fused(A, u0, W.STEPS)
    _, ka, kb = oracle.lanczos(A, u0, 20)
    pa, pb = oracle.lanczos_fused(A, u0, 20, pipelined=True)
    worst = 0.0
    for r, d in enumerate(res):
        b, cnt = int(d["row_begin"]), int(d["rows"])
        assert int(d["nranks"]) == P and int(d["errors"]) == 0
        D = W.N * W.N
        assert int(d["halo_recv"]) == D * ((r > 0) + (r < P - 1)) == int(d["halo_send"])
        assert int(d["march_variant"]) == 15
        assert np.array_equal(d["y"], y_ref[b:b + cnt]), f"rank {r}: eig_mv not bitwise the oracle row loop"
        for name in ("march", "sell"):
            for tr in ("mailbox", "mailbox-step"):
                for mode in ("split", "whole", "graph"):
                    a, be = d[f"a_{name}_{tr}_{mode}"], d[f"b_{name}_{tr}_{mode}"]
                    da, db = _rel(a, ra), _rel(be[1:], rb[1:])
                    worst = max(worst, da, db)
                    assert da <= 1e-12 and db <= 1e-12, (r, name, tr, mode, da, db)
                    # every rank holds the same coefficients
                    assert np.array_equal(a, res[0][f"a_{name}_{tr}_{mode}"])
                assert bool(d[f"captured_{name}_{tr}"]), (name, tr)
                # the in-kernel exchange sums the same slots in the same order as the allreduce launch
                for mode in ("split", "whole", "graph"):
                    assert np.array_equal(d[f"a_{name}_mailbox-step_{mode}"], d[f"a_{name}_mailbox_{mode}"])
                    assert np.array_equal(d[f"b_{name}_mailbox-step_{mode}"], d[f"b_{name}_mailbox_{mode}"])
        assert str(d["sell_kernel"]).startswith("k_lanczos_fused_b1"), d["sell_kernel"]
        assert _rel(d["a_pipe"], pa) <= 1e-12 and _rel(d["b_pipe"][1:], pb[1:]) <= 1e-12
        assert np.allclose(d["a_classic"], ka, rtol=1e-12, atol=0) and np.allclose(d["b_classic"][:20], kb[:20],
                                                                                   rtol=1e-12, atol=0)
        assert np.allclose(d["ritz_dist"], d["ritz_serial"], rtol=1e-10, atol=0), (d["ritz_dist"], d["ritz_serial"])
        cnt_ = d["counters"]
        assert int(cnt_[0]) == 0 and int(cnt_[2]) > 0, cnt_  # no RCCL allreduce; halo groups exchanged
    # bitwise the loopback transport: the halo moves exact copies and both allreduces sum the ranks'
    # values in rank order, so the transport must not change a bit
    lb = _loopback_runs(P)
    for r, d in enumerate(res):
        assert "error" not in lb[r], lb[r]
        for (name, halo), (a, be) in lb[r].items():
            assert np.array_equal(d[f"a_{name}_mailbox_{halo}"], a), (r, name, halo)
            assert np.array_equal(d[f"b_{name}_mailbox_{halo}"], be), (r, name, halo)
    if P == 3:
        # the matrix coupling ranks 0 and 1 only, run first: exchange counters per pair of ranks
        G, cuts = W.partial_matrix()
        Ap = oracle.CSR(G.shape[0], G.indptr.astype(np.int64), G.indices.astype(np.int32), G.data)
        xq = np.random.default_rng(5).standard_normal(G.shape[0])
        yq = oracle.csr_mv(Ap, xq)
        qa, qb = oracle.lanczos_fused(Ap, oracle.random_vec(Ap.n, 123), 20)
        for r, d in enumerate(res):
            assert int(d["partial_halo"]) == (256 if r < 2 else 0)
            assert np.array_equal(d["partial_y"], yq[cuts[r]:cuts[r + 1]]), r
            assert _rel(d["partial_a"], qa) <= 1e-12 and _rel(d["partial_b"][1:], qb[1:]) <= 1e-12, r
    print(f"P={P}: worst rel diff vs orc_lanczos_fused {worst:.2e}; Ritz {res[0]['ritz_dist']}")


def test_halo_mailbox_peer_never_arrives(tmp_path):
    res = _spawn(2, str(tmp_path), "stall")
    d = res[0]
    print(f"stalled peer: {int(d['nan_rows'])} NaN rows after {float(d['seconds']):.2f} s")
    assert float(d["seconds"]) < 60.0 and int(d["errors"]) == 1
    assert int(d["nan_rows"]) > 0
