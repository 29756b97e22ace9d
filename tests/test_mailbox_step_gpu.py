"""The fused Lanczos step's allreduce inside the step kernel (EIG_AR_MAILBOX_STEP, csrc/xch_dev.h;
VERDICT r4 next #3): the last workgroup of launch L publishes the three sums to every peer's xGMI
mailbox and gathers theirs before the kernel ends, with no allreduce launch between two steps.

* One rank (a one-rank RCCL communicator + mailbox, EIG_COMM_ALWAYS): a one-rank sum is the
  identity, so alpha / beta under rccl, mailbox and mailbox-step must be BITWISE those of the run
  without a communicator -- on the benchmark's value march (variant 15, the geometric prologue under
  the first plane loads), the SELL / stencil image (k_lanczos_fused_b1) and the P1 Kuhn march
  (variant 20); eager batches, a hipGraph replay and the forced final repair (exact beta).
* Processes on one GPU (P = 2, 3; a block-diagonal matrix, rank r owning one random 7-point box, so
  no halo): mailbox-step BITWISE equal to the mailbox allreduce launch (both sum the slots in rank
  order), and within 1e-12 of the serial restatement orc_lanczos_fused on the global matrix.
* A peer that never steps: the exchange times out (bounded polling), the step call returns
  EIG_ERR_RCCL within seconds instead of hanging.
The reference has no distribution (src/dune-eigensolver.cc:742-748): SURVEY 8(e), north_star."""
import os
import subprocess
import sys

import numpy as np
import pytest

import eigmi
import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mailbox_step_worker as W  # noqa: E402


@pytest.fixture(scope="module")
def mb_ctx():
    c = eigmi.Context(0)
    c.comm_init(1, 0, eigmi.Context.unique_id(), mailbox=True, always=True)
    yield c
    c.close()


def _mats():
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_VARCOEF3D, 64)
    yield "varcoef64", (rp, c, v), 0, 15
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, 64)
    yield "poisson64_arrays", (rp, c, v), eigmi.MAT_NO_UNIFORM, 15
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_POISSON3D, 32)
    yield "poisson32_sell", (rp, c, v), eigmi.MAT_NO_BAND, -1
    rp, c, v = eigmi.gen_matrix(eigmi.GEN_P1STIFF3D_VAR, 64)
    yield "p1var64", (rp, c, v), 0, 20


def _run(ctx, mat, flags, variant, graph):
    M = eigmi.Matrix.from_bcsr(ctx, *mat, flags=flags)
    ws = eigmi.LanczosWorkspace(M, 40, seed=123, fused=variant == "fused", pipelined=variant == "pipelined")
    try:
        ws.step(4)
        if graph:
            ws.capture(20)
            ws.replay()
        else:
            ws.step(20)
        ws.step(3)
        a, b = ws.tridiag()
        mv = M.info.march_variant
    finally:
        ws.close()
        M.close()
    return a, b, mv


@pytest.mark.parametrize("name,mat,flags,mv", list(_mats()), ids=[m[0] for m in _mats()])
def test_step_exchange_one_rank_bitwise(ctx, mb_ctx, name, mat, flags, mv):
    ref = _run(ctx, mat, flags, "fused", False)
    assert ref[2] == mv
    for tr in ("rccl", "mailbox", "mailbox-step"):
        mb_ctx.select_allreduce(tr)
        for graph in (False, True):
            a, b, _ = _run(mb_ctx, mat, flags, "fused", graph)
            assert np.array_equal(a, ref[0]) and np.array_equal(b, ref[1]), (tr, graph)
        assert mb_ctx.comm_info()["mailbox_errors"] == 0
    # the pipelined step keeps the mailbox allreduce launch under the step mode
    pref = _run(ctx, mat, flags, "pipelined", False)
    a, b, _ = _run(mb_ctx, mat, flags, "pipelined", False)
    assert np.array_equal(a, pref[0]) and np.array_equal(b, pref[1])
    assert mb_ctx.comm_info()["allreduce"] == "xgmi-mailbox-step"
    mb_ctx.select_allreduce("rccl")


def test_select_halo_one_rank(ctx, mb_ctx):
    """eig_comm_select_halo: accepted on a context with RCCL and the mailbox (one rank: no halo to move,
    the recurrence bitwise unchanged), refused without RCCL."""
    mat = list(_mats())[1]
    ref = _run(ctx, mat[1], mat[2], "fused", False)
    mb_ctx.select_allreduce("mailbox")
    for hx in ("mailbox", "rccl"):
        mb_ctx.select_halo(hx)
        a, b, _ = _run(mb_ctx, mat[1], mat[2], "fused", True)
        assert np.array_equal(a, ref[0]) and np.array_equal(b, ref[1]), hx
    mb_ctx.select_allreduce("rccl")
    with pytest.raises(eigmi.EigError):
        ctx.select_halo("mailbox")  # no transport at all


def _spawn(P, wd, mode):
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mailbox_step_worker.py"), str(r), str(P),
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


@pytest.mark.parametrize("P", [2, 3])
def test_step_exchange_processes(tmp_path, P):
    res = _spawn(P, str(tmp_path), "run")
    G = W.global_matrix(P)
    A = oracle.CSR(G.shape[0], G.indptr.astype(np.int64), G.indices.astype(np.int32), G.data)
    k = sum(W.STEPS)
    ra, rb = oracle.lanczos_fused(A, oracle.random_vec(A.n, 123), k)
    for r, d in enumerate(res):
        assert int(d["nranks"]) == P and int(d["halo"]) == 0 and int(d["errors"]) == 0
        a, b = d["alpha_mailbox-step"], d["beta_mailbox-step"]
        # the same rank-order sums as the mailbox allreduce launch: bitwise
        assert np.array_equal(a, d["alpha_mailbox"]) and np.array_equal(b, d["beta_mailbox"]), r
        assert int(d["launches_mailbox-step"]) == int(d["launches_mailbox"])
        assert bool(d["captured_mailbox-step"])
        # and every rank holds the same coefficients
        assert np.array_equal(a, res[0]["alpha_mailbox-step"]) and np.array_equal(b, res[0]["beta_mailbox-step"])
        assert np.allclose(a, ra, rtol=1e-12, atol=0) and np.allclose(b, rb, rtol=1e-12, atol=0), r
        pa, pb = oracle.lanczos_fused(A, oracle.random_vec(A.n, 123), 20, pipelined=True)
        assert np.allclose(d["alpha_pipe"], pa, rtol=1e-12, atol=0) and np.allclose(d["beta_pipe"], pb, rtol=1e-12, atol=0)
    print(f"P={P}: march variant {[int(d['march_variant']) for d in res]}, {k} steps, "
          f"max rel diff vs restatement {np.max(np.abs(res[0]['alpha_mailbox-step'] - ra) / np.abs(ra)):.2e}")


def test_step_exchange_peer_never_arrives(tmp_path):
    res = _spawn(2, str(tmp_path), "stall")
    d = res[0]
    print(f"stalled peer: code {int(d['code'])} after {float(d['seconds']):.2f} s ({d['msg'] if 'msg' in d else ''})")
    assert int(d["code"]) == eigmi.EIG_ERR_RCCL
    assert float(d["seconds"]) < 60.0 and int(d["errors"]) == 1


def test_step_exchange_peer_never_arrives_in_tridiag(tmp_path):
    """eig_lanczos_tridiag's forced final repair launch exchanges its sums in-kernel; a peer
    that never launches it must make the call return EIG_ERR_RCCL after the bounded poll."""
    res = _spawn(2, str(tmp_path), "stall_tridiag")
    d = res[0]
    print(f"stalled peer in tridiag: code {int(d['code'])} after {float(d['seconds']):.2f} s "
          f"({d['msg'] if 'msg' in d else ''})")
    assert int(d["code"]) == eigmi.EIG_ERR_RCCL
    assert float(d["seconds"]) < 60.0 and int(d["errors"]) == 1
