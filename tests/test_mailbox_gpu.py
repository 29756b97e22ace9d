"""The xGMI mailbox allreduce (k_comm.hip) across real processes: P ranks on the one GPU of the
test box, each its own process and context, attached through eig_comm_ipc_handle / _open (IPC
mappings of each other's uncached mailboxes -- the same mechanism eig_comm_init uses between
GPUs).  Checks: every allreduce returns the rank-order sum bitwise (identical on all ranks),
100-value calls (two mailbox rounds), 300 back-to-back calls through the parity buffers, a
distributed dot, and no timeouts."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mailbox_worker  # noqa: E402


def expected(P):
    out = []
    for it in range(mailbox_worker.ROUNDS):
        vs = [mailbox_worker.values(r, it) for r in range(P)]
        s = np.zeros_like(vs[0])
        for v in vs:  # rank order, one rounding per addition: what every rank computes
            s = s + v
        out.append(s)
    return np.concatenate(out)


@pytest.mark.parametrize("P", [2, 3])
def test_mailbox_allreduce_processes(tmp_path, P):
    wd = str(tmp_path)
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mailbox_worker.py"), str(r), str(P), wd],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(P)]
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
    want = expected(P)
    n = 1 << 16
    x = np.random.default_rng(7).standard_normal(n)
    res = [np.load(os.path.join(wd, f"r{r}.npz")) for r in range(P)]
    print(f"P={P}: mailbox allreduce {[round(float(d['us']), 2) for d in res]} us/call (one GPU, processes)")
    for r, d in enumerate(res):
        assert str(d["allreduce"]) == "xgmi-mailbox" and int(d["nranks"]) == P
        assert int(d["errors"]) == 0
        assert np.array_equal(d["flat"], want), f"rank {r}: allreduce differs from the rank-order sum"
        assert float(d["dot"]) == float(res[0]["dot"])
        assert abs(float(d["dot"]) - float(x @ x)) <= 1e-12 * float(x @ x)
