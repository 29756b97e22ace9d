"""Config C4 (3-D Poisson 256^3 row-partitioned) at its own size on one GPU: P = 2, 4, 8
virtual ranks over the loopback hub, each running the benchmark's step kernel on its z-slab
(tests/loopback_c4_worker.py).  Against the CPU restatement on the global matrix: distributed eig_mv
bitwise oracle.csr_mv (kernels_cpp.hh:596-621), 60 fused steps within rtol 1e-12 of
orc_lanczos_fused, under split and whole halo launches, with the loopback allreduce and with the
allreduce inside the step kernel (EIG_AR_MAILBOX_STEP); on every rank the value march the bench runs at
that rank size (variant 15 on the 2 M-row slabs of the 8-way split, the 2-line variant 22 on larger ranks)."""
import json
import os
import subprocess
import sys

import pytest

import eigmi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, STEPS, PS = 256, 60, (2, 4, 8)
RUNS = ("loopback/split", "loopback/whole", "mailbox-step/split", "mailbox-step/whole")


@pytest.fixture(scope="module")
def c4_lines():
    # the virtual ranks' in-kernel exchange waits for the peers' kernels: one hardware queue per stream
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(3 * max(PS)))
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "loopback_c4_worker.py"), str(N),
                        str(STEPS)] + [str(p) for p in PS], capture_output=True, text=True, timeout=900, env=env)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    lines = {}
    for s in r.stdout.splitlines():
        if s.startswith("{"):
            d = json.loads(s)
            lines[d["P"]] = d
    return lines


@pytest.mark.gpu
@pytest.mark.parametrize("P", PS)
def test_c4_partition_256(c4_lines, P):
    d = c4_lines[P]
    assert len(d["ranks"]) == P
    for rk in d["ranks"]:
        r = rk["rank"]
        assert rk["error"] is None, rk
        assert rk["rows"] == N * N * (N // P)
        assert rk["halo"] == (N * N if r > 0 else 0) + (N * N if r < P - 1 else 0)
        # the benched kernel on every rank: the fused value march with the values streamed -- variant 15
        # on the 2 M-row slabs of the 8-way split (the bench's N = 8 ranks), the 2-line march (22) on
        # ranks of at least EIG_MARCH_2L_MIN_ROWS rows
        want = 22 if rk["rows"] >= eigmi.MARCH_2L_MIN_ROWS else 15
        assert rk["kernel"] == "k_lanczos_fused_march" and rk["variant"] == want and rk["uniform"] == 0, rk
        assert rk["mv_bitwise"], f"rank {r}: distributed eig_mv not bitwise the oracle row loop"
        assert set(rk["rel"]) == set(RUNS)
        for key in RUNS:
            da, db = rk["rel"][key]
            assert da <= 1e-12 and db <= 1e-12, f"rank {r} {key}: alpha {da:.2e} beta {db:.2e} vs orc_lanczos_fused"
        assert rk["allreduce"] == "xgmi-mailbox-step" and rk["mailbox_errors"] == 0, rk
