"""RCCL on one GPU (verdict r2 'next' #1): a one-rank communicator created with EIG_COMM_ALWAYS
routes every allreduce of the Lanczos drivers through ncclAllReduce -- the main communicator for
the classic / fused steps, the ncclCommSplit communicator on the reduction stream for the pipelined
step -- eagerly and inside an eig_lanczos_capture hipGraph.  A one-rank sum is the identity, so
alpha / beta must be BITWISE those of the same run without a communicator.  The grouped
ncclSend / ncclRecv of the halo exchange is rehearsed by tests/cpp/rccl_self_test.cc (rank 0 to
itself, eager and captured).  SURVEY 8(e); the reference has no distribution
(src/dune-eigensolver.cc:742-748)."""
import os
import subprocess

import numpy as np
import pytest

import eigmi
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = {"classic": {}, "fused": {"fused": True}, "pipelined": {"pipelined": True}}


@pytest.fixture(scope="module")
def rccl_self_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("rccl") / "rccl_self_test")
    libdir = os.path.join(ROOT, "dune-eigensolver_amd", "lib")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                           "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include",
                           os.path.join(ROOT, "tests", "cpp", "rccl_self_test.cc"), "-L" + libdir, "-leigmi",
                           "-L/opt/rocm/lib", "-lrccl", "-lamdhip64", "-Wl,-rpath," + libdir,
                           "-Wl,-rpath,/opt/rocm/lib", "-o", out])
    return out


def test_rccl_self_builds(rccl_self_bin):
    assert os.path.exists(rccl_self_bin)


def _run(ctx, A_csr, variant, steps, graph):
    M = eigmi.Matrix.from_bcsr(ctx, A_csr.rowptr, A_csr.col, A_csr.val)
    ws = eigmi.LanczosWorkspace(M, steps + 4, seed=123, **VARIANTS[variant])
    try:
        if graph:
            ws.step(3)  # eager head, then a captured batch (the bench's N > 1 launch)
            captured = ws.capture(steps - 3)
            ws.replay()
        else:
            ws.step(steps)
            captured = None
        a, b = ws.tridiag()
    finally:
        ws.close()
        M.close()
    return a, b, captured


@pytest.fixture(scope="module")
def rccl_ctx():
    c = eigmi.Context(0)
    c.comm_init(1, 0, eigmi.Context.unique_id(), always=True)
    yield c
    c.close()


@pytest.fixture(scope="module")
def plain_ctx():
    c = eigmi.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
def test_one_rank_comm_reports_rccl(rccl_ctx):
    info = rccl_ctx.comm_info()
    assert info["nranks"] == 1 and info["allreduce"] == "rccl"


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
@pytest.mark.parametrize("variant", list(VARIANTS))
@pytest.mark.parametrize("N", [24, 64])
def test_lanczos_through_rccl_bitwise(rccl_ctx, plain_ctx, variant, graph, N):
    A = oracle.poisson3d(N)
    steps = 40
    c0 = rccl_ctx.comm_counters()
    a1, b1, cap = _run(rccl_ctx, A, variant, steps, graph)
    c1 = rccl_ctx.comm_counters()
    a0, b0, _ = _run(plain_ctx, A, variant, steps, graph)
    assert plain_ctx.comm_counters() == {"allreduce": 0, "allreduce_split": 0, "halo_groups": 0, "p2p": 0}
    assert np.array_equal(a1, a0) and np.array_equal(b1, b0), (variant, graph, np.abs(a1 - a0).max())
    # the collectives really went to RCCL: one allreduce per step (two for the classic step), the
    # pipelined step's on the split communicator
    issued = c1["allreduce"] - c0["allreduce"], c1["allreduce_split"] - c0["allreduce_split"]
    if variant == "pipelined":
        assert issued[1] >= steps - 3
    else:
        assert issued[0] >= (2 if variant == "classic" else 1) * (steps - 3)
    if graph:
        print(f"{variant} N={N}: hipGraph capture with RCCL collectives accepted = {cap}")
        assert cap, "hipGraph capture of RCCL collectives refused"
    # and the recurrence itself is the restatement's
    if variant == "classic":
        _, qa, qb = oracle.lanczos(A, oracle.random_vec(A.n, 123), steps)
    else:
        qa, qb = oracle.lanczos_fused(A, oracle.random_vec(A.n, 123), steps, pipelined=variant == "pipelined")
    assert np.allclose(a1, qa, rtol=1e-12, atol=1e-12) and np.allclose(b1, qb, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_rccl_allreduce_identity(rccl_ctx):
    v = np.array([1.0, -2.5, np.pi, 1e300, -0.0])
    d = rccl_ctx.array(v)
    rccl_ctx.allreduce_sum(d)
    assert np.array_equal(d.get(), v)


@pytest.mark.gpu
def test_rccl_self_send_recv(rccl_self_bin):
    r = subprocess.run([rccl_self_bin], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
