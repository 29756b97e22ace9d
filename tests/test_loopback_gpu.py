"""The distributed device path on one GPU (virtual ranks over the in-process loopback transport):
tests/cpp/loopback_test.cc compared with the single-rank run of the same matrix -- SpMV bitwise,
global dots, Lanczos alpha/beta (rtol 1e-12) and Ritz values (1e-10); and the fused step with its
allreduce inside the step kernel (EIG_AR_MAILBOX_STEP) over split / whole halo launches."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def loopback_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("loopback") / "loopback_test")
    libdir = os.path.join(ROOT, "dune-eigensolver_amd", "lib")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "loopback_test.cc"), "-L" + libdir, "-leigmi",
                           "-lpthread", "-Wl,-rpath," + libdir, "-o", out])
    return out


def test_loopback_builds(loopback_bin):
    assert os.path.exists(loopback_bin)


@pytest.mark.gpu
@pytest.mark.parametrize("P,N", [(2, 16), (3, 24), (4, 32), (8, 64)])
def test_loopback_virtual_ranks(loopback_bin, P, N):
    # the mailbox phase's virtual ranks wait for each other's kernels: every stream its own hardware queue
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(max(4, 3 * P)))
    r = subprocess.run([loopback_bin, str(P), str(N)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
