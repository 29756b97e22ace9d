"""The C++ drop-in facade (include/eigmi.hh) compiled with the host compiler against libeigmi.so:
reference-style code (ISTL-concept matrix, MultiVector<double,8>-compatible container, reference
kernel names, ARPACK++ operator) -- tests/cpp/facade_test.cc."""
import os
import subprocess

import pytest

import eigmi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def facade_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("facade") / "facade_test")
    libdir = os.path.join(ROOT, "dune-eigensolver_amd", "lib")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "facade_test.cc"), "-L" + libdir, "-leigmi",
                           "-Wl,-rpath," + libdir, "-o", out])
    return out


def test_facade_compiles_and_reports_no_device(facade_bin):
    if eigmi.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = subprocess.run([facade_bin, "--no-device"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "no device" in r.stdout


@pytest.mark.gpu
def test_facade_on_gpu(facade_bin):
    r = subprocess.run([facade_bin], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
