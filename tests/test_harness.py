"""harness parity -- dune-eigensolver_amd/bin/eigmi_harness reads the reference's
INI keys (src/dune-eigensolver.ini) with "-key value" overrides (ParameterTreeParser::readOptions)
and prints the reference's lines (src/dune-eigensolver.cc): "eval[  i]=...", the
"N_M_TOL_..." LaTeX rows of the convergence tests (.cc:617-626, :715-724) and the
"P_n_m_i_iblocked_perfn_perfb_perfv" row of the Gram-Schmidt benchmark (.cc:283-296).
The ini below is written by the test (same keys and values as the reference's file, smaller N)."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "dune-eigensolver_amd", "bin", "eigmi_harness")
INI = """[grid]
N = 5
refine = 1

[mv]
N = 5
n_iter = 1000
m = 64

[ev]
N = 16
m =  4 #24
maxiter = 4000
shift = 1e-3
regularization = 0.0
tol = 2e-3
verbose = 0
overlap = 3
method = raes
seed = 123

[parallel]
numthreads = 1

[mgs]
n = 2000
m = 16
n_iter = 3
"""


@pytest.fixture(scope="module")
def ini(tmp_path_factory):
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "dune-eigensolver_amd"), "bin/eigmi_harness"])
    p = tmp_path_factory.mktemp("harness") / "dune-eigensolver.ini"
    p.write_text(INI)
    return str(p)


def run(ini, *args, timeout=300):
    r = subprocess.run([BIN, "-ini", ini, *args], capture_output=True, text=True, timeout=timeout,
                       cwd=os.path.dirname(ini))
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def evals(out):
    return [float(m.group(1)) for m in re.finditer(r"eval\[\s*\d+\]=\s*([-+0-9.eE]+)", out)]


def test_ini_and_options(ini):
    out = run(ini, "-print-config", "-ev.N", "64", "-ev.tol", "1e-6")
    cfg = dict(line.split(" = ", 1) for line in out.splitlines() if " = " in line)
    assert cfg["ev.N"] == "64" and cfg["ev.tol"] == "1e-6" and cfg["ev.m"] == "4" and cfg["mgs.n_iter"] == "3"
    assert cfg["parallel.numthreads"] == "1" and cfg["ev.method"] == "raes"


@pytest.mark.gpu
def test_largest_convergence(ini):
    out = run(ini, "-ev.tol", "1e-10")
    row = out.split("N_M_TOL_ESARERROR_ARPERROR_ESANERROR_TIMERATIO_ARPACKITER")[1].splitlines()[1]
    f = [float(x) for x in row.replace("\\\\", "").split("&")]
    assert int(f[0]) == 256 and int(f[1]) == 4 and f[2] == 1e-10
    ev = evals(out)
    N = 16
    h = np.pi / (N + 1)
    s = 4 * np.sin(np.arange(1, N + 1) * h / 2) ** 2
    largest = np.sort((s[:, None] + s[None, :]).ravel())[::-1][:4]
    assert np.allclose(sorted(ev, reverse=True), largest, rtol=1e-2)  # printed with 2 digits


@pytest.mark.gpu
def test_smallest_convergence(ini):
    out = run(ini, "-run", "smallest", "-ev.tol", "1e-8")
    row = [l for l in out.splitlines() if l.startswith("N_M_TOL_RASERROR_ARPERROR_TIMERATIO_ARPACKITER")][0]
    f = [float(x) for x in row.split(" ", 1)[1].replace("\\\\", "").split("&")]
    assert int(f[0]) == 256 and int(f[1]) == 4
    assert f[3] < 1e-6 and f[4] < 1e-6  # GeneralizedInverse vs ARPACK, ARPACK at tol vs 1e-14


@pytest.mark.gpu
def test_eigenvalues_raes_vs_arpack(ini):
    raes = evals(run(ini, "-run", "eigenvalues", "-ev.tol", "1e-10"))
    arp = evals(run(ini, "-run", "eigenvalues", "-ev.method", "arpack", "-ev.tol", "1e-12"))
    assert len(raes) == 4 and len(arp) == 4
    assert np.allclose(sorted(raes), sorted(arp), rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_mgs_performance_row(ini):
    out = run(ini, "-run", "mgs")
    row = [l for l in out.splitlines() if l.startswith("P_n_m_i_iblocked_perfn_perfb_perfv")][0].split()[1:]
    assert row[:3] == ["1", "2000", "16"] and all(float(x) > 0 for x in row[3:])


@pytest.mark.gpu
def test_smallest_reference_default_size(ini):
    """The smallest-eigenvalue experiment at the reference's default size (src/dune-eigensolver.ini:
    ev.N = 200, n = 40000): GeneralizedInverse and the shift-invert (ARPACK-mode) solve of the GenEO
    pencil on device-factored LU (k_band.hip) agree, and ARPACK-mode at tol with itself at 1e-14."""
    out = run(ini, "-run", "smallest", "-ev.N", "200", "-ev.tol", "1e-8")
    row = [l for l in out.splitlines() if l.startswith("N_M_TOL_RASERROR_ARPERROR_TIMERATIO_ARPACKITER")][0]
    f = [float(x) for x in row.split(" ", 1)[1].replace("\\\\", "").split("&")]
    assert int(f[0]) == 40000 and int(f[1]) == 4
    assert f[3] < 1e-6 and f[4] < 1e-6
