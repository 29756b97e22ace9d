"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: the
.cpp host sources of libeigmi (envelope LU, Matrix Market, reordering, generators, distributed
plans, argument checks) built with -fsanitize=address,undefined (make sanitize ->
lib/libeigmi_san.so) and driven by tests/sanitize_worker.py with the clang ASan runtime preloaded.
No device code runs; any sanitizer report fails the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dune-eigensolver_amd")


def test_host_code_sanitized():
    rt = subprocess.run(["/opt/rocm/bin/hipcc", "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True,
                        text=True).stdout.strip()
    if not rt or not os.path.exists(rt):
        pytest.skip("clang ASan runtime not found")
    subprocess.check_call(["make", "-C", PKG, "-j8", "sanitize"], stdout=subprocess.DEVNULL)
    pre = os.environ.get("LD_PRELOAD")  # (kept: the runtime goes first, whatever else is preloaded stays)
    env = dict(os.environ, EIGMI_LIB_VARIANT="san", LD_PRELOAD=rt + (":" + pre if pre else ""),
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               PYTHONPATH=os.pathsep.join([PKG, os.path.join(ROOT, "oracle")]))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sanitize_worker.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "sanitize worker ok" in r.stdout, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
