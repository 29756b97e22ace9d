"""Host-side unit check of the march-variant selection (tests/cpp/march_select_test.cc): the P1 Kuhn
value-pack marches must not be chosen where their 32-bit buffer descriptor would wrap."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_kuhn_pack_descriptor_guard(tmp_path):
    out = str(tmp_path / "march_select_test")
    libdir = os.path.join(ROOT, "dune-eigensolver_amd", "lib")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-x", "c++", "-std=c++17", "-O1", "-D__HIP_PLATFORM_AMD__",
                           "-I" + os.path.join(ROOT, "include"), "-I/opt/rocm/include",
                           os.path.join(ROOT, "tests", "cpp", "march_select_test.cc"), "-L" + libdir, "-leigmi",
                           "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath," + libdir, "-Wl,-rpath,/opt/rocm/lib",
                           "-o", out])
    r = subprocess.run([out], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
