"""Config C5 (generalised block Lanczos, k = 32, variable-coefficient P1 K/M) row-partitioned at its
own size, 256^3, on ONE GPU: P = 8 z-slabs (32 planes per virtual rank, the 8-GPU split) over the
loopback hub (tests/loopback_c5_worker.py).  Every rank streams the box image the one-rank run streams
(k_box_mv32 SpMM, k_box_mv32_cheb mass-solve step): a slab's box kernel reads its ghost planes from
the window as planes -1 / nz (k_box.hip box_prepare, launch_box) -- the kernels an 8-GPU run takes.
Against the one-rank run of the same pencil: the
block-tridiagonal T within 1e-10 of max |T|, the 8 largest Ritz values within 1e-10 relative, their
residuals within 1e-7 relative (eigensolver.hh:283-325, kernels_cpp.hh:356-591).
The constant-coefficient pencil (kinds 6 / 7, row classes kept: every rank on the row-class kernels,
k_boxc_mv8 / k_boxc_mv8_cheb with classes by global plane) runs the same way with EIGMI_C5_PART_CONST=1
(profiles/r06zk_*); the default suite covers those slab kernels at 64^3 (tests/cpp/loopback_test.cc,
8 ranks, block 16) and keeps one 256^3 pencil here to bound the suite's time."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, STEPS, PS = 256, 3, (8,)


KERNELS = {"var": ("k_box_mv32", "k_box_mv32_cheb"), "const": ("k_boxc_mv8", "k_boxc_mv8_cheb")}


@pytest.fixture(scope="module", params=["var", "const"] if os.environ.get("EIGMI_C5_PART_CONST") else ["var"])
def c5_lines(request):
    extra = ["--const"] if request.param == "const" else []
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "loopback_c5_worker.py"), str(N),
                        str(STEPS)] + [str(p) for p in PS] + extra, capture_output=True, text=True, timeout=900)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    lines = {}
    for s in r.stdout.splitlines():
        if s.startswith("{"):
            d = json.loads(s)
            lines[d["P"]] = d
    lines["pencil"] = request.param
    return lines


@pytest.mark.gpu
@pytest.mark.parametrize("P", PS)
def test_c5_partition_256(c5_lines, P):
    kspmm, kcheb = KERNELS[c5_lines["pencil"]]
    one = c5_lines[1]
    assert one["spmm"] == kspmm and one["cheb"] == kcheb, one
    d = c5_lines[P]
    assert len(d["ranks"]) == P
    for rk in d["ranks"]:
        r = rk["rank"]
        assert rk["error"] is None, rk
        assert rk["rows"] == N * N * (N // P)
        assert rk["spmm"] == kspmm and rk["cheb"] == kcheb, rk
        assert rk["T_shape_ok"], rk
        assert rk["T_rel"] <= 1e-10, f"rank {r}: T differs from the one-rank run by {rk['T_rel']:.2e} of max |T|"
        assert rk["ev_rel"] <= 1e-10, f"rank {r}: Ritz values differ by {rk['ev_rel']:.2e}"
        assert rk["res_rel"] <= 1e-7, f"rank {r}: residuals differ by {rk['res_rel']:.2e}"
