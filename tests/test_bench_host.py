"""Host-side pieces of bench.py (no GPU): the roofline's PMC traffic lookup must parse every
committed profiles/*_pmc_summary.json (a crash there would cost the round's bench line) and prefer
a summary profiled on the same build and the same matrix image."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_committed_traffic_parses_all_profiles():
    import bench
    import eigmi
    for img in bench.IMAGES:
        tr = bench.committed_traffic("k_lanczos_fused_march", 256, 1, eigmi.build_id(), img)
        assert tr is None or (tr[0] > 0 and tr[1].startswith("profiles/") and tr[2] in (True, False))
    assert bench.committed_traffic("no_such_kernel", 256, 1, None, "arrays") is None


def test_committed_traffic_prefers_same_build(tmp_path, monkeypatch):
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    k = "eigmi::k_lanczos_fused_march<unsigned char, true, 10>"
    for tag, build, stamp, b, img in (("old", "aaa", 1.0, 111, "arrays"), ("new", "bbb", 2.0, 222, "arrays"),
                                      ("newest", "bbb", 3.0, 333, "uniform")):
        line = {"config": {"N": 64, "image": img}, "n_gpus": 1}
        (prof / f"{tag}_pmc_summary.json").write_text(json.dumps(
            {"tag": tag, "build": build, "collected": stamp, "bench_line_under_trace": line,
             "kernels": {k: {"hbm_bytes": b}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    kk = "k_lanczos_fused_march<unsigned char, true, 10>"
    assert bench.committed_traffic(kk, 64, 1, "aaa", "arrays") == (111, "profiles/old_pmc_summary.json", True)
    assert bench.committed_traffic(kk, 64, 1, "ccc", "arrays") == (222, "profiles/new_pmc_summary.json", False)
    assert bench.committed_traffic("k_lanczos_fused_march", 64, 1, "ccc", "uniform")[0] == 333
    # another template instance of the same kernel is not this image's kernel
    assert bench.committed_traffic("k_lanczos_fused_march<unsigned char, true, 7>", 64, 1, "ccc", "arrays") is None
