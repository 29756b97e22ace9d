"""Host-side pieces of bench.py (no GPU): the roofline's PMC traffic lookup must parse every
committed profiles/*_pmc_summary.json (a crash there would cost the round's bench line) and prefer
a summary profiled on the same build."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_committed_traffic_parses_all_profiles():
    import bench
    import eigmi
    tr = bench.committed_traffic("k_lanczos_fused_march", 256, 1, eigmi.build_id())
    assert tr is None or (tr[0] > 0 and tr[1].startswith("profiles/") and tr[2] in (True, False))
    assert bench.committed_traffic("no_such_kernel", 256, 1, None) is None


def test_committed_traffic_prefers_same_build(tmp_path, monkeypatch):
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    line = {"config": {"N": 64}, "n_gpus": 1}
    k = "eigmi::k_lanczos_fused_march"
    for tag, build, stamp, b in (("old", "aaa", 1.0, 111), ("new", "bbb", 2.0, 222)):
        (prof / f"{tag}_pmc_summary.json").write_text(json.dumps(
            {"tag": tag, "build": build, "collected": stamp, "bench_line_under_trace": line,
             "kernels": {k: {"hbm_bytes": b}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.committed_traffic("k_lanczos_fused_march", 64, 1, "aaa") == (111, "profiles/old_pmc_summary.json", True)
    assert bench.committed_traffic("k_lanczos_fused_march", 64, 1, "ccc") == (222, "profiles/new_pmc_summary.json", False)
