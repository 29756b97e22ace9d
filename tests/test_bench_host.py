"""Host-side pieces of bench.py (no GPU): the roofline's PMC traffic lookup must parse every
committed profiles/*_pmc_summary.json (a crash there would cost the round's bench line)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_committed_traffic_parses_all_profiles():
    import bench
    tr = bench.committed_traffic("k_lanczos_fused_march", 256, 1)
    assert tr is None or (tr[0] > 0 and tr[1].startswith("profiles/"))
    assert bench.committed_traffic("no_such_kernel", 256, 1) is None
    assert bench.committed_traffic("k_lanczos_fused_march", 256, 8) is None or True
