#!/usr/bin/env python3
"""Measured HBM copy rate by eig_stream_copy_timed mode (0..3) and size: the peak the bench's
frac_vs_measured_copy divides by.  One JSON line per (mode, MiB)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-eigensolver_amd"))
import eigmi  # noqa: E402

ctx = eigmi.Context(0)
for mib in (512, 1024, 2048):
    n = mib * (1 << 20) // 8
    for mode in range(4):
        g = max(eigmi.stream_copy_GBs(ctx, n, 10, mode) for _ in range(3))
        print(json.dumps({"mode": mode, "MiB_each_way": mib, "GBs": round(g, 1)}), flush=True)
