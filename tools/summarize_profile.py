#!/usr/bin/env python3
"""Turn a tools/profile_round.sh output directory into the committed evidence under profiles/:
  profiles/<tag>_kernel_stats.csv    rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<tag>_pmc_summary.json    per-kernel FETCH_SIZE / WRITE_SIZE averages, corrected

gfx950 corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of a coalesced streaming read, so it is doubled.  The factor was
re-checked on this path's own kernels with known byte counts: k_dot<true> (8-B loads, n doubles)
and k_lanczos_update (16-B loads, 2n doubles) both read exactly 2 x FETCH_SIZE.

usage: python tools/summarize_profile.py gpurun_out/prof_r01 r01
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(src, tag):
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    fetch = pmc(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE")
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_stats.csv"))):
        stats[r["Name"].split("(")[0].replace("void ", "")] = float(r["AverageNs"])
    import time
    out = {"tag": tag, "collected": time.time(),
           "units": "bytes per launch (FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024)", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        name = k.replace("void ", "")
        f = fetch.get(k, 0.0) * 2 * 1024
        w = write.get(k, 0.0) * 1024
        out["kernels"][name] = {"fetch_bytes": round(f), "write_bytes": round(w), "hbm_bytes": round(f + w),
                                "avg_ns_trace": stats.get(name)}
    for fn in ("bench_trace.json",):
        p = os.path.join(src, fn)
        if os.path.exists(p):
            out["bench_line_under_trace"] = json.loads(open(p).read().strip().splitlines()[-1])
            out["build"] = out["bench_line_under_trace"].get("build")  # eigmi.build_id() of the profiled library
    with open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
