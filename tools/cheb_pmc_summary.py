#!/usr/bin/env python3
"""Summarise gpurun_out/cheb_pmc (tools/gpu_cheb_pmc.sh): per variant the median k_box_mv32<1> launch
(kernel trace) and its WRITE_SIZE bytes."""
import csv
import glob
import os
import sys

O = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/cheb_pmc"
for line in open(os.path.join(O, "variants.txt")):
    i, v = line.split(maxsplit=1)
    t = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
         for f in glob.glob(f"{O}/t{i}/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))
         if ("k_box_mv32<1>" in r["Kernel_Name"] or "k_boxc_mv8<1," in r["Kernel_Name"])]
    w = [float(r["Counter_Value"]) for f in glob.glob(f"{O}/w{i}/**/*counter_collection.csv", recursive=True)
         for r in csv.DictReader(open(f)) if ("k_box_mv32<1>" in r["Kernel_Name"] or "k_boxc_mv8<1," in r["Kernel_Name"])]
    t.sort()
    print(v.strip(), "launch_ms", round(t[len(t) // 2] / 1e6, 3) if t else None,
          "write_GB", round(sum(w) / len(w) * 1024 / 1e9, 3) if w else None)
