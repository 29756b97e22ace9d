#!/usr/bin/env python3
"""Average PMC counters per kernel from rocprofv3 --pmc csv directories (one row per dispatch).
    python tools/pmc_summary.py <dir> [<dir> ...] [--match SUBSTR]"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    if "--match" in sys.argv:
        match = sys.argv[sys.argv.index("--match") + 1]
        args.remove(match)
    out = collections.defaultdict(dict)
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            agg = collections.defaultdict(list)
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if match and match not in k:
                    continue
                agg[(k.split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
            for (k, c), v in agg.items():
                out[k][c] = sum(v) / len(v)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
