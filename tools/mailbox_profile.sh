#!/bin/bash
# Two mailbox ranks (processes) on the box's one GPU, each under rocprofv3 kernel trace:
# per-call k_mailbox_allreduce duration vs the host-observed period.  Run from the repo root.
set -e
export TMPDIR=/tmp
out=${1:-gpurun_out/mbox_prof}
wd=$(mktemp -d)
mkdir -p "$out"
for r in 0 1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/r$r" -o trace -- python3 tests/mailbox_worker.py $r 2 "$wd" &
done
wait
python3 - "$wd" <<'PY'
import sys, numpy as np
for r in range(2):
    d = np.load(f"{sys.argv[1]}/r{r}.npz")
    print("rank", r, "us/call", float(d["us"]), "errors", int(d["errors"]))
PY
