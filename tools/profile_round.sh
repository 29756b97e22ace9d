#!/bin/bash
# Collect the rocprofv3 evidence for bench.py on one MI355X (run through gpurun from the repo root):
#   1. kernel trace + stats of the default bench command (per-kernel average durations)
#   2. separate PMC passes (FETCH_SIZE, WRITE_SIZE cannot share one pass on gfx950: TCC slots)
# Outputs land in gpurun_out/prof_<tag>/; copy the summaries into profiles/.
set -euo pipefail
TAG=${1:-r01}
STEPS=${STEPS:-50}
EXTRA=${BENCH_ARGS:-}   # e.g. BENCH_ARGS="--variant classic"
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
  python3 bench.py --steps "$STEPS" --warmup 5 --no-cpu-baseline $EXTRA > "$OUT/bench_trace.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-events $EXTRA > "$OUT/bench_fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-events $EXTRA > "$OUT/bench_write.json"
echo "profile done: $OUT"
