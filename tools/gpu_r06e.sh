#!/bin/bash
# round 6, session e: the 2-line value march (variants 22 / 23 / 24) on the benchmark's image
set -o pipefail
TAG=${TAG:-r06e}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python3 tools/lanczos_sweep.py --N 256 --rounds 3 --steps 40 \
  --variants fused:arrays,fused:arrays#16,fused:arrays#17,fused:arrays#18,fused:arrays@8#16,fused:arrays@12#16,fused:arrays@20#16,fused:arrays@24#16,fused:arrays@8#17,fused:arrays@12#17,fused:arrays@24#17,mv:arrays,mv:arrays#16 \
  > $O/sweep256.jsonl 2> $O/sweep.err || exit 1
timeout -k 10 300 python3 tools/lanczos_sweep.py --N 128 --rounds 3 --steps 40 \
  --variants fused:arrays,fused:arrays#16,fused:arrays#17,fused:arrays@32#16,fused:arrays@16#16 \
  > $O/sweep128.jsonl 2>> $O/sweep.err || exit 1
timeout -k 10 300 python3 tools/lanczos_sweep.py --N 256 --slab 32 --rounds 3 --steps 40 \
  --variants fused:arrays,fused:arrays#16,fused:arrays#17,fused:arrays@4#16,fused:arrays@8#16 \
  > $O/sweepslab.jsonl 2>> $O/sweep.err || exit 1
