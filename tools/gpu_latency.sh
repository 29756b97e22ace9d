#!/bin/bash
# Fixed cost vs streaming of the fused step: kernel time of the fused step and of eig_mv across cube
# sizes and one-rank slabs, and the plane-run count of the march kernels (tools/lanczos_sweep.py).
set -o pipefail
TAG=${TAG:-r03c}
OUT=gpurun_out/lat_$TAG
mkdir -p $OUT
run() { timeout -k 10 150 python3 tools/lanczos_sweep.py "$@" --rounds 3 --steps 40 >> $OUT/sweep.jsonl; }
run --N 128 --variants fused,fused@32,fused@28,fused@16,fused@12,mv,mv@16 && \
run --N 256 --variants fused,fused@8,fused@7,fused@6,fused@4,mv,mv@7 && \
run --N 256 --slab 32 --variants fused,fused@1,fused@4,fused@7,mv && \
run --N 256 --slab 16 --variants fused,fused@2,fused@4,fused@7,mv && \
run --N 192 --variants fused,mv
