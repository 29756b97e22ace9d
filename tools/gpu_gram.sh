#!/bin/bash
# a6 Gram / a9 orthonormalize / C5 panel products: parity tests, then timing under a kernel trace.
set -o pipefail
TAG=${TAG:-r03b}
OUT=gpurun_out/gram_$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_blas_mv8.py tests/test_block_lanczos.py -q -s --timeout 120 \
  --timeout-method thread > $OUT/tests.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
  python3 tools/bench_configs.py gram > $OUT/gram.jsonl 2> $OUT/gram.err && \
timeout -k 10 300 python3 tools/bench_configs.py c5 > $OUT/c5.jsonl 2> $OUT/c5.err
