#!/bin/bash
# round 6, session j: the MGS error word in host-mapped memory (no copy at eig_ctx_sync)
set -o pipefail
TAG=${TAG:-r06j}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_blas_mv8.py tests/test_gpu_drivers.py tests/test_inverse.py -m gpu -v -s \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "pytest rc $?" >> $O/tests.log
timeout -k 10 200 python -u tools/bench_configs.py ortho > $O/ortho.jsonl 2> $O/ortho.err || exit 1
timeout -k 10 200 python -u tools/bench_configs.py c1 c2 > $O/cfg_c12.jsonl 2> $O/cfg.err || exit 1
