#!/bin/bash
# round 6, session k: the quad-layout first read pass of the look-ahead MGS
set -o pipefail
TAG=${TAG:-r06k}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_blas_mv8.py tests/test_gpu_drivers.py tests/test_gpu_config_size.py -m gpu -v -s \
  --timeout 300 --timeout-method thread -k "not eigenpairs" > $O/tests.log 2>&1
echo "pytest rc $?" >> $O/tests.log
timeout -k 10 200 python -u tools/bench_configs.py ortho > $O/ortho.jsonl 2> $O/ortho.err || exit 1
TAG=$TAG bash tools/gpu.sh orthopmc
