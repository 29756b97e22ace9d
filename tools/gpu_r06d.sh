#!/bin/bash
# round 6, session d: StandardInverse basis fix, folded Gram close, 2-line march plane-run sweep
set -o pipefail
TAG=${TAG:-r06d}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_inverse.py tests/test_gpu_drivers.py tests/test_gpu_blas_mv8.py -m gpu -v -s \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "pytest rc $?" >> $O/tests.log
timeout -k 10 200 python -u tools/bench_configs.py c1 c2 > $O/cfg_c12.jsonl 2> $O/cfg.err || exit 1
timeout -k 10 300 python3 tools/lanczos_sweep.py --N 256 --rounds 3 --steps 40 \
  --variants fused#13,fused@8#16,fused@6#16,fused@4#16,fused@10#16,fused@8#17,fused@6#17,fused@4#17,fused@8#13 \
  > $O/sweep256.jsonl 2> $O/sweep.err || exit 1
TAG=$TAG bash tools/gpu.sh sltrace
