#!/bin/bash
# round 6, session c: determinism probe, SL Gram fusion timings, 2-line value march (tests + sweep + probe)
set -o pipefail
TAG=${TAG:-r06c}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -u tools/det_probe.py > $O/det_probe.log 2>&1 || exit 1
timeout -k 10 1200 python -u -m pytest tests/test_inverse.py tests/test_mailbox_step_gpu.py tests/test_loopback_c4.py \
  tests/test_gpu_value_march.py tests/test_gpu_config_size.py -m gpu -v -s --timeout 600 --timeout-method thread \
  > $O/tests.log 2>&1
echo "pytest rc $?" >> $O/tests.log
timeout -k 10 200 python -u tools/bench_configs.py c1 c2 > $O/cfg_c12.jsonl 2> $O/cfg.err || exit 1
EIGMI_NO_SPMM_GRAM=1 timeout -k 10 200 python -u tools/bench_configs.py c1 c2 > $O/cfg_c12_nogram.jsonl 2>> $O/cfg.err || exit 1
timeout -k 10 300 python3 tools/lanczos_sweep.py --N 256 --rounds 3 --steps 40 \
  --variants fused#13,fused#16,fused#17,fused@12#16,fused@20#16,fused@24#16,fused@12#17,fused@24#17,mv,mv#16 \
  > $O/sweep256.jsonl 2> $O/sweep.err || exit 1
timeout -k 10 200 tools/march_copy 256 values ablation 8 > $O/march_copy_abl.jsonl || exit 1
TAG=$TAG bash tools/gpu.sh sltrace
