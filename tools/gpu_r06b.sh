#!/bin/bash
# round 6, session b: StandardLargest Gram fusion, inverse-driver loops, mailbox restart, 2-line probe
set -o pipefail
TAG=${TAG:-r06b}
O=gpurun_out/$TAG
mkdir -p $O
TAG=$TAG bash tools/gpu.sh tests:test_gpu_drivers.py,test_gpu_blas_mv8.py,test_facade_cpp.py,test_inverse.py,test_mailbox_step_gpu.py,test_loopback_c4.py || exit 1
timeout -k 10 200 python -u tools/bench_configs.py c1 c2 > $O/cfg_c12.jsonl 2> $O/cfg.err || exit 1
EIGMI_NO_SPMM_GRAM=1 timeout -k 10 200 python -u tools/bench_configs.py c1 c2 > $O/cfg_c12_nogram.jsonl 2>> $O/cfg.err || exit 1
timeout -k 10 200 tools/march_copy 256 values ablation 8 > $O/march_copy_abl.jsonl || exit 1
TAG=$TAG bash tools/gpu.sh sltrace
