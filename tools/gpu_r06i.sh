#!/bin/bash
# round 6, session i: configuration lines on the round-6 build (C1-C3, C5 both coefficient kinds, inverse modes)
set -o pipefail
TAG=${TAG:-r06i}
O=gpurun_out/$TAG
mkdir -p $O
TAG=$TAG bash tools/gpu.sh configs || exit 1
EIGMI_C5_VAR=1 EIGMI_C5_N=256 timeout -k 10 300 python -u tools/bench_configs.py c5 > $O/cfg_c5_var.jsonl 2> $O/cfg_c5_var.err || exit 1
timeout -k 10 200 python -u tools/bench_configs.py ortho > $O/ortho.jsonl 2> $O/ortho.err || exit 1
