set -o pipefail
O=gpurun_out/inv3
mkdir -p $O
EIGMI_TRACE_SETUP=1 timeout -k 10 200 python -u tools/time_setup.py 64 > $O/setup64.log 2>&1 || exit 1
EIGMI_INV_N=64 timeout -k 10 200 python -u tools/bench_configs.py inv > $O/inv64.jsonl 2> $O/inv64.err || exit 1
