# Round-end config lines on the current build: C1-C3, C5 (256^3), and the inverse / shift-invert
# drivers at 64^2 and the reference's default ev.N = 200 (one line per op; tools/bench_configs.py)
set -o pipefail
O=gpurun_out/cfg_${TAG:-r02k}
mkdir -p $O
timeout -k 10 300 python -u tools/bench_configs.py c1 c2 c3 > $O/c123.jsonl 2> $O/c123.err || exit 1
EIGMI_C5_N=256 timeout -k 10 300 python -u tools/bench_configs.py c5 > $O/c5.jsonl 2> $O/c5.err || exit 1
EIGMI_INV_N=64 timeout -k 10 300 python -u tools/bench_configs.py inv > $O/inv64.jsonl 2> $O/inv64.err || exit 1
EIGMI_INV_N=200 timeout -k 10 400 python -u tools/bench_configs.py inv > $O/inv200.jsonl 2> $O/inv200.err || exit 1
