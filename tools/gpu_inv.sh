# INV rows (tools/bench_configs.py inv) at 64^2 and the reference's default 200^2, and the harness
# smallest experiment at ev.N = 200
set -o pipefail
O=gpurun_out/inv
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_harness.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/harness.log 2>&1 || { tail -30 $O/harness.log; exit 1; }
tail -2 $O/harness.log
EIGMI_INV_N=64 timeout -k 10 300 python -u tools/bench_configs.py inv > $O/inv64.jsonl 2> $O/inv64.err || { tail $O/inv64.err; exit 1; }
EIGMI_INV_N=200 timeout -k 10 600 python -u tools/bench_configs.py inv > $O/inv200.jsonl 2> $O/inv200.err || { tail $O/inv200.err; exit 1; }
cat $O/inv64.jsonl $O/inv200.jsonl
