# Inverse / shift-invert after the setup changes: GPU tests, setup phases, driver timings at 64^2 and 200^2
set -o pipefail
O=gpurun_out/inv2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_inverse.py tests/test_shift_invert.py \
  tests/test_harness.py tests/test_facade_cpp.py tests/test_arnoldi.py -m gpu > $O/tests.log 2>&1 || exit 1
EIGMI_TRACE_SETUP=1 timeout -k 10 200 python -u tools/time_setup.py 64 > $O/setup64.log 2>&1 || exit 1
EIGMI_TRACE_SETUP=1 timeout -k 10 300 python -u tools/time_setup.py 200 > $O/setup200.log 2>&1 || exit 1
EIGMI_INV_N=64 timeout -k 10 200 python -u tools/bench_configs.py inv > $O/inv64.jsonl 2> $O/inv64.err || exit 1
EIGMI_INV_N=200 timeout -k 10 400 python -u tools/bench_configs.py inv > $O/inv200.jsonl 2> $O/inv200.err || exit 1
