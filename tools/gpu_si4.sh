# Shift-invert tests and timings (tools/time_setup.py) at 64^2 and 200^2
set -o pipefail
O=gpurun_out/si4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_shift_invert.py tests/test_harness.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/time_setup.py 64 x > $O/t64.log 2>&1 || { cat $O/t64.log; exit 1; }
cat $O/t64.log
timeout -k 10 400 python -u tools/time_setup.py 200 x > $O/t200.log 2>&1 || { cat $O/t200.log; exit 1; }
cat $O/t200.log
