# Device band LU (k_band.hip): the LU / inverse / shift-invert tests, then setup + solve timings
set -o pipefail
O=gpurun_out/band
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_inverse.py tests/test_shift_invert.py tests/test_harness.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
EIGMI_TRACE_SETUP=1 timeout -k 10 300 python -u tools/time_apply.py 200 > $O/a200.log 2>&1 || { cat $O/a200.log; exit 1; }
cat $O/a200.log
timeout -k 10 200 python -u tools/time_setup.py 64 x > $O/t64.log 2>&1 || { cat $O/t64.log; exit 1; }
cat $O/t64.log
timeout -k 10 400 python -u tools/time_setup.py 200 x > $O/t200.log 2>&1 || { cat $O/t200.log; exit 1; }
cat $O/t200.log
