# Shift-invert block vs one-vector Lanczos: the shift-invert tests, then timings at 64^2 and 200^2
# (tools/time_setup.py; scipy ARPACK + SuperLU on the box's host beside them)
set -o pipefail
O=gpurun_out/si2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_shift_invert.py tests/test_arnoldi.py tests/test_harness.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u tools/time_setup.py 64 > $O/t64.log 2>&1 || { cat $O/t64.log; exit 1; }
cat $O/t64.log
timeout -k 10 400 python -u tools/time_setup.py 200 x > $O/t200.log 2>&1 || { cat $O/t200.log; exit 1; }
cat $O/t200.log
