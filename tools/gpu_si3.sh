# Shift-invert: tests, then timings (tools/time_setup.py) and one traced 200^2 solve
set -o pipefail
O=gpurun_out/si3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_shift_invert.py tests/test_inverse.py tests/test_harness.py tests/test_arnoldi.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u tools/time_setup.py 64 x > $O/t64.log 2>&1 || { cat $O/t64.log; exit 1; }
cat $O/t64.log
timeout -k 10 400 python -u tools/time_setup.py 200 x > $O/t200.log 2>&1 || { cat $O/t200.log; exit 1; }
cat $O/t200.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p200 -o si -- python3 -u tools/si_once.py 200 > $O/p200.log 2>&1 || { cat $O/p200.log; exit 1; }
grep "block:" $O/p200.log
