# Shift-invert driver breakdown: setup phases (EIGMI_TRACE_SETUP) at 64^2 and 200^2, kernel trace of
# the 64^2 solve with the factors given
set -o pipefail
O=gpurun_out/si
mkdir -p $O
EIGMI_TRACE_SETUP=1 timeout -k 10 200 python -u tools/time_setup.py 64 > $O/setup64.log 2>&1 || exit 1
EIGMI_TRACE_SETUP=1 timeout -k 10 300 python -u tools/time_setup.py 200 > $O/setup200.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o si -- python3 -u tools/time_setup.py 64 > $O/prof.log 2>&1 || exit 1
