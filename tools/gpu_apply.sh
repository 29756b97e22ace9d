# Block-inverse solve time vs columns (tools/time_apply.py) with setup phases, and its kernel trace
set -o pipefail
O=gpurun_out/apply
mkdir -p $O
EIGMI_TRACE_SETUP=1 timeout -k 10 300 python -u tools/time_apply.py 200 > $O/a200.log 2>&1 || { cat $O/a200.log; exit 1; }
cat $O/a200.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ap -- python3 -u tools/time_apply.py 200 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-8 {} | head -12
