# Kernel trace of one 200^2 and one 64^2 GenEO shift-invert solve (tools/si_once.py)
set -o pipefail
O=gpurun_out/siprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for N in 200 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$N -o si -- python3 -u tools/si_once.py $N > $O/p$N.log 2>&1 || { cat $O/p$N.log; exit 1; }
  cat $O/p$N.log
done
find $O -name "*kernel_stats.csv"
