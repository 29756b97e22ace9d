# Block-inverse chain on the matrix cores (EIG_TRSV_BLOCKINV_MFMA): agreement with the vector chain
# and apply time vs columns at 64^2 and 200^2
set -o pipefail
O=gpurun_out/chain
mkdir -p $O
timeout -k 10 120 python -u tools/time_apply.py 64 > $O/a64.log 2>&1 || { cat $O/a64.log; exit 1; }
cat $O/a64.log
timeout -k 10 300 python -u tools/time_apply.py 200 > $O/a200.log 2>&1 || { cat $O/a200.log; exit 1; }
cat $O/a200.log
