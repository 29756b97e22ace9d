set -o pipefail
O=gpurun_out/csr2
mkdir -p $O
for ord in 0 1; do
EIGMI_EXP_ORDER=$ord timeout -k 10 300 python -u tools/csr_general.py > $O/csr_ord$ord.jsonl 2> $O/csr_ord$ord.err || exit 1
EIGMI_EXP_ORDER=$ord timeout -k 10 300 python -u tools/lanczos_sweep.py --rounds 3 --variants fused:sell,classic:sell,mv:sell,mv:explicit,fused:explicit > $O/sweep_ord$ord.jsonl 2> $O/sweep_ord$ord.err || exit 1
done
