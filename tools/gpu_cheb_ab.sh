# A/B of the box Chebyshev step in ONE process (interleaved rounds): in place (EIGMI_EXP_INPLACE),
# nontemporal X loads (EIGMI_EXP_NTX), plain stores (EIGMI_EXP_PLAINST); 32 launches per difference
set -o pipefail
O=gpurun_out/cheb_ab
mkdir -p $O
SWEEP="EIGMI_NOTHING=1;EIGMI_EXP_INPLACE=1;EIGMI_EXP_NTX=1;EIGMI_EXP_INPLACE=1,EIGMI_EXP_NTX=1;EIGMI_EXP_PLAINST=1" timeout -k 10 600 python -u tools/cheb_sweep.py --rounds 5 --dlo 2 --dhi 34 > $O/cheb.jsonl 2> $O/cheb.err || exit 1
