# PMC of the C5 Chebyshev launch on the box kernel (tools/cheb_sweep.py, one variant)
set -o pipefail
O=gpurun_out/prof_box
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export SWEEP="EIGMI_NOTHING=1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o tr -- python3 tools/cheb_sweep.py --rounds 1 > $O/c.json 2> $O/c.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o pmc -- python3 tools/cheb_sweep.py --rounds 1 > /dev/null 2>$O/f.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o pmc -- python3 tools/cheb_sweep.py --rounds 1 > /dev/null 2>$O/w.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/sq -o pmc -- python3 tools/cheb_sweep.py --rounds 1 > /dev/null 2>$O/s.err || exit 1
