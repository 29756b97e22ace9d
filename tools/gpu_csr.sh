# General CSR/ELL path at 256^3 (tools/csr_general.py): timing line, kernel trace, PMC passes.
set -o pipefail
O=gpurun_out/csr
mkdir -p $O
timeout -k 10 300 python -u tools/csr_general.py > $O/csr.jsonl 2> $O/csr.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 tools/csr_general.py --reps 5 --steps 10 > $O/trace.jsonl 2> $O/trace.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 tools/csr_general.py --reps 5 --steps 10 > /dev/null 2> $O/f.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 tools/csr_general.py --reps 5 --steps 10 > /dev/null 2> $O/w.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_tcc -o pmc -- python3 tools/csr_general.py --reps 5 --steps 10 > /dev/null 2> $O/t.err || exit 1
