# C5 Chebyshev / SpMM kernels: PMC passes on the block-Lanczos config (EIGMI_C5_N, default 160).
set -o pipefail
O=gpurun_out/prof_c5
mkdir -p $O
export EIGMI_C5_N=${EIGMI_C5_N:-160}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o tr -- python3 tools/bench_configs.py c5 > $O/c5.json 2> $O/c5.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o pmc -- python3 tools/bench_configs.py c5 > /dev/null 2>$O/f.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o pmc -- python3 tools/bench_configs.py c5 > /dev/null 2>$O/w.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/sq -o pmc -- python3 tools/bench_configs.py c5 > /dev/null 2>$O/s.err || exit 1
