# PMC passes of the plane-march kernels (fused step via bench.py; SpMV / K1 via the sweep tool).
set -o pipefail
O=gpurun_out/prof_march
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for V in ${PVARS:-fused}; do
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$V -o pmc -- python3 tools/lanczos_sweep.py --rounds 1 --steps 10 --variants $V > $O/f_$V.json 2>$O/f_$V.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$V -o pmc -- python3 tools/lanczos_sweep.py --rounds 1 --steps 10 --variants $V > $O/w_$V.json 2>$O/w_$V.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/sq_$V -o pmc -- python3 tools/lanczos_sweep.py --rounds 1 --steps 10 --variants $V > $O/s_$V.json 2>$O/s_$V.err || exit 1
done
