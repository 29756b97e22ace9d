# A/B sweep of the fused step's matrix images + PMC passes of the symmetric-band fused kernel.
set -o pipefail
mkdir -p gpurun_out/prof_sym
O=gpurun_out/prof_sym
timeout -k 10 300 python -u tools/lanczos_sweep.py --rounds 5 --variants fused:sym1:w8,fused:sym1:w5,fused:sym1:w6,fused:sym0:w8 > $O/sweep.jsonl 2> $O/sweep.err && \
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o pmc -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-events > $O/b1.json 2>$O/b1.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o pmc -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-events > $O/b2.json 2>$O/b2.err && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/sq -o pmc -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-events > $O/b3.json 2>$O/b3.err && \
EIGMI_SYM=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/sq0 -o pmc -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-events > $O/b4.json 2>$O/b4.err
