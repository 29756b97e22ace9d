#!/bin/bash
# Round-4 GPU session d: value-march variants (10 arrays/buffer, 14 arrays/global, 13 pack/buffer,
# 15 pack/global) x plane runs at 256^3, their TA / SQ counters, and the Kuhn march plane runs.
O=gpurun_out/${TAG:-r04d}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step vtests 300 python -u -m pytest tests/test_gpu_value_march.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
V="fused,fused#12,fused#11,fused#13,fused#15,fused@16#15,fused@12#15,fused@16#13,fused@16#12,fused@16,mv,mv#12,mv#13,mv#15,mv#1"
step sweep 300 python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 3 --steps 40 --variants $V > $O/latency.jsonl 2> $O/sweep.err
cat $O/latency.jsonl
step slab 200 python3 tools/lanczos_sweep.py --N 256 --slab 32 --matrix varcoef --rounds 3 --steps 40 \
  --variants fused,fused#12,fused#13,fused#15,fused@4#15,mv,mv#15 > $O/slab.jsonl 2>> $O/sweep.err
cat $O/slab.jsonl
step p1k 300 python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 2 --steps 30 \
  --variants fused@16,fused@24,fused@16#14,fused#14,mv@16,mv#14 > $O/p1k.jsonl 2>> $O/sweep.err
cat $O/p1k.jsonl
P="fused,fused#12,fused#13,fused#15,mv#15"
step ta 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr --output-format csv -d $O/pmc_ta -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 1 --steps 10 --variants $P > /dev/null 2> $O/pmc_ta.err
step sq 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU --output-format csv -d $O/pmc_sq -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 1 --steps 10 --variants $P > /dev/null 2> $O/pmc_sq.err
python3 tools/pmc_summary.py $O/pmc_sq $O/pmc_ta --match march > $O/pmc_summary.json
cat $O/pmc_summary.json
