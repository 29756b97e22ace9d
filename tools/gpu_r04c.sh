#!/bin/bash
# Round-4 GPU session c: full GPU tests (no -x), value-march variants at 256^3 (timing + SQ / TA /
# FETCH / WRITE counters per kernel instance).  Abnormal ends (124/137/134/139) stop the call.
O=gpurun_out/${TAG:-r04c}; mkdir -p $O
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
step tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -8 $O/tests.log
V="fused,fused#12,fused#1,fused@16,fused@4,mv,mv#12,mv#1"
step sweep 300 python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 3 --steps 40 --variants $V > $O/latency.jsonl 2> $O/sweep.err
cat $O/latency.jsonl
P="fused,fused#12,fused#1,mv,mv#1"
step sq 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM --output-format csv -d $O/pmc_sq -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 1 --steps 10 --variants $P > /dev/null 2> $O/pmc_sq.err
step ta 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr --output-format csv -d $O/pmc_ta -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 1 --steps 10 --variants $P > /dev/null 2> $O/pmc_ta.err
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 1 --steps 10 --variants $P > /dev/null 2> $O/pmc_fetch.err
step write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 1 --steps 10 --variants $P > /dev/null 2> $O/pmc_write.err
python3 tools/pmc_summary.py $O/pmc_sq $O/pmc_ta $O/pmc_fetch $O/pmc_write --match march > $O/pmc_summary.json
cat $O/pmc_summary.json
