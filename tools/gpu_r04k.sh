#!/bin/bash
# Round-4 GPU session k: the P1 Kuhn fused step (march variant 16) -- plane runs and FETCH / WRITE PMC.
O=gpurun_out/${TAG:-r04k}; mkdir -p $O
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
step p1k 300 python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 3 --steps 30 \
  --variants fused,fused@8,fused@12,fused@20,fused@32,fused,mv > $O/p1k.jsonl 2> $O/sweep.err
cat $O/p1k.jsonl
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 1 --steps 10 --variants fused,mv > /dev/null 2> $O/pmc_f.err
step write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 1 --steps 10 --variants fused,mv > /dev/null 2> $O/pmc_w.err
step ta 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr --output-format csv -d $O/pmc_ta -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 1 --steps 10 --variants fused,mv > /dev/null 2> $O/pmc_ta.err
