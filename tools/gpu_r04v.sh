#!/bin/bash
# Round-4 GPU session v: the Kuhn pack's once-read pair streams with the default cache policy
# (EIG_TUNE_CACHE bit 1) vs nontemporal -- time and FETCH_SIZE.
O=gpurun_out/${TAG:-r04v}; mkdir -p $O
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
step kuhn_tests 300 python -u -m pytest tests/test_gpu_value_march.py -m gpu -x -q -k "kuhn" --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
step p1k 300 python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 3 --steps 30 \
  --variants fused,fused%2,fused@8,fused@8%2,fused,fused%2,mv,mv%2 > $O/p1k.jsonl 2> $O/sweep.err
cat $O/p1k.jsonl
step fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 1 --steps 10 --variants fused%2 > /dev/null 2> $O/pmc_f.err
