#!/bin/bash
# Round-4 GPU session j: k_box_mv32's XCD-contiguous tile map (EIG_TUNE_BOX_MAP) -- parity, timing
# and FETCH_SIZE against the dispatch-order map.
O=gpurun_out/${TAG:-r04j}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
step push_tests 300 python -u -m pytest tests/test_gpu_sym.py -m gpu -x -q -k "box_push" --timeout 120 --timeout-method thread > $O/push_tests.log 2>&1
tail -3 $O/push_tests.log
grep -q " passed" $O/push_tests.log && ! grep -q "failed" $O/push_tests.log || { echo "[r04] tests failed: stopping" >&2; exit 1; }
EIGMI_BOXK_VAR=1 EIGMI_BOX_COLS=32,33,32,33 step boxk 300 python3 tools/bench_configs.py boxk > $O/boxk.jsonl 2> $O/boxk.err
cat $O/boxk.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
EIGMI_BOXK_VAR=1 EIGMI_BOX_COLS=33 step fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 tools/bench_configs.py boxk > /dev/null 2> $O/pmc_f.err
EIGMI_BOXK_VAR=1 EIGMI_BOX_COLS=33 step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 tools/bench_configs.py boxk > /dev/null 2> $O/pmc_w.err
