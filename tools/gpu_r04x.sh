#!/bin/bash
# Round-4 GPU session x (measurement build, since reverted): k_box_mv32 cache policies at 256^3.
O=gpurun_out/${TAG:-r04x}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
step box_tests 300 python -u -m pytest tests/test_gpu_sym.py -m gpu -x -q -k "box_push" --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q "failed" $O/tests.log || { echo "[r04] tests failed: stopping" >&2; exit 1; }
EIGMI_BOXK_VAR=1 EIGMI_BOX_COLS=32 EIGMI_BOX_CACHE=0,2,6,1,3,7,0,2,6 step boxk 400 python3 tools/bench_configs.py boxk > $O/boxk.jsonl 2> $O/boxk.err
cat $O/boxk.jsonl
