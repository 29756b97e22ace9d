#!/bin/bash
# Round-4 GPU session h: the push-order box kernel (k_box_mv16p) -- parity, then k_box_mv32 vs
# k_box_mv16p at 256^3 on the variable-coefficient P1 K / M under a kernel trace; CholQR2 test.
O=gpurun_out/${TAG:-r04h}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
step push_tests 300 python -u -m pytest tests/test_gpu_sym.py -m gpu -x -q -k "box" --timeout 120 --timeout-method thread > $O/push_tests.log 2>&1
tail -3 $O/push_tests.log
grep -q " passed" $O/push_tests.log && ! grep -q "failed" $O/push_tests.log || { echo "[r04] push tests failed: stopping" >&2; exit 1; }
step blanczos 300 python -u -m pytest tests/test_block_lanczos.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/blanczos.log 2>&1
tail -3 $O/blanczos.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
EIGMI_BOXK_VAR=1 EIGMI_BOX_COLS=32,16,32,16 step boxk 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/boxk_trace -o trace -- \
  python3 tools/bench_configs.py boxk > $O/boxk.jsonl 2> $O/boxk.err
cat $O/boxk.jsonl
