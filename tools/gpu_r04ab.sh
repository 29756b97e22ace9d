#!/bin/bash
# Round-4 GPU session ab: the 16-wave block-inverse chain (k_binv_chain16) -- parity, then A/B
# against the 8-wave chain (EIGMI_BINV_CHAIN=8) on the 200^2 shift-invert and the INV configs.
O=gpurun_out/${TAG:-r04ab}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
step inv_tests 400 python -u -m pytest tests/test_inverse.py tests/test_shift_invert.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q "failed" $O/tests.log || { echo "[r04] tests failed: stopping" >&2; exit 1; }
step si16 200 python3 tools/si_profile.py 200 > $O/si16.txt 2>&1
EIGMI_BINV_CHAIN=8 step si8 200 python3 tools/si_profile.py 200 > $O/si8.txt 2>&1
step si16_64 200 python3 tools/si_profile.py 64 > $O/si16_64.txt 2>&1
EIGMI_BINV_CHAIN=8 step si8_64 200 python3 tools/si_profile.py 64 > $O/si8_64.txt 2>&1
cat $O/si16.txt $O/si8.txt $O/si16_64.txt $O/si8_64.txt
EIGMI_INV_N=200 step inv200 400 python -u tools/bench_configs.py inv > $O/cfg_inv200.jsonl 2> $O/cfg_inv200.err
EIGMI_INV_N=64 step inv64 300 python -u tools/bench_configs.py inv > $O/cfg_inv64.jsonl 2> $O/cfg_inv64.err
