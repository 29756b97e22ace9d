#!/bin/bash
# Round-4 end-of-round evidence on the final build (after the 16-wave block-inverse chain): GPU tests,
# smoke, the bench's kernel trace and FETCH / WRITE PMC passes (tools/profile_round.sh), the bench
# line, the INV configurations.
O=gpurun_out/${TAG:-r04z3}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
step tests 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
step profile 400 bash tools/profile_round.sh r04z3 > $O/profile.log 2>&1
step bench 300 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
EIGMI_INV_N=200 step inv200 400 python -u tools/bench_configs.py inv > $O/cfg_inv200.jsonl 2> $O/cfg_inv200.err
EIGMI_INV_N=64 step inv64 300 python -u tools/bench_configs.py inv > $O/cfg_inv64.jsonl 2> $O/cfg_inv64.err
