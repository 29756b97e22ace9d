#!/bin/bash
# Round-4 GPU session e: all GPU tests, the bench line, C5 on the variable-coefficient box image.
O=gpurun_out/${TAG:-r04e}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
step tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -4 $O/tests.log
step bench 400 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
step boxkvar 300 env EIGMI_BOXK_VAR=1 python -u tools/bench_configs.py boxk > $O/boxk_var.jsonl 2> $O/boxk_var.err
cat $O/boxk_var.jsonl
step c5var 400 env EIGMI_C5_VAR=1 EIGMI_C5_N=256 python -u tools/bench_configs.py c5 > $O/c5_var.jsonl 2> $O/c5_var.err
cat $O/c5_var.jsonl
step sweep 300 python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 3 --steps 40 \
  --variants fused,fused#15,fused@12#15,fused@16#15,fused#12,mv > $O/latency.jsonl 2> $O/sweep.err
cat $O/latency.jsonl
step slab 200 python3 tools/lanczos_sweep.py --N 256 --slab 32 --matrix varcoef --rounds 3 --steps 40 \
  --variants fused,fused#15,fused@4#15,fused@1#15,pipelined,mv > $O/slab.jsonl 2>> $O/sweep.err
cat $O/slab.jsonl
