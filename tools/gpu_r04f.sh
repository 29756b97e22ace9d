#!/bin/bash
# Round-4 GPU session f: Kuhn march occupancy variant, a6 / panel Gram timings, C5 smallest end on the
# variable-coefficient pencil.
O=gpurun_out/${TAG:-r04f}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
step p1k 300 python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 3 --steps 30 \
  --variants fused,fused#15,fused@16#15,fused@12#15,fused@6#15,mv,mv#15 > $O/p1k.jsonl 2> $O/sweep.err
cat $O/p1k.jsonl
step gram 300 python3 tools/bench_configs.py gram > $O/gram.jsonl 2> $O/gram.err
cat $O/gram.jsonl
step c5sivar 600 env EIGMI_C5_VAR=1 EIGMI_C5_N=256 python -u tools/bench_configs.py c5si > $O/c5si_var.jsonl 2> $O/c5si_var.err
cat $O/c5si_var.jsonl
