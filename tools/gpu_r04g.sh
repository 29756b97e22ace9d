#!/bin/bash
# Round-4 GPU session g: cache policies of the fused value march (EIG_TUNE_CACHE bits) at 256^3.
O=gpurun_out/${TAG:-r04g}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
step cache 300 python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 3 --steps 40 \
  --variants fused,fused%1,fused%2,fused%3,fused%4,fused%5,fused%6,fused%7 > $O/cache.jsonl 2> $O/sweep.err
cat $O/cache.jsonl
step cacheslab 200 python3 tools/lanczos_sweep.py --N 256 --slab 32 --matrix varcoef --rounds 3 --steps 40 \
  --variants fused,fused%1,fused%2,fused%4,fused%6 > $O/cacheslab.jsonl 2>> $O/sweep.err
cat $O/cacheslab.jsonl
step c2 300 python3 tools/bench_configs.py c2 > $O/c2.jsonl 2> $O/c2.err
cat $O/c2.jsonl
step blanczos 300 python -u -m pytest tests/test_block_lanczos.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/blanczos.log 2>&1
tail -3 $O/blanczos.log
