#!/bin/bash
# Round-4 GPU session: GPU tests, value-march / Kuhn-march / slab sweeps, the bench line.
# A step that fails its assertions does not stop the call; a step that times out, aborts or faults
# (exit 124 / 137 / 134 / 139) ends it -- nothing more runs on the GPU after that.
O=gpurun_out/${TAG:-r04b}; mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -5 $O/tests.log
step sweep256 300 python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --rounds 3 --steps 40 \
  --variants fused,fused@6,fused@12,fused#1,fused#10,fused#11,fused@6#11,mv,mv#1,mv#10,mv#11,fused:sell > $O/latency.jsonl 2> $O/sweep.err
cat $O/latency.jsonl
step slab 200 python3 tools/lanczos_sweep.py --N 256 --slab 32 --matrix varcoef --rounds 3 --steps 40 \
  --variants fused,fused@1,fused@4,fused#1,fused#10,fused#11,pipelined,mv > $O/slab.jsonl 2>> $O/sweep.err
cat $O/slab.jsonl
step p1k 300 python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 3 --steps 30 \
  --variants fused,fused@6,fused@12,fused#1,mv,mv#1 > $O/p1k.jsonl 2>> $O/sweep.err
cat $O/p1k.jsonl
step bench 400 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
