#!/bin/bash
# Round-4 GPU session af (round-end build): the general scrambled + RCM 256^3 matrix (csrpmc: trace +
# FETCH / WRITE) and the P1 Kuhn K fused step's FETCH / WRITE passes -- VERDICT r3 #3's same-build PMC.
O=gpurun_out/${TAG:-r04af}; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "[r04] $name" >&2
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[r04] $name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "[r04] $name ended abnormally: stopping" >&2; exit $rc ;; esac
  return 0
}
TAG=${TAG:-r04af} step csrpmc 1100 bash tools/gpu.sh csrpmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step kfetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/kpmc/fetch -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 1 --steps 10 --variants fused,mv > /dev/null 2> $O/kpmc_f.err
step kwrite 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/kpmc/write -o pmc -- python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 1 --steps 10 --variants fused,mv > /dev/null 2> $O/kpmc_w.err
step ktrace 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kpmc/trace -o trace -- python3 tools/lanczos_sweep.py --N 256 --matrix p1k --rounds 3 --steps 30 --variants fused,mv > $O/kuhn.jsonl 2> $O/kpmc_t.err
cat $O/csrpmc.jsonl $O/kuhn.jsonl
