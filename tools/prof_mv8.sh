#!/bin/bash
# PMC passes over the window-layout SpMM / Chebyshev kernels (tools/spmm_sweep.py child, one
# mapping), run through gpurun from the repo root.  Outputs under gpurun_out/prof_mv8_<kind>/.
set -euo pipefail
KIND=${1:-quad}
N=${SWEEP_N:-224}
M=${SWEEP_M:-32}
OUT=gpurun_out/prof_mv8_${KIND}_m${M}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export EIGMI_MV8_KERNEL=$KIND
case "$KIND" in rows1) export EIGMI_MV8_KERNEL1=rows ;; grp1) export EIGMI_MV8_KERNEL1=grp ;; esac
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
  python3 tools/spmm_sweep.py child "$KIND" "$N" "$M" > "$OUT/sweep.jsonl"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc$i" -o pmc -- \
    python3 tools/spmm_sweep.py child "$KIND" "$N" "$M" > /dev/null 2> "$OUT/pmc$i.err" || echo "pass $i ($set) failed"
done
echo done
