# Sweeps only (no tests): SWEEPS="N:variants N:variants ..."
set -o pipefail
mkdir -p gpurun_out/sweep
i=0
for S in $SWEEPS; do
  N=${S%%:*}; V=${S#*:}
  timeout -k 10 300 python -u tools/lanczos_sweep.py --N $N ${SLAB:+--slab $SLAB} --rounds 5 --variants $V > gpurun_out/sweep/s$i.jsonl 2> gpurun_out/sweep/s$i.err || exit 1
  i=$((i+1))
done
