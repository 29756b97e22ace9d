# Plane-run length of the fused march on one rank's slab (strong-scaling share): EIGMI_EXP_RUNDIV
set -o pipefail
O=gpurun_out/rundiv
mkdir -p $O
for d in 15 10 8 6 4; do
  EIGMI_EXP_RUNDIV=$d timeout -k 10 120 python -u tools/lanczos_sweep.py --slab 32 --variants fused --rounds 5 > $O/slab32_$d.jsonl 2>&1 || exit 1
done
for d in 15 8 4; do
  EIGMI_EXP_RUNDIV=$d timeout -k 10 120 python -u tools/lanczos_sweep.py --slab 64 --variants fused --rounds 5 > $O/slab64_$d.jsonl 2>&1 || exit 1
done
