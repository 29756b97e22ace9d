# Pipelined one-reduction step: GPU parity (guard tests, loopback ranks) and the per-rank cost
# of fused vs pipelined on one rank's 256x256x32 slab and on the full 256^3 cube
set -o pipefail
O=gpurun_out/pipe
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fused_guard.py \
  tests/test_loopback_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/lanczos_sweep.py --slab 32 --variants fused,pipelined,mv --rounds 5 > $O/slab.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/lanczos_sweep.py --variants fused,pipelined,mv --rounds 3 > $O/cube.jsonl 2>&1 || exit 1
