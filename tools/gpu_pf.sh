# Plane-prefetching march (low-occupancy launches): parity tests, then slab timing with / without it
set -o pipefail
O=gpurun_out/pf
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sym.py \
  tests/test_gpu_fused_guard.py tests/test_loopback_gpu.py tests/test_gpu_drivers.py -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/lanczos_sweep.py --slab 32 --variants fused,pipelined,mv --rounds 5 > $O/slab_pf.jsonl 2>&1 || exit 1
EIGMI_EXP_NOPF=1 timeout -k 10 200 python -u tools/lanczos_sweep.py --slab 32 --variants fused,pipelined,mv --rounds 5 > $O/slab_nopf.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/lanczos_sweep.py --slab 16 --variants fused,mv --rounds 5 > $O/slab16_pf.jsonl 2>&1 || exit 1
EIGMI_EXP_NOPF=1 timeout -k 10 200 python -u tools/lanczos_sweep.py --slab 16 --variants fused,mv --rounds 5 > $O/slab16_nopf.jsonl 2>&1 || exit 1
