# C5 after the Chebyshev changes: box / block-Lanczos GPU tests, the Chebyshev launch sweep, and the
# 256^3 block step with kernel trace + PMC (FETCH / WRITE) of every kernel
set -o pipefail
O=gpurun_out/c5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sym.py tests/test_block_lanczos.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
SWEEP="EIGMI_NOTHING=1" timeout -k 10 300 python -u tools/cheb_sweep.py --rounds 3 > $O/cheb.jsonl 2> $O/cheb.err || exit 1
EIGMI_C5_N=256 bash tools/prof_c5.sh || exit 1
