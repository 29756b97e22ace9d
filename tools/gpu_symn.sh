set -o pipefail
mkdir -p gpurun_out/symn
O=gpurun_out/symn
timeout -k 10 400 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_spmv.py tests/test_loopback_gpu.py tests/test_gpu_drivers.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/lanczos_sweep.py --rounds 5 --variants fused:sym2:w8,fused:sym2:w5,fused:sym1:w8,fused:sym0:w8,classic:sym2,classic:sym1 > $O/sweep.jsonl 2> $O/sweep.err
