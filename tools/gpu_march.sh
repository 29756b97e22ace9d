set -o pipefail
mkdir -p gpurun_out/march
O=gpurun_out/march
timeout -k 10 400 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_drivers.py tests/test_gpu_spmv.py tests/test_loopback_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/lanczos_sweep.py --rounds 5 --variants fused:march1,fused:march0,classic:march1,classic:march0 > $O/sweep.jsonl 2> $O/sweep.err && \
timeout -k 10 300 python -u tools/spmv_sweep.py > $O/spmv.jsonl 2> $O/spmv.err
