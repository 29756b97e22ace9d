set -o pipefail
mkdir -p gpurun_out/march
O=gpurun_out/march
timeout -k 10 400 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_drivers.py tests/test_gpu_spmv.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/lanczos_sweep.py --rounds 5 --variants ${VARIANTS:-fused:march1,fused:march2,fused:march3,fused:march0,classic:march1,classic:march2,classic:march3,mv:march1,mv:march2,mv:march3,mv:march0} > $O/sweep.jsonl 2> $O/sweep.err
