set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_spmv.py tests/test_loopback_gpu.py tests/test_gpu_drivers.py -x -v --timeout 200 --timeout-method thread > gpurun_out/sym_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_sym.json 2> gpurun_out/bench_sym.err && \
EIGMI_SYM=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_nosym.json 2> gpurun_out/bench_nosym.err
