# C1-C3 configs on the current build: GPU tests of the SpMM / orthonormalisation kernels, then the
# config lines under a kernel trace and FETCH / WRITE PMC passes (verdict r1 weak #5)
set -o pipefail
O=gpurun_out/c2
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sym.py tests/test_gpu_blas_mv8.py tests/test_gpu_drivers.py -m gpu > $O/tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2/trace -o tr -- python3 tools/bench_configs.py c1 c2 c3 > gpurun_out/prof_c2/c123.jsonl 2> $O/c.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_c2/fetch -o pmc -- python3 tools/bench_configs.py c2 > /dev/null 2> $O/f.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_c2/write -o pmc -- python3 tools/bench_configs.py c2 > /dev/null 2> $O/w.err || exit 1
