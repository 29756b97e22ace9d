set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02a/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err
