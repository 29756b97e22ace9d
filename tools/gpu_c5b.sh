# Two-degree Chebyshev kernel: box / block-Lanczos tests, then the C5 block step with kernel trace
set -o pipefail
O=gpurun_out/c5b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sym.py tests/test_block_lanczos.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
EIGMI_C5_N=256 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o tr -- python3 tools/bench_configs.py c5 > $O/c5.json 2> $O/c5.err || exit 1
