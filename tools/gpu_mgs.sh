#!/bin/bash
# Small-block MGS check: the BLAS / inverse / driver GPU tests, then the INV and C1 config lines.
set -e
mkdir -p gpurun_out/mgs
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_blas_mv8.py tests/test_inverse.py tests/test_gpu_drivers.py tests/test_harness.py > gpurun_out/mgs/pytest.log 2>&1
timeout -k 10 200 python -u tools/bench_configs.py inv > gpurun_out/mgs/inv.jsonl 2> gpurun_out/mgs/inv.err
timeout -k 10 200 python -u tools/bench_configs.py c1 > gpurun_out/mgs/c1.jsonl 2> gpurun_out/mgs/c1.err
EIGMI_MGS_SMALL=0 timeout -k 10 200 python -u tools/bench_configs.py inv > gpurun_out/mgs/inv_grid.jsonl 2> gpurun_out/mgs/inv_grid.err
