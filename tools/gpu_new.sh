# GPU tests of the components added this session (non-symmetric Arnoldi, split CholQR, facade)
set -o pipefail
O=gpurun_out/new
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_arnoldi.py \
  tests/test_gpu_blas_mv8.py tests/test_facade_cpp.py > $O/tests.log 2>&1
