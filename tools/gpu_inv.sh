#!/bin/bash
# Inverse-row check on one GPU: the factor-apply / inverse-driver tests, the INV bench lines with
# the default (block-inverse) and the bitwise staged kernel, and a kernel trace of the default.
set -e
mkdir -p gpurun_out/inv
export PYTHONPATH=$PWD/dune-eigensolver_amd:$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_inverse.py tests/test_shift_invert.py > gpurun_out/inv/pytest.log 2>&1
timeout -k 10 200 python -u tools/bench_configs.py inv > gpurun_out/inv/default.jsonl 2> gpurun_out/inv/default.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/inv/prof -o inv -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py inv > $GRAFT_REPO_ROOT/gpurun_out/inv/prof.log 2>&1
