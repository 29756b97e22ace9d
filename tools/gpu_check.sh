set -o pipefail
TAG=${TAG:-r02a}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
TAG=$TAG bash tools/profile_round.sh $TAG > gpurun_out/$TAG/prof.log 2>&1
