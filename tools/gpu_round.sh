# Round evidence: profile (trace + PMC) of the default bench, then the full default bench line.
set -o pipefail
TAG=${TAG:-r01d}
bash tools/profile_round.sh $TAG && \
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
