set -o pipefail
O=gpurun_out/${TAG:-r05c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mailbox_step_gpu.py tests/test_gpu_config_size.py tests/test_gpu_value_march.py tests/test_mailbox_gpu.py tests/test_rccl_one_rank.py tests/test_gpu_fused_guard.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; grep -E "stalled|P=|eigenpairs|fused steps vs" $O/tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/lanczos_sweep.py --N 256 --slab 32 --matrix varcoef --comm self --rounds 3 --steps 40 --variants fused~rccl,fused~mailbox,fused~step,mv > $O/slab.jsonl 2> $O/slab.err && cat $O/slab.jsonl &&
timeout -k 10 200 python3 tools/lanczos_sweep.py --N 256 --matrix poisson --comm self --rounds 3 --steps 40 --variants fused:arrays~rccl,fused:arrays~mailbox,fused:arrays~step > $O/cube.jsonl 2> $O/cube.err && cat $O/cube.jsonl &&
timeout -k 10 300 python bench.py --comm-self --rehearse-trial --no-cpu-baseline --side-steps 0 --general-steps 0 > $O/trial.json 2> $O/trial.err && cat $O/trial.json
