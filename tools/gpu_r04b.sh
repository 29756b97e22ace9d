set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_value_march.py tests/test_gpu_sym.py tests/test_loopback_gpu.py tests/test_gpu_config_size.py tests/test_multigrid.py tests/test_block_lanczos.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 tools/lanczos_sweep.py --N 256 --matrix varcoef --variants fused,fused@6,fused@12,fused#1,fused#10,fused#11,fused@6#11,mv,mv#1,mv#10,mv#11,fused:sell --rounds 3 --steps 40 > $O/latency.jsonl 2> $O/sweep.err || exit 1
cat $O/latency.jsonl
timeout -k 10 200 python3 tools/lanczos_sweep.py --N 256 --slab 32 --matrix varcoef --variants fused,fused@1,fused@4,fused#1,fused#10,pipelined,mv --rounds 3 --steps 40 > $O/slab.jsonl 2>> $O/sweep.err || exit 1
cat $O/slab.jsonl
timeout -k 10 300 python3 tools/lanczos_sweep.py --N 256 --matrix p1k --variants fused,fused@6,fused@12,fused#1,mv,mv#1 --rounds 3 --steps 30 > $O/p1k.jsonl 2>> $O/sweep.err || exit 1
cat $O/p1k.jsonl
