#!/bin/bash
# GPU-box task runner (run through gpurun from the repo root): one script, one subcommand per
# measurement, outputs under gpurun_out/<TAG>/.  Every GPU step has its own time limit; the first
# failing step ends the call (no retries).
#
#   TAG=r03x bash tools/gpu.sh <task> [<task> ...]
#
# tasks:
#   tests[:<file,file>]  pytest -m gpu (all, or the listed tests/ files)       -> tests.log
#   smoke                __graft_entry__.smoke()                              -> smoke.log
#   bench                python bench.py (the driver's default line)          -> bench.json
#   profile              rocprofv3 kernel trace + FETCH / WRITE PMC passes of the bench (tools/profile_round.sh)
#   configs              tools/bench_configs.py c1 c2 c3, c5 (256^3), inv (64^2, 200^2)  -> cfg_*.jsonl
#   boxsegs              box kernels' z segments per tile column swept (tools/box_segs.py) -> box_segs.jsonl
#   inv                  the inverse-mode configs alone (64^2, 200^2)        -> cfg_inv*.jsonl
#   gram                 a6 / a9 / panel-Gram timings under a kernel trace    -> gram.jsonl, gram_trace/
#   grampmc              FETCH_SIZE / WRITE_SIZE passes over the gram timings -> grampmc/{fetch,write}
#   boxkpmc              FETCH_SIZE / WRITE_SIZE / TA busy of the variable-coefficient box kernels -> boxkpmc/
#   boxk                 row-class box kernels alone (SpMM, Chebyshev step) at 256^3 under a kernel trace -> boxk.jsonl, boxk_trace/
#   c5 | c5si            block Lanczos 256^3: largest end / smallest end (multigrid solve)  -> c5*.jsonl
#   c5trace              both under a kernel trace                            -> c5_trace/, c5si_trace/
#   latency              fused step vs eig_mv across sizes and slabs, plane-run counts  -> latency.jsonl
#   marchcopy            the march streams alone (tools/march_copy.hip)       -> march_copy.jsonl
#   prefetch             geometric march prefetch variants x plane runs (256^3, 128^3, slab) -> latency.jsonl
#   slabruns             plane runs on the per-rank slabs and 128^3 with the geo2 variants -> latency.jsonl
#   march256             fused step / eig_mv plane-run sweep at 256^3 and 128^3  -> latency.jsonl
#   sqpmc                SQ wave-cycle buckets and TA busy of the bench (PMC)   -> sqpmc/
#   pipe                 fused vs pipelined on one rank's slab and the cube   -> pipe.jsonl
#   csr                  general (scrambled + RCM) 256^3 matrix: SpMV / Lanczos kernels  -> csr.jsonl
#   csrpmc               the same under a kernel trace and FETCH_SIZE / WRITE_SIZE passes -> csrpmc/
#   sltrace              one C2 StandardLargest solve under a kernel trace (per-iteration kernels) -> sl/
#   smallortho           orthonormalize_blocked m = 8 at n = 512 .. 4096: default look-ahead vs one workgroup
#   commself             bench.py with and without a one-rank RCCL allreduce per step (eager / graph, 128^3 / 256^3)
#   sweep                tools/lanczos_sweep.py $SWEEP (e.g. SWEEP="--N 256 --matrix p1k --variants fused,mv") -> sweep.jsonl
#   sweeppmc             the same $SWEEP under a kernel trace, then FETCH_SIZE / WRITE_SIZE passes -> sweeppmc/
#   sweepsq              SQ wave-cycle buckets + TA busy over $SWEEP                    -> sweepsq/
#   p1kpmc               P1 Kuhn K 256^3 fused step + eig_mv: trace, FETCH_SIZE, WRITE_SIZE -> sweeppmc/
#   round                tests smoke profile bench (the round-end evidence set)
#   cfgtrace             tools/bench_configs.py $CFG under a kernel trace -> $CFG_trace/
#   ortho                a9 orthonormalize_blocked m = 8 / 32 at 128^3: look-ahead L = 8/4/2, stepwise replay, in-place -> ortho.jsonl
#   orthopmc             the same under a kernel trace + FETCH_SIZE / WRITE_SIZE passes -> orthopmc/
#   sweep2l              the fused step's 1-line (15) vs 2-line (22 / 23 / 24) value march: 256^3, 128^3, slab -> sweep2l_*.jsonl
#   ablation             tools/march_copy.hip's value-march ablation incl. the 2- / N-line probes -> march_copy_abl.jsonl
#   c4                   C4's row partition at 256^3 on 2 / 4 / 8 virtual ranks vs the oracle (tests/test_loopback_c4.py)
#   slgram               StandardLargest with and without the fused window Gram (C1, C2) + one C2 solve's kernel trace
#   detprobe             run-to-run determinism of the inverse-iteration pieces (tools/det_probe.py)
#   xch                  the step's allreduce transports on one GPU (one-rank RCCL / mailbox / in-kernel
#                        mailbox-step): slab and cube sweeps + the bench's N > 1 trial rehearsed -> xch_*.jsonl
#   threshold            variant 15 vs the 2-line march on 4 / 6 / 8 M-row slabs (EIG_MARCH_2L_MIN_ROWS) -> threshold.jsonl
#   halotime             the halo mailbox between 2 / 4 processes on one GPU (kernel trace) + the trial rehearsal
#   mbonly               bench.py --gpus 2 / 4 --transport mailbox-only on ONE GPU (the whole N > 1 bench path)
#   runs2l               plane runs of the 1- and 2-line value marches (256^3, 128^3, 256^2 slabs)  -> runs_*.jsonl
#   spmmruns             plane runs of the 8-column SpMM / SpMM + dots + Gram (tools/spmm_runs.py)
#   c5part               C5 256^3 block Lanczos on 8 loopback ranks vs one rank (variable / constant coefficients), traced
#   chebsegs             C5's Chebyshev step per box z-segment count (tools/cheb_segs.py; whole-solve differences)
#
# Session scripts of earlier rounds (tools/gpu_r04*.sh) are these tasks chained, e.g.
#   TAG=r05a bash tools/gpu.sh tests:test_gpu_value_march.py sweep sweeppmc
set -o pipefail
TAG=${TAG:-scratch}
O=gpurun_out/$TAG
mkdir -p "$O"
prof_env() { cd /tmp && export TMPDIR=/tmp && cd - > /dev/null; }
sweep() { timeout -k 10 150 python3 tools/lanczos_sweep.py "$@" --rounds 3 --steps 40 >> "$O/latency.jsonl"; }

run_task() {
  case "$1" in
    tests)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 ;;
    tests:*)
      local files
      files=$(echo "${1#tests:}" | tr ',' ' ' | sed 's#\([^ ]*\)#tests/\1#g')
      timeout -k 10 900 python -u -m pytest $files -m gpu -x -v -s --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    bench)
      timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" ;;
    profile)
      bash tools/profile_round.sh "$TAG" > "$O/profile.log" 2>&1 ;;
    configs)
      timeout -k 10 300 python -u tools/bench_configs.py c1 c2 c3 > "$O/cfg_c123.jsonl" 2> "$O/cfg_c123.err" && \
      EIGMI_C5_N=256 timeout -k 10 300 python -u tools/bench_configs.py c5 > "$O/cfg_c5.jsonl" 2> "$O/cfg_c5.err" && \
      EIGMI_INV_N=64 timeout -k 10 300 python -u tools/bench_configs.py inv > "$O/cfg_inv64.jsonl" 2> "$O/cfg_inv64.err" && \
      EIGMI_INV_N=200 timeout -k 10 400 python -u tools/bench_configs.py inv > "$O/cfg_inv200.jsonl" 2> "$O/cfg_inv200.err" ;;
    boxsegs)
      timeout -k 10 400 python -u tools/box_segs.py 128 256 > "$O/box_segs.jsonl" 2> "$O/box_segs.err" ;;
    boxsegsvar)
      EIGMI_BOXSEG_VAR=1 timeout -k 10 400 python -u tools/box_segs.py 128 256 > "$O/box_segs_var.jsonl" 2> "$O/box_segs_var.err" ;;
    inv)
      EIGMI_INV_N=64 timeout -k 10 300 python -u tools/bench_configs.py inv > "$O/cfg_inv64.jsonl" 2> "$O/cfg_inv64.err" && \
      EIGMI_INV_N=200 timeout -k 10 400 python -u tools/bench_configs.py inv > "$O/cfg_inv200.jsonl" 2> "$O/cfg_inv200.err" ;;
    gram)
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/gram_trace" -o trace -- \
        python3 tools/bench_configs.py gram > "$O/gram.jsonl" 2> "$O/gram.err" ;;
    grampmc)
      # PMC of the Gram timings (separate FETCH_SIZE / WRITE_SIZE passes; tools/summarize_pmc_dirs.py)
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/grampmc/trace" -o trace -- \
        python3 tools/bench_configs.py gram > "$O/grampmc.jsonl" 2> "$O/grampmc_t.err" && \
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/grampmc/fetch" -o pmc -- \
        python3 tools/bench_configs.py gram > /dev/null 2> "$O/grampmc_f.err" && \
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/grampmc/write" -o pmc -- \
        python3 tools/bench_configs.py gram > /dev/null 2> "$O/grampmc_w.err" ;;
    boxk)
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/boxk_trace" -o trace -- \
        python3 tools/bench_configs.py boxk > "$O/boxk.jsonl" 2> "$O/boxk.err" && \
      EIGMI_BOXK_VAR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/boxkvar_trace" -o trace -- \
        python3 tools/bench_configs.py boxk >> "$O/boxk.jsonl" 2>> "$O/boxk.err" ;;
    boxkpmc)
      # FETCH_SIZE / WRITE_SIZE / TA busy passes over the variable-coefficient box kernels (k_box_mv32)
      prof_env
      EIGMI_BOXK_VAR=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/boxkpmc/fetch" -o pmc -- \
        python3 tools/bench_configs.py boxk > "$O/boxkpmc.jsonl" 2> "$O/boxkpmc_f.err" && \
      EIGMI_BOXK_VAR=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/boxkpmc/write" -o pmc -- \
        python3 tools/bench_configs.py boxk > /dev/null 2> "$O/boxkpmc_w.err" && \
      EIGMI_BOXK_VAR=1 timeout -s KILL 300 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr --output-format csv -d "$O/boxkpmc/ta" -o pmc -- \
        python3 tools/bench_configs.py boxk > /dev/null 2> "$O/boxkpmc_t.err" ;;
    c5)
      EIGMI_C5_N=256 timeout -k 10 300 python -u tools/bench_configs.py c5 > "$O/c5.jsonl" 2> "$O/c5.err" ;;
    c5si)
      EIGMI_C5_N=256 timeout -k 10 600 python -u tools/bench_configs.py c5si > "$O/c5si.jsonl" 2> "$O/c5si.err" ;;
    c5trace)
      # C5 block steps (both ends) under a kernel trace: the per-kernel split of a block step
      prof_env
      EIGMI_C5_N=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c5_trace" -o trace -- \
        python3 tools/bench_configs.py c5 > "$O/c5t.jsonl" 2> "$O/c5t.err" && \
      EIGMI_C5_N=256 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c5si_trace" -o trace -- \
        python3 tools/bench_configs.py c5si > "$O/c5sit.jsonl" 2> "$O/c5sit.err" ;;
    latency)
      sweep --N 128 --variants fused,fused@32,fused@28,fused@16,fused@12,mv,mv@16 && \
      sweep --N 256 --variants fused,fused@8,fused@7,fused@6,fused@4,mv,mv@7 && \
      sweep --N 256 --slab 32 --variants fused,fused@1,fused@4,fused@7,mv && \
      sweep --N 256 --slab 16 --variants fused,fused@2,fused@4,fused@7,mv && \
      sweep --N 64 --variants fused,fused@64,fused@32,fused@16,mv ;;
    marchcopy)
      # the march's streams without the matrix (tools/march_copy.hip, built on the CPU host)
      timeout -k 10 120 tools/march_copy 256 > "$O/march_copy.jsonl" && \
      timeout -k 10 60 tools/march_copy 128 >> "$O/march_copy.jsonl" ;;
    prefetch)
      # geometric march variants (eig_mat_tune EIG_TUNE_MARCH_PREFETCH #1..#5) x plane runs
      sweep --N 256 --variants fused@6#1,fused@6#6,fused@8#6,fused@6#7,fused@4#8,fused@8#7,fused@4#5,mv#1,mv#5,mv#6,mv#7,mv#8 && \
      sweep --N 128 --variants fused#1,fused#5,fused#6,fused#7,fused#8,fused@16#7,fused@6#8,mv#1,mv#5,mv#6,mv#7 && \
      sweep --N 256 --slab 32 --variants fused#1,fused#5,fused#6,fused#7,fused#8,mv#5,mv#6,mv#7 && \
      sweep --N 256 --slab 16 --variants fused#1,fused#5,fused#7,fused#8 ;;
    slabruns)
      # plane runs per column on the per-rank slabs and C2 with the geo2 variants
      sweep --N 256 --slab 32 --variants fused@2#7,fused@4#7,fused@8#7,fused@16#7,fused@2#8,fused@4#8,fused@8#8,fused@16#8 && \
      sweep --N 256 --slab 16 --variants fused@2#7,fused@4#7,fused@8#7,fused@16#7,fused@2#8,fused@4#8 && \
      sweep --N 128 --variants fused@4#8,fused@8#8,fused@12#8,fused@16#8,fused@32#8,fused@8#7,fused@16#7,fused@32#7 ;;
    march256)
      sweep --N 256 --variants fused,fused@16,fused@12,fused@8,fused@6,fused@4,mv && \
      sweep --N 128 --variants fused,fused@24,fused@12,fused@8,fused@4,mv ;;
    sqpmc)
      # where the fused march's wave cycles go (SQ counters) and how busy the texture-address path is
      prof_env
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM --output-format csv -d "$O/sqpmc/sq" -o pmc -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> "$O/sqpmc_sq.err" && \
      timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr --output-format csv -d "$O/sqpmc/ta" -o pmc -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> "$O/sqpmc_ta.err" ;;
    pipe)
      timeout -k 10 200 python -u tools/lanczos_sweep.py --slab 32 --variants fused,pipelined,mv --rounds 5 > "$O/pipe.jsonl" 2>&1 && \
      timeout -k 10 200 python -u tools/lanczos_sweep.py --variants fused,pipelined,mv --rounds 3 >> "$O/pipe.jsonl" 2>&1 ;;
    commself)
      for L in eager graph; do
        for N in 128 256; do
          timeout -k 10 300 python bench.py --N $N --no-cpu-baseline --launch $L --comm-self >> "$O/commself.jsonl" 2>> "$O/commself.err" && \
          timeout -k 10 300 python bench.py --N $N --no-cpu-baseline --launch $L >> "$O/commself.jsonl" 2>> "$O/commself.err" || return 1
        done
      done ;;
    csr)
      timeout -k 10 400 python -u tools/csr_general.py > "$O/csr.jsonl" 2> "$O/csr.err" ;;
    sltrace)
      prof_env
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/sl" -o sl -- \
        python3 -u tools/sl_trace.py > "$O/sl.log" 2>&1 ;;
    smallortho)
      timeout -k 10 200 python3 -u tools/small_ortho.py > "$O/small_ortho.jsonl" 2> "$O/small_ortho.err" ;;
    csrpmc)
      # the general-matrix kernels under a kernel trace and FETCH_SIZE / WRITE_SIZE passes
      prof_env
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/csrpmc/trace" -o trace -- \
        python3 tools/csr_general.py --reps 10 --steps 20 > "$O/csrpmc.jsonl" 2> "$O/csrpmc_t.err" && \
      timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/csrpmc/fetch" -o pmc -- \
        python3 tools/csr_general.py --reps 10 --steps 20 > /dev/null 2> "$O/csrpmc_f.err" && \
      timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/csrpmc/write" -o pmc -- \
        python3 tools/csr_general.py --reps 10 --steps 20 > /dev/null 2> "$O/csrpmc_w.err" ;;
    sweep)
      timeout -k 10 300 python3 tools/lanczos_sweep.py $SWEEP > "$O/sweep.jsonl" 2> "$O/sweep.err" ;;
    sweeppmc)
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/sweeppmc/trace" -o trace -- \
        python3 tools/lanczos_sweep.py $SWEEP > "$O/sweeppmc.jsonl" 2> "$O/sweeppmc_t.err" && \
      timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/sweeppmc/fetch" -o pmc -- \
        python3 tools/lanczos_sweep.py $SWEEP > /dev/null 2> "$O/sweeppmc_f.err" && \
      timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/sweeppmc/write" -o pmc -- \
        python3 tools/lanczos_sweep.py $SWEEP > /dev/null 2> "$O/sweeppmc_w.err" ;;
    sweepsq)
      prof_env
      timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM --output-format csv -d "$O/sweepsq/sq" -o pmc -- \
        python3 tools/lanczos_sweep.py $SWEEP > /dev/null 2> "$O/sweepsq_sq.err" && \
      timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr --output-format csv -d "$O/sweepsq/ta" -o pmc -- \
        python3 tools/lanczos_sweep.py $SWEEP > /dev/null 2> "$O/sweepsq_ta.err" ;;
    p1kpmc)
      SWEEP="--N 256 --matrix p1k --rounds 1 --steps 10 --variants fused,mv" run_task sweeppmc ;;
    xch)
      timeout -k 10 200 python3 tools/lanczos_sweep.py --N 256 --slab 32 --matrix varcoef --comm self --rounds 3 --steps 40 \
        --variants fused~rccl,fused~mailbox,fused~step,mv > "$O/xch_slab.jsonl" 2> "$O/xch.err" && \
      timeout -k 10 200 python3 tools/lanczos_sweep.py --N 256 --comm self --rounds 3 --steps 40 \
        --variants fused:arrays~rccl,fused:arrays~mailbox,fused:arrays~step > "$O/xch_cube.jsonl" 2>> "$O/xch.err" && \
      timeout -k 10 300 python bench.py --comm-self --rehearse-trial --no-cpu-baseline --side-steps 0 --general-steps 0 \
        > "$O/xch_trial.json" 2>> "$O/xch.err" ;;
    ortho)
      timeout -k 10 200 python -u tools/bench_configs.py ortho > "$O/ortho.jsonl" 2> "$O/ortho.err" && \
      EIGMI_MGS_INPLACE=1 timeout -k 10 200 python -u tools/bench_configs.py ortho >> "$O/ortho.jsonl" 2>> "$O/ortho.err" ;;
    orthopmc)
      # a9 under a kernel trace and FETCH_SIZE / WRITE_SIZE passes (tools/summarize_pmc_dirs.py)
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/orthopmc/trace" -o trace -- \
        python3 tools/bench_configs.py ortho > "$O/orthopmc.jsonl" 2> "$O/orthopmc_t.err" && \
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/orthopmc/fetch" -o pmc -- \
        python3 tools/bench_configs.py ortho > /dev/null 2> "$O/orthopmc_f.err" && \
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/orthopmc/write" -o pmc -- \
        python3 tools/bench_configs.py ortho > /dev/null 2> "$O/orthopmc_w.err" ;;
    c5part)
      # C5's block Lanczos at 256^3 on 8 loopback ranks (tests/loopback_c5_worker.py) under a kernel trace
      prof_env
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c5part_trace" -o trace -- \
        python3 tests/loopback_c5_worker.py 256 2 8 > "$O/c5part.jsonl" 2> "$O/c5part.err" && \
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c5partc_trace" -o trace -- \
        python3 tests/loopback_c5_worker.py 256 2 8 --const > "$O/c5partc.jsonl" 2> "$O/c5partc.err" ;;
    orthogrid)
      # the read-only passes' grid (EIGMI_MGS_GRID workgroups at most)
      for g in 256 512 1024 2048; do
        EIGMI_MGS_GRID=$g timeout -k 10 200 python -u tools/bench_configs.py ortho >> "$O/orthogrid.jsonl" 2>> "$O/ortho.err" || return 1
      done ;;
    cfgtrace)
      # tools/bench_configs.py $CFG under a kernel trace (per-kernel durations of one configuration)
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${CFG}_trace" -o trace -- \
        python3 tools/bench_configs.py $CFG > "$O/${CFG}_t.jsonl" 2> "$O/${CFG}_t.err" ;;
    sweep2l)
      timeout -k 10 400 python3 tools/lanczos_sweep.py --N 256 --rounds 3 --steps 40 \
        --variants fused:arrays#13,fused:arrays#16,fused:arrays#17,fused:arrays#18,fused:arrays@8#16,fused:arrays@24#16,mv:arrays,mv:arrays#16 \
        > "$O/sweep2l_256.jsonl" 2> "$O/sweep2l.err" && \
      timeout -k 10 300 python3 tools/lanczos_sweep.py --N 128 --rounds 3 --steps 40 \
        --variants fused:arrays#13,fused:arrays#16,fused:arrays#17 > "$O/sweep2l_128.jsonl" 2>> "$O/sweep2l.err" && \
      timeout -k 10 300 python3 tools/lanczos_sweep.py --N 256 --slab 32 --rounds 3 --steps 40 \
        --variants fused:arrays#13,fused:arrays#16,fused:arrays#17 > "$O/sweep2l_slab.jsonl" 2>> "$O/sweep2l.err" ;;
    halotime)
      # the halo mailbox between 2 / 4 mailbox-only processes on one GPU (256^3 z-slabs) under a kernel
      # trace; then the bench's N > 1 trial rehearsed at one rank (the halo selection included)
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/halo_trace" -o trace -- \
        python3 tools/halo_time.py 256 2 20 40 > "$O/halo_time.jsonl" 2> "$O/halo_time.err" && \
      timeout -k 10 200 python3 tools/halo_time.py 256 4 20 40 >> "$O/halo_time.jsonl" 2>> "$O/halo_time.err" && \
      timeout -k 10 300 python bench.py --comm-self --rehearse-trial --no-cpu-baseline --side-steps 0 --general-steps 0 \
        > "$O/trial.json" 2> "$O/trial.err" ;;
    mbonly)
      # the whole N > 1 bench path (launcher, z-slab partition, trial, timed graph, max over ranks) on ONE
      # GPU: mailbox-only ranks (no RCCL, which refuses two ranks on a device), every rank on device 0
      EIGMI_FORCE_DEVICE=0 timeout -k 10 600 python bench.py --gpus 2 --transport mailbox-only --steps 50 --warmup 5 \
        > "$O/bench_mbonly2.json" 2> "$O/bench_mbonly2.err" && \
      EIGMI_FORCE_DEVICE=0 timeout -k 10 600 python bench.py --gpus 4 --transport mailbox-only --steps 50 --warmup 5 \
        > "$O/bench_mbonly4.json" 2> "$O/bench_mbonly4.err" ;;
    runs2l)
      # plane runs of the 2-line march (#16) and the 1-line march (#13): few long wave chains, one
      # workgroup per CU, vs the default plan
      timeout -k 10 300 python3 tools/lanczos_sweep.py --N 256 --rounds 3 --steps 40 \
        --variants fused:arrays#16,fused:arrays@1#16,fused:arrays@2#16,fused:arrays#13,fused:arrays@1#13,fused:arrays@2#13,fused:arrays@4#13,mv:arrays,mv:arrays@1,mv:arrays@2,mv:arrays@4 \
        > "$O/runs_256.jsonl" 2> "$O/runs.err" && \
      timeout -k 10 300 python3 tools/lanczos_sweep.py --N 128 --rounds 3 --steps 40 \
        --variants fused:arrays#13,fused:arrays#16,fused:arrays@1#16,fused:arrays@2#16,fused:arrays@4#16,fused:arrays@1#13,fused:arrays@2#13 \
        > "$O/runs_128.jsonl" 2>> "$O/runs.err" && \
      for s in 32 64 96 128; do
        timeout -k 10 200 python3 tools/lanczos_sweep.py --N 256 --slab $s --rounds 3 --steps 40 \
          --variants fused:arrays#13,fused:arrays#16,fused:arrays@1#16,fused:arrays@2#16,fused:arrays@1#13,fused:arrays@2#13 \
          >> "$O/runs_slab.jsonl" 2>> "$O/runs.err" || return 1
      done ;;
    chebsegs)
      timeout -k 10 400 python3 tools/cheb_segs.py 256 > "$O/cheb_segs.jsonl" 2> "$O/cheb_segs.err" ;;
    spmmruns)
      timeout -k 10 300 python3 tools/spmm_runs.py 128 256 > "$O/spmm_runs.jsonl" 2> "$O/spmm_runs.err" ;;
    threshold)
      # EIG_MARCH_2L_MIN_ROWS: variant 15 (#13) vs the 2-line march (#16) on 4 M / 6 M / 8 M-row slabs
      for s in 64 96 128; do
        timeout -k 10 200 python3 tools/lanczos_sweep.py --N 256 --slab $s --rounds 3 --steps 40 \
          --variants fused:arrays#13,fused:arrays#16 >> "$O/threshold.jsonl" 2>> "$O/threshold.err" || return 1
      done ;;
    ablation)
      timeout -k 10 300 tools/march_copy 256 values ablation 8 > "$O/march_copy_abl.jsonl" ;;
    c4)
      timeout -k 10 900 python -u -m pytest tests/test_loopback_c4.py -m gpu -v -s --timeout 900 --timeout-method thread \
        > "$O/c4.log" 2>&1 ;;
    slgram)
      timeout -k 10 200 python -u tools/bench_configs.py c1 c2 > "$O/cfg_c12.jsonl" 2> "$O/cfg.err" && \
      EIGMI_NO_SPMM_GRAM=1 timeout -k 10 200 python -u tools/bench_configs.py c1 c2 > "$O/cfg_c12_nogram.jsonl" 2>> "$O/cfg.err" && \
      run_task sltrace ;;
    detprobe)
      timeout -k 10 300 python3 -u tools/det_probe.py > "$O/det_probe.log" 2>&1 ;;
    round)
      run_task tests && run_task smoke && run_task profile && run_task bench ;;
    *)
      echo "unknown task $1" >&2; return 2 ;;
  esac
}

for t in "$@"; do
  echo "[gpu.sh] $t" >&2
  run_task "$t" || { echo "[gpu.sh] task $t failed (status $?)" >&2; exit 1; }
done
