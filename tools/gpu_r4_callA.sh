#!/bin/bash
# Round 4 call A: the generator changes (randbelow_seq, pcg_cell, object choice folded into draw_cell) and the
# rollout-before-refill launch order through the parity tests, then A/B against libmgx_r3.so (the round-3
# generator, same engine) on the driver's line, the default line and config 4; a kernel trace of the driver's line.
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_rollout.py -k "fixture or oracle_1024 or full_size or bench_shape or reset_paths or shards or wrap or equals_per_step" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/a_tests.log 2>&1 || { tail -30 gpurun_out/a_tests.log; exit 1; }
tail -2 gpurun_out/a_tests.log
TAG=gen20 ROUNDS=3 LIBS="- minigrid-rl_amd/mgx/libmgx_r3.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=gen2048 ROUNDS=2 LIBS="- minigrid-rl_amd/mgx/libmgx_r3.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=genc4 ROUNDS=1 LIBS="- minigrid-rl_amd/mgx/libmgx_r3.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
TAG=prod20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0" bash tools/gpu_trace.sh | tail -16
