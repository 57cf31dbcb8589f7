#!/bin/bash
# Round 4 call A: every GPU test and smoke(), then A/B against libmgx_r3.so (round 3's engine) on the driver's
# line, the default line and config 4; a kernel trace of the driver's line.
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_tests.sh                          # every GPU test + smoke()
TAG=gen20 ROUNDS=3 LIBS="- minigrid-rl_amd/mgx/libmgx_r3.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=gen2048 ROUNDS=2 LIBS="- minigrid-rl_amd/mgx/libmgx_r3.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=genc4 ROUNDS=1 LIBS="- minigrid-rl_amd/mgx/libmgx_r3.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
TAG=prod20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0" bash tools/gpu_trace.sh | tail -16
