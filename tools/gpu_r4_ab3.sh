#!/bin/bash
# Round 4: refill issue priority 3 and wave-uniform MT window top-up (2 / 4 groups left) on the driver's line,
# the default line and config 4.
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
TAG=v20 ROUNDS=2 LIBS="- $L/libmgx_prio3.so $L/libmgx_topup4.so $L/libmgx_topup2.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=v2048 ROUNDS=1 LIBS="- $L/libmgx_prio3.so $L/libmgx_topup4.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=vc4 ROUNDS=1 LIBS="- $L/libmgx_prio3.so $L/libmgx_topup4.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
