#!/bin/bash
# Round 4: launch order (refill first = product, rollout first) and the Bresenham round cap (bres) on the
# 20-step line, the default line and configs 4 and 5.
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
TAG=o20 ROUNDS=2 LIBS="- $L/libmgx_rollfirst.so $L/libmgx_bres.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=o2048 ROUNDS=1 LIBS="- $L/libmgx_rollfirst.so $L/libmgx_bres.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=oc4 ROUNDS=1 LIBS="- $L/libmgx_rollfirst.so $L/libmgx_bres.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
TAG=oc5 ROUNDS=1 LIBS="- $L/libmgx_rollfirst.so" BENCH_ARGS="--config 5" bash tools/gpu_ab.sh
