#!/bin/bash
# Round 4: what the refill's mission-token copy costs (elimination build: the fused layout reads no tokens).
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
TAG=nt20 ROUNDS=3 LIBS="- $L/libmgx_notok.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=nt2048 ROUNDS=1 LIBS="- $L/libmgx_notok.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=ntc4 ROUNDS=1 LIBS="- $L/libmgx_notok.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
