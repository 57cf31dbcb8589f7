#!/bin/bash
# Round 4: the rollout's barrier bound again now that the row stores come before the post-logic barrier:
# product (8) vs 4 / 12 / 16 on the default line and the driver's line.
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
TAG=vc2048 ROUNDS=2 LIBS="- $L/libmgx_vm4.so $L/libmgx_vm12.so $L/libmgx_vm16.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=vc20 ROUNDS=2 LIBS="- $L/libmgx_vm4.so $L/libmgx_vm12.so $L/libmgx_vm16.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
