#!/bin/bash
# Round 4: bounded rollout barriers, more repeats: product (__syncthreads) vs vmcnt(4 / 6 / 8 / 12) on the
# driver's line (3 rounds) and the default line (2 rounds).
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
TAG=vmb20 ROUNDS=3 LIBS="- $L/libmgx_vm4.so $L/libmgx_vm6.so $L/libmgx_vm8.so $L/libmgx_vm12.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=vmb2048 ROUNDS=2 LIBS="- $L/libmgx_vm4.so $L/libmgx_vm6.so $L/libmgx_vm8.so $L/libmgx_vm12.so" BENCH_ARGS="" bash tools/gpu_ab.sh
