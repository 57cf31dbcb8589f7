#!/bin/bash
# Round 4: 32-env refill waves (auto below one 64-env wave per SIMD): every GPU test (small-N tests run the
# 32-env waves), then A/B against 64-env waves at config 4 and the 20-step line (config 2 keeps 64).
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
bash tools/gpu_tests.sh
TAG=epw_c4 ROUNDS=2 LIBS="- $L/libmgx_epw64.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
TAG=epw_k20 ROUNDS=1 LIBS="- $L/libmgx_epw32.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
