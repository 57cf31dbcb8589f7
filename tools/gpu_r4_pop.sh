#!/bin/bash
# Round 4: rollout resets counted by ballot + popcount: fused tests (counts included), A/B against the per-pop
# LDS atomic on the default line and the driver's line; then the PPO lines (horizon 16 and 1024).
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
timeout -k 10 700 python -u -m pytest tests/test_rollout.py tests/test_gpu_parity.py -k "rollout or fused or bench_shape or accounting or stats" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pop_tests.log 2>&1 || { tail -30 gpurun_out/pop_tests.log; exit 1; }
tail -1 gpurun_out/pop_tests.log
TAG=pc2048 ROUNDS=2 LIBS="- $L/libmgx_popatomic.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=pc20 ROUNDS=2 LIBS="- $L/libmgx_popatomic.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
bash tools/gpu_ppo.sh 2>&1 | grep -E '^\{' | cut -c1-200
