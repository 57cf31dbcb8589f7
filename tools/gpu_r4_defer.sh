#!/bin/bash
# Round 4: the fused rollout with deferred row copy-out (product): fused parity tests, smoke, then A/B against
# the end-of-step copy-out (nodefer) on the driver's line (3 rounds), the default line and config 5.
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
timeout -k 10 700 python -u -m pytest tests/test_rollout.py tests/test_gpu_parity.py -k "rollout or fused or bench_shape or wrap or shards" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/defer_tests.log 2>&1 || { tail -30 gpurun_out/defer_tests.log; exit 1; }
tail -1 gpurun_out/defer_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
TAG=df20 ROUNDS=3 LIBS="- $L/libmgx_nodefer.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=df2048 ROUNDS=2 LIBS="- $L/libmgx_nodefer.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=dfc5 ROUNDS=1 LIBS="- $L/libmgx_nodefer.so" BENCH_ARGS="--config 5" bash tools/gpu_ab.sh
