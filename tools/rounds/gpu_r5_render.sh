#!/bin/bash
# Round 5: the dword-writing render (render_row) -- the fused-rollout parity tests, then A/B against the previous
# build (ab_libs/libmgx_base.so) on the driver's line and config 5.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rollout.py tests/test_gpu_parity.py tests/test_compact.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/render_tests.log 2>&1 || { tail -40 gpurun_out/render_tests.log; exit 1; }
tail -2 gpurun_out/render_tests.log
LIBS="- ab_libs/libmgx_base.so" BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --host-wait spin" ROUNDS=3 TAG=render_k20 bash tools/gpu_ab.sh
LIBS="- ab_libs/libmgx_base.so" BENCH_ARGS="--config 5 --host-wait spin" ROUNDS=1 TAG=render_c5 bash tools/gpu_ab.sh
LIBS="- ab_libs/libmgx_base.so" BENCH_ARGS="--host-wait spin" ROUNDS=1 TAG=render_def bash tools/gpu_ab.sh
