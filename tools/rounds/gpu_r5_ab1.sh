#!/bin/bash
# Round 5 A/B 1: fence-free MT slide (product) vs __threadfence slide; ring_pubn acquire (product) vs relaxed;
# logic-phase priority 3 vs none -- on the driver's 20-step line and the default line.  Parity first.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rollout.py tests/test_gpu_parity.py -k "bench_shape or mt_ or clock or wrap or full_size or shards" \
  -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/ab1_tests.log 2>&1 || { tail -40 gpurun_out/ab1_tests.log; exit 1; }
tail -2 gpurun_out/ab1_tests.log
K20="--steps 20 --warmup 5"
TAG=r5k20 ROUNDS=3 LIBS="- ab_libs/libmgx_sfence.so ab_libs/libmgx_relaxed.so ab_libs/libmgx_lprio3.so" BENCH_ARGS="$K20" bash tools/gpu_ab.sh
TAG=r5def ROUNDS=2 LIBS="- ab_libs/libmgx_lprio3.so ab_libs/libmgx_sfence.so" BENCH_ARGS="" bash tools/gpu_ab.sh
echo done
