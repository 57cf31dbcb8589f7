#!/bin/bash
# Round 4: MT slide with its loads ahead of its stores: the slide/ring/MT tests and the fused graph test, then
# A/B against the previous slide (libmgx_oldslide.so, built from the previous commit's source) on the driver's
# line (3 rounds) and the default line, and a kernel trace of the driver's line.
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_rollout.py -k "mt_stream or refill or ring or bench_shape or full_size or shards" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/slide_tests.log 2>&1 || { tail -30 gpurun_out/slide_tests.log; exit 1; }
tail -1 gpurun_out/slide_tests.log
TAG=sl20 ROUNDS=3 LIBS="- $L/libmgx_oldslide.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=sl2048 ROUNDS=1 LIBS="- $L/libmgx_oldslide.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=slide20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0" bash tools/gpu_trace.sh | sed -n 10,20p
