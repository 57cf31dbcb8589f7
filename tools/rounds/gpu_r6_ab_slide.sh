#!/bin/bash
# Round 6 A/B (rotating order): the product (slide after the refill, the refill publishing its tails), the slide beside
# the refill (ab_libs/libmgx_sbeside.so), and commit 371b29a (the slide copying the tails) -- the driver's line.
set -e
cd $GRAFT_REPO_ROOT
LIBS="- ab_libs/libmgx_sbeside.so ab_libs/libmgx_c371.so" ROUNDS=${ROUNDS:-3} TAG=slide20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_ab.sh
LIBS="- ab_libs/libmgx_sbeside.so ab_libs/libmgx_c371.so" ROUNDS=2 TAG=slide2048 BENCH_ARGS="" bash tools/gpu_ab.sh
