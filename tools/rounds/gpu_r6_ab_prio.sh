#!/bin/bash
# Round 6 A/B (rotating order), with the prefix records in (the refill and the rollout now balanced): the rollout's
# step logic at issue priority 3 (lprio3), the refill at priority 1 / 3 instead of 2, both (lp3p1) -- the driver's line,
# then config 4 and the default line.
set -e
cd $GRAFT_REPO_ROOT
L="- ab_libs/libmgx_lprio3.so ab_libs/libmgx_prio1.so ab_libs/libmgx_prio3.so ab_libs/libmgx_lp3p1.so"
LIBS="$L" ROUNDS=${ROUNDS:-3} TAG=prio20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_ab.sh
LIBS="$L" ROUNDS=1 TAG=prio2048 BENCH_ARGS="" bash tools/gpu_ab.sh
LIBS="$L" ROUNDS=1 TAG=prioc4 BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
