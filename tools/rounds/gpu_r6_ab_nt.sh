#!/bin/bash
# Round 6 A/B (rotating order): non-temporal row stores (fused rollout), + non-temporal ring records (refill), + the slide
# without its L2 write-back (MGX_SLIDE_FENCE=0), the slide alone without it -- the driver's line, then the default
# line; then the timed region's launch (hipGraph replay vs one prepared C call per chunk) on the product library.
set -e
cd $GRAFT_REPO_ROOT
L="- ab_libs/libmgx_ntrows.so ab_libs/libmgx_ntboth.so ab_libs/libmgx_ntboth_sf0.so ab_libs/libmgx_sfence0.so"
LIBS="$L" ROUNDS=${ROUNDS:-3} TAG=nt20b BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_ab.sh
LIBS="$L" ROUNDS=1 TAG=nt2048b BENCH_ARGS="" bash tools/gpu_ab.sh
VARIANTS="--launch graph|--launch eager" ROUNDS=3 TAG=launch20b BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_ab_args.sh
