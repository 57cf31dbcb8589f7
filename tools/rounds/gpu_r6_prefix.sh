#!/bin/bash
# Round 6: the marginal cost of the MT-only generator prefix -- a build that runs every prefix draw
# sequence twice (ab_libs/libmgx_prefix2.so; outputs unchanged: the fixture tests run on it) vs the product, rotating
# order: the driver's line, config 4 (refill-bound), the default line.
set -e
cd $GRAFT_REPO_ROOT
MGX_LIB_PATH=$GRAFT_REPO_ROOT/ab_libs/libmgx_prefix2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fixture" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_prefix_tests.log 2>&1 || { tail -30 gpurun_out/r6_prefix_tests.log; exit 1; }
tail -1 gpurun_out/r6_prefix_tests.log
LIBS="- ab_libs/libmgx_prefix2.so" ROUNDS=3 TAG=prefix20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_ab.sh
LIBS="- ab_libs/libmgx_prefix2.so" ROUNDS=2 TAG=prefixc4 BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
