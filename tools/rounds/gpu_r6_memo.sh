#!/bin/bash
# Round 6: the MT-only generator prefix looked up in per-position records (product) -- the whole
# GPU suite + smoke, then A/B against the same build drawing every prefix (ab_libs/libmgx_nomemo.so), rotating order:
# the driver's line, config 4, config 5, the default line.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6memo
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
LIBS="- ab_libs/libmgx_nomemo.so" ROUNDS=3 TAG=memo20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_ab.sh
LIBS="- ab_libs/libmgx_nomemo.so" ROUNDS=2 TAG=memoc4 BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
LIBS="- ab_libs/libmgx_nomemo.so" ROUNDS=1 TAG=memoc5 BENCH_ARGS="--config 5" bash tools/gpu_ab.sh
LIBS="- ab_libs/libmgx_nomemo.so" ROUNDS=1 TAG=memo2048 BENCH_ARGS="" bash tools/gpu_ab.sh
