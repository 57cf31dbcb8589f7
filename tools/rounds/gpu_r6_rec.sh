#!/bin/bash
# Round 6: the epoch's prefix records beside the refill (mgx_prefix_epoch_kernel) and the rollout dispatched before the slide, with the
# rollout logic at priority 3 -- the whole GPU suite + smoke, then A/B against the prefix-record build with the same
# priority (ab_libs/libmgx_memolp3.so), rotating order: the driver's line, the default line, configs 4 and 5.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6rec
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
L="- ab_libs/libmgx_memolp3.so"
LIBS="$L" ROUNDS=3 TAG=rec20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_ab.sh
LIBS="$L" ROUNDS=1 TAG=rec2048 BENCH_ARGS="" bash tools/gpu_ab.sh
LIBS="$L" ROUNDS=1 TAG=recc4 BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
LIBS="$L" ROUNDS=1 TAG=recc5 BENCH_ARGS="--config 5" bash tools/gpu_ab.sh
