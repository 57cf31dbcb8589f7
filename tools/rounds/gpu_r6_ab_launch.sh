#!/bin/bash
# Round 6: the random-policy tests + one fused-rollout parity file (the prepared-launch refactor of CompactBuffer.rollout),
# then A/B of the timed region's launch (hipGraph replay vs one prepared C call per chunk) on the driver's line and the
# default line, then the NT-store / slide-fence library A/B (tools/gpu_r6_ab_nt.sh).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_random_actions.py tests/test_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r6_launch_tests.log 2>&1 || { tail -40 $O/r6_launch_tests.log; exit 1; }
tail -1 $O/r6_launch_tests.log
VARIANTS="--launch graph|--launch eager" ROUNDS=3 TAG=launch20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_ab_args.sh
VARIANTS="--launch graph|--launch eager" ROUNDS=1 TAG=launch2048 BENCH_ARGS="" bash tools/gpu_ab_args.sh
bash tools/gpu_r6_ab_nt.sh
