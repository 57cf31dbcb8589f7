#!/bin/bash
# Round 5 A/B 2 (rotating order): logic-phase priority 3, the fenced MT slide, both, both + relaxed pubn, vs the
# product -- on the driver's 20-step line (separate GAE and the LDS-staged fused GAE epilogue) and the default
# line.  Parity of the fused-GAE / bench-shape paths first.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_rollout.py -k "bench_shape or clock or gae" \
  -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/ab2_tests.log 2>&1 || { tail -40 gpurun_out/ab2_tests.log; exit 1; }
tail -2 gpurun_out/ab2_tests.log
K20="--steps 20 --warmup 5"
L="- ab_libs/libmgx_lprio3.so ab_libs/libmgx_sfence.so ab_libs/libmgx_lp3sf.so ab_libs/libmgx_lp3sfrx.so"
TAG=r5k20b ROUNDS=3 LIBS="$L" BENCH_ARGS="$K20" bash tools/gpu_ab.sh
TAG=r5k20g ROUNDS=2 LIBS="- ab_libs/libmgx_lp3sf.so" BENCH_ARGS="$K20 --gae-fused 1" bash tools/gpu_ab.sh
TAG=r5defb ROUNDS=1 LIBS="- ab_libs/libmgx_lprio3.so ab_libs/libmgx_lp3sf.so" BENCH_ARGS="" bash tools/gpu_ab.sh
echo done
