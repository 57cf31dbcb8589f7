#!/bin/bash
# Round 5 A/B 4: the fused rollout's grouped LDS reads (product) vs the previous build, parity of the rollout paths
# first; then the GTG model after its second segment under the test() protocol.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rollout.py tests/test_gpu_parity.py -k "rollout or bench_shape" \
  -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/ab4_tests.log 2>&1 || { tail -40 gpurun_out/ab4_tests.log; exit 1; }
tail -2 gpurun_out/ab4_tests.log
TAG=r5k20c ROUNDS=3 LIBS="- ab_libs/libmgx_prev.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=r5defc ROUNDS=2 LIBS="- ab_libs/libmgx_prev.so" BENCH_ARGS="" bash tools/gpu_ab.sh
timeout -k 10 600 python -u tools/eval_protocol.py --ckpt eval_ck/gtg2_ck.pt --columns GTG,ALL --fresh 0 --out gpurun_out/eval_gtg2.json 2> gpurun_out/eval_gtg2.err || { tail -20 gpurun_out/eval_gtg2.err; exit 1; }
echo done
