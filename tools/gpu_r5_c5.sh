#!/bin/bash
# Round 5: 32-env rollout blocks at S = 16 (config 5) -- parity of the S = 16 rollout paths with that build
# (fixtures, full-size config-5 oracle compare, shards), then config 5 A/B vs the product; then the test()
# protocol evaluation of the GTG checkpoint (GTG and ALL columns).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
MGX_LIB_PATH=$R/ab_libs/libmgx_epb32.so timeout -k 10 600 python -u -m pytest tests/test_rollout.py -k "s16 or size16 or 16 or cfg5 or 131072 or clock" \
  -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/c5_tests.log 2>&1 || { tail -40 gpurun_out/c5_tests.log; exit 1; }
tail -2 gpurun_out/c5_tests.log
TAG=r5c5 ROUNDS=2 LIBS="- ab_libs/libmgx_epb32.so" BENCH_ARGS="--config 5" BENCH_TIMEOUT=300 bash tools/gpu_ab.sh
timeout -k 10 600 python -u tools/eval_protocol.py --ckpt eval_ck/gtg_ck.pt --columns GTG,ALL --fresh 0 --out gpurun_out/eval_gtg.json 2> gpurun_out/eval_gtg.err || { tail -20 gpurun_out/eval_gtg.err; exit 1; }
echo done
