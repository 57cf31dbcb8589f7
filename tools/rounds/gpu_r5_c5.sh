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
# the driver's line with its chunk replayed from a hipGraph (default) vs enqueued eagerly, interleaved
for r in 1 2 3; do
  for g in 1 0; do
    timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0 --graph $g > gpurun_out/g_line.json 2> gpurun_out/g_err.log || { tail -20 gpurun_out/g_err.log; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/g_line.json')); r=d['roofline']; print('graph=$g', '%.3e'%d['value'], 'kern_us=%.2f'%r['avg_launch_us'], 'pipe_us=%.2f'%r['step_pipeline_us'], 'refill_us=%.1f'%(r.get('refill') or {}).get('avg_launch_us', 0))" | tee -a gpurun_out/ab_r5graph.txt
  done
done
echo done
