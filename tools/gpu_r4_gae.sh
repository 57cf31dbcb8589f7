#!/bin/bash
# Round 4: GAE fused into the rollout launch (mgx_rollout_compact_gae): the bench-shape graph tests (fused,
# fused_gae, compact at 8,192 and 65,536 envs) and the rollout tests, then the driver's line with and without
# the fused GAE (3 rounds interleaved), and a kernel trace.
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_rollout.py tests/test_abi.py -k "bench_shape or rollout or abi or export" -m "gpu or not gpu" -x -q --timeout 300 --timeout-method thread > gpurun_out/gae_tests.log 2>&1 || { tail -30 gpurun_out/gae_tests.log; exit 1; }
tail -1 gpurun_out/gae_tests.log
O=gpurun_out
for r in 1 2 3; do
  for g in 1 0; do
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0 --gae-fused $g > $O/gae_line.json 2> $O/gae_err.log || { tail -20 $O/gae_err.log; exit 1; }
    python -c "import json; d=json.load(open('$O/gae_line.json')); r=d['roofline']; print('gae_fused=$g', '%.3e'%d['value'], 'pipe_us=%.2f'%r['step_pipeline_us'], d['config']['timed'][-60:])"
  done
done
TAG=gae20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0" bash tools/gpu_trace.sh | sed -n 12,18p
