#!/bin/bash
# One gpurun call: GPU tests, then bench lines for BASELINE configs 4 and 5 (per-GPU share) and the PPO loop.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/gpu_tests.log | tail -30; exit 1; }
tail -2 $O/gpu_tests.log
for c in 4 5; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 0 > $O/bench_cfg$c.json 2>$O/bench_cfg$c.err || { tail -20 $O/bench_cfg$c.err; exit 1; }
  cat $O/bench_cfg$c.json
done
