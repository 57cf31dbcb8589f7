#!/bin/bash
# Compact layout: parity tests (gather vs materialised stacks, collectors), then a short PPO bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_compact.py tests/test_ppo.py -x -v -m gpu --timeout 300 --timeout-method thread -rf > $O/gpu_compact.log 2>&1 || { tail -60 $O/gpu_compact.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/gpu_compact.log | tail -12
timeout -k 10 600 python bench.py --workload ppo --steps 2 --warmup 1 --horizon 16 > $O/ppo16.json 2>$O/ppo16.err || { tail -20 $O/ppo16.err; exit 1; }
cat $O/ppo16.json; tail -4 $O/ppo16.err
