#!/bin/bash
# Deferred refill join: engine parity + PPO/compact GPU tests, driver-shaped line, default line.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_compact.py tests/test_vec_env.py tests/test_ppo.py -x -q -m gpu --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for a in "20 5" "2048 128" "20 5"; do
  set -- $a
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --cpu-seconds 0 --both-layouts 0 > $O/j.json 2>$O/j.err || { tail -5 $O/j.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/j.json')); r=d['roofline']
print('K $1 value %.4g ms/step %.5f step %.2f pipeline %.2f' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us']), d['window'])"
done
