#!/bin/bash
# Round 6: mgx_random_actions (tests), the marked-region trace of the driver's command, and its line with the torch
# replay vs a raw hipGraphLaunch (rotating order).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6c
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_random_actions.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TAG=c bash tools/gpu_r6_trace.sh | head -30
summ() { python -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1])
r=d['roofline']; s=d.get('steady_state') or {}
print('$1'.split('/')[-1], 'value %.3e steady %.3e ratio %.3f pc %.3f after %d frac %.3f kernel %.2f refill %.1f gpu_ms %.3f' % (d['value'], s.get('value',0), s.get('ratio_to_value',0), d['window']['produced_over_consumed'], d['steps_after_reset'], r['frac'], r['avg_launch_us'], (r.get('refill') or {}).get('avg_launch_us',0), d['gpu_time_ms']))
"; }
for i in 1 2; do
  for gl in torch raw; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0 --graph-launch $gl > $O/k20_${gl}_$i.json 2> $O/k20_${gl}_$i.err
    summ $O/k20_${gl}_$i.json
  done
done
