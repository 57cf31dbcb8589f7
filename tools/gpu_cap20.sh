#!/bin/bash
# Refill cap A/B on the 20-step window (E = 20): engine default (4) vs 3.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for rep in 1 2; do for c in 0 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --refill-cap $c --cpu-seconds 0 --both-layouts 0 > $O/j.json 2>$O/j.err || { tail -5 $O/j.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/j.json')); r=d['roofline']
print('cap $c value %.4g gpu_ms %.4f pipeline %.2f' % (d['value'], d['gpu_time_ms'], r['step_pipeline_us']), d['window'])"
done; done
