#!/bin/bash
# A/B: step-kernel issue priority over the concurrent refill (MGX_STEP_PRIO), compact headline workload.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for rep in 1 2; do for P in 0 1 3; do
  MGX_STEP_PRIO=$P timeout -k 10 120 python bench.py --cpu-seconds 0 --both-layouts 0 > $O/prio.json 2>$O/prio.err || { tail -5 $O/prio.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/prio.json')); r=d['roofline']
print('prio $P value %.4g step %.2f us pipeline %.2f us' % (d['value'], r['avg_launch_us'], r['step_pipeline_us']))"
done; done
