#!/bin/bash
# A/B: step-kernel issue priority (MGX_STEP_PRIO) on BASELINE configs 4 and 5 (per GPU).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for C in 4 5; do for P in 0 1; do
  MGX_STEP_PRIO=$P timeout -k 10 200 python bench.py --config $C --cpu-seconds 0 --both-layouts 0 > $O/prio.json 2>$O/prio.err || { tail -5 $O/prio.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/prio.json')); r=d['roofline']
print('config $C prio $P value %.4g step %.2f us pipeline %.2f us' % (d['value'], r['avg_launch_us'], r['step_pipeline_us']))"
done; done
