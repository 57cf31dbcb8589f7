#!/bin/bash
# Step-kernel priority (MGX_STEP_PRIO 0 / 1) A/B on configs 2 / 4 / 5 at the default window and
# the driver-shaped one (--steps 20 --warmup 5).  Two repeats, interleaved.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for rep in 1 2; do
for c in 4 5 2; do
for w in "2048 128" "20 5"; do
for pr in 0 1; do
  set -- $w
  MGX_STEP_PRIO=$pr timeout -k 10 200 python bench.py --config $c --steps $1 --warmup $2 --cpu-seconds 0 --both-layouts 0 > $O/pab.json 2>$O/pab.err || { tail -5 $O/pab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/pab.json')); r=d['roofline']
print('cfg $c K $1 prio $pr value %.4g ms/step %.5f step %.2f pipeline %.2f' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us']))"
done; done; done; done
