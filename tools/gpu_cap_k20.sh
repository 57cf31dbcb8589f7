#!/bin/bash
# Refill production cap A/B on the driver-shaped window (--steps 20 --warmup 5, E = 20) and the
# default long window (E = 32).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for rep in 1 2; do
for a in "20 5 0" "20 5 3" "20 5 2" "2048 128 0" "2048 128 5"; do
  set -- $a
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --refill-cap $3 --cpu-seconds 0 --both-layouts 0 > $O/cap.json 2>$O/cap.err || { tail -5 $O/cap.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/cap.json')); r=d['roofline']
print('K $1 cap $3 value %.4g ms/step %.5f step %.2f pipeline %.2f' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us']), d['window'])"
done; done
