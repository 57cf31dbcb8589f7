#!/bin/bash
# Roofline probe check: default, driver-shaped and config-4 lines (probe avg vs pipeline).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for a in "2048 128 2" "20 5 2" "2048 128 4"; do
  set -- $a
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --config $3 --cpu-seconds 0 --both-layouts 0 > $O/j.json 2>$O/j.err || { tail -5 $O/j.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/j.json')); r=d['roofline']
print('K $1 config $3 value %.4g ms/step %.5f step %.2f pipeline %.2f frac %.3f' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us'], r['frac']))"
done
