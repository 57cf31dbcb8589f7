#!/bin/bash
# Refill epoch length / production cap sweep on the compact-layout rollout bench (steady state: long warm-up).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for EC in "32 5" "32 6" "32 7" "32 5" "32 6"; do
  set -- $EC; E=$1; C=$2
  timeout -k 10 120 python bench.py --steps 2048 --warmup 2048 --cpu-seconds 0 --both-layouts 0 --refill-every $E --refill-cap $C > $O/sw.json 2>$O/sw.err || { tail -5 $O/sw.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/sw.json')); r=d['roofline']; w=d['window']
print('E=$E cap=$C value %.4g step %.2f us pipeline %.2f us produced/consumed %.4f' % (d['value'], r['avg_launch_us'], r['step_pipeline_us'], w['episodes_produced']/w['episodes_consumed']))"
done
