#!/bin/bash
# Refill epoch length / production cap sweep on the compact-layout rollout bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for E in 16 32 64; do for C in 4 6 8; do
  timeout -k 10 120 python bench.py --steps 2048 --cpu-seconds 0 --both-layouts 0 --refill-every $E --refill-cap $C > $O/sw_${E}_${C}.json 2>$O/sw.err || { tail -5 $O/sw.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/sw_${E}_${C}.json')); r=d['roofline']; w=d['window']
print('E=$E cap=$C value %.4g step %.2f us pipeline %.2f us produced/consumed %.4f' % (d['value'], r['avg_launch_us'], r['step_pipeline_us'], w['episodes_produced']/w['episodes_consumed']))"
done; done
