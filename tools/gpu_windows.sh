#!/bin/bash
# Bench lines at several window lengths (--steps K --warmup W pairs given as "K W" arguments).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for a in "$@"; do
  set -- $a
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --cpu-seconds 0 --both-layouts 0 > $O/j.json 2>$O/j.err || { tail -5 $O/j.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/j.json')); r=d['roofline']
print('K $1 value %.4g ms/step %.5f gpu_ms %.4f step %.2f pipeline %.2f E %d warmup %d' % (d['value'], d['ms_per_step'], d['gpu_time_ms'], r['avg_launch_us'], r['step_pipeline_us'], d['config']['refill_every'], d['warmup']), d['window'])"
done
