#!/bin/bash
# Driver-shaped window (--steps 20 --warmup 5) A/B: refill epoch E (20 / 10) x step-kernel
# priority (MGX_STEP_PRIO 0 / 1), and the default long window at each priority.  Two repeats.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for rep in 1 2; do
for a in ${CASES:-"20 5 20 0" "20 5 10 0" "20 5 20 1" "20 5 10 1" "2048 128 0 0" "2048 128 0 1"}; do
  set -- $a
  MGX_STEP_PRIO=$4 timeout -k 10 200 python bench.py --steps $1 --warmup $2 --refill-every $3 --cpu-seconds 0 --both-layouts 0 > $O/ab.json 2>$O/ab.err || { tail -5 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/ab.json')); r=d['roofline']
print('K $1 E %d prio $4 value %.4g ms/step %.5f step %.2f pipeline %.2f' % (d['config']['refill_every'], d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us']), d['window'])"
done; done
