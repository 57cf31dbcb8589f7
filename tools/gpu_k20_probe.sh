#!/bin/bash
# Driver-shaped window diagnosis: E = 20 at a long window, the 20-step window with the refill
# serial, and 40 / 32-step windows.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for a in ${CASES:-"2000 128 0" "20 5 0" "20 5 1" "40 5 0" "32 5 0" "64 5 0"}; do
  set -- $a
  MGX_SERIAL_REFILL=$3 timeout -k 10 200 python bench.py --steps $1 --warmup $2 --cpu-seconds 0 --both-layouts 0 > $O/j.json 2>$O/j.err || { tail -5 $O/j.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/j.json')); r=d['roofline']
print('K $1 serial $3 value %.4g ms/step %.5f gpu_ms %.4f step %.2f pipeline %.2f E %d' % (d['value'], d['ms_per_step'], d['gpu_time_ms'], r['avg_launch_us'], r['step_pipeline_us'], d['config']['refill_every']), d['window'])"
done
