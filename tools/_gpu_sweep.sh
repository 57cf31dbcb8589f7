#!/bin/bash
# One gpurun call: bench.py under refill-schedule knobs ("name:--flag v --flag v").
set -e
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; args=""; [ "$spec" != "$name" ] && args=${spec#*:}
  timeout -k 10 200 python bench.py --steps 1024 --warmup 64 --cpu-seconds 0 --probe 128 $args > gpurun_out/sw_$name.json 2>gpurun_out/sw_$name.err
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$name.json')); r=d['roofline']; print('%-10s %-40s %.3f G/s %6.2f us/step kernel %6.2f us' % ('$name', '$args', d['value']/1e9, d['ms_per_step']*1e3, r['avg_launch_us']))"
done
