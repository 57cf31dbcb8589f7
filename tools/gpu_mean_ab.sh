#!/bin/bash
# Refill production capped at the wave's mean deficit (MGX_REFILL_MEAN=1, default) vs the busiest
# lane's (0): ring / refill / full-size GPU tests, then configs 2 (default and driver-shaped
# windows), 4 and 5, interleaved, two repeats.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "ring or refill or reset_paths or full_size or oracle_1024 or reference_fixture" > $O/mean_tests.log 2>&1 || { tail -40 $O/mean_tests.log; exit 1; }
tail -2 $O/mean_tests.log
for rep in 1 2; do
for a in "2 20 5" "2 2048 128" "4 2048 128" "5 2048 128"; do
for m in 0 1; do
  set -- $a
  MGX_REFILL_MEAN=$m timeout -k 10 200 python bench.py --config $1 --steps $2 --warmup $3 --cpu-seconds 0 --both-layouts 0 > $O/mab.json 2>$O/mab.err || { tail -5 $O/mab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/mab.json')); r=d['roofline']
print('cfg $1 K $2 mean $m value %.4g ms/step %.5f step %.2f pipeline %.2f' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us']), d['window'])"
done; done; done
