#!/bin/bash
# Refill issue priority (MGX_REFILL_PRIO) x layout on config 2 (and 5), two repeats.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prio
mkdir -p $O
for rep in 1 2; do
for cfg in ${CFGS:-2}; do
for lay in fused compact; do
for pr in 0 1 3; do
  MGX_REFILL_PRIO=$pr timeout -k 10 300 python bench.py --config $cfg --layout $lay --both-layouts 0 --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/b.json')); r=d['roofline']
print('rep $rep cfg $cfg $lay prio $pr value %.4e ms/step %.4f kernel/step %.2f' % (d['value'], d['ms_per_step'], r['avg_launch_us']))"
done; done; done; done
