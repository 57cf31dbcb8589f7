#!/bin/bash
# Refill lead (MGX_REFILL_LEAD: the fork joins the refill of the epoch before last) x production ceiling
# (MGX_REFILL_CAPMAX: -1 auto, 0 none) on the fused pipeline of configs 2 / 4 / 5, two repeats.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lead
mkdir -p $O
summ() {
  python3 -c "
import json
for l in open('$1'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']; w=d['window']
        print('$2', 'value %.4e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'kernel %.2f' % r['avg_launch_us'], 'prod/cons %.4f' % (w['episodes_produced']/w['episodes_consumed']))"
}
for rep in 1 2; do
for CL in ${CONFIGS:-"2 fused" "4 fused" "5 fused"}; do
  set -- $CL
  for LM in ${LMS:-"0 0" "1 0" "0 -1" "1 -1"}; do
    set -- $CL $LM
    MGX_REFILL_LEAD=$3 MGX_REFILL_CAPMAX=$4 timeout -k 10 200 python bench.py --config $1 --layout $2 --both-layouts 0 --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    summ $O/b.json "lead=$3 capmax=$4 cfg$1 $2"
  done
done
done
