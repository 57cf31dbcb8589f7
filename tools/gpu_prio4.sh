#!/bin/bash
# Refill issue priority 0 vs 2 on the other configs / layouts.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/p4
mkdir -p $O
summ() {
  python3 -c "
import json
for l in open('$1'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']
        print('$2', 'value %.4e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'kernel %.2f' % r['avg_launch_us'])"
}
for rep in 1 2; do
for P in 0 2; do
  for CL in "2 compact" "4 compact" "4 fused" "5 fused" "5 compact"; do
    set -- $CL
    MGX_REFILL_PRIO=$P timeout -k 10 200 python bench.py --config $1 --layout $2 --both-layouts 0 --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    summ $O/b.json "prio=$P cfg$1 $2"
  done
done
done
