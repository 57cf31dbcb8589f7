#!/bin/bash
# Generic A/B of bench.py variants: VARIANTS = newline-separated "label|ENV=.. ENV=..|bench args" lines,
# each run REPS times (default 2), one summary line per run.  -> gpurun_out/vab/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/vab
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
while IFS='|' read -r label envs args; do
  [ -z "$label" ] && continue
  env $envs timeout -k 10 240 python bench.py --both-layouts 0 --cpu-seconds 0 $args > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "
import json
for l in open('$O/b.json'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']; w=d['window']
        print('%-28s' % '$label', 'value %.4e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'kernel %.2f' % r['avg_launch_us'], 'E %d' % d['config']['refill_every'], 'prod/cons %.4f' % (w['episodes_produced']/w['episodes_consumed']))"
done <<< "$VARIANTS"
done
