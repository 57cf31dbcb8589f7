#!/bin/bash
# Production rule A/B: per-wave mean consumption rounded up (MGX_REFILL_MEAN=2) vs grid-wide credit (3).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/m3
mkdir -p $O
for M in 3 2; do
  MGX_REFILL_MEAN=$M MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_rclock.so NS="65536" timeout -k 10 200 python tools/diag_refill_lanes.py | sed "s/^/mean=$M /"
done
for rep in 1 2; do
for M in 3 2; do
  for CL in "2 compact" "2 fused" "4 fused" "5 fused"; do
    set -- $CL
    MGX_REFILL_MEAN=$M timeout -k 10 200 python bench.py --config $1 --layout $2 --both-layouts 0 --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "
import json
for l in open('$O/b.json'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']; w=d['window']
        print('mean=$M cfg$1 $2', 'value %.4e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'kernel %.2f' % r['avg_launch_us'], 'p/c %.3f' % (w['episodes_produced']/w['episodes_consumed']))"
  done
done
done
