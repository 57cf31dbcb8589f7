#!/bin/bash
# Refill issue priority vs the fused rollout (config 2) and the driver-shaped 20-step window per layout.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/p3
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
for P in 0 1 2 3; do
  MGX_REFILL_PRIO=$P timeout -k 10 200 python bench.py --config 2 --layout fused --both-layouts 0 --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  summ $O/b.json "prio=$P cfg2 fused"
done
done
for L in fused compact; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --layout $L --both-layouts 0 --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  summ $O/b.json "k20 $L"
done
