#!/bin/bash
# Round 6: ring depth 512 (default) with fresh actions -- the ring levels over 20,000 steps, the driver's command twice,
# the default command and configs 4 / 5 (headline window >= 20,480 steps after the reset, steady_state beside it).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6b
mkdir -p $O
cd $R
timeout -k 10 240 env ACTIONS=fresh WINDOWS=${WINDOWS:-20} python -u tools/diag_ring_levels.py > $O/levels_fresh512.jsonl 2> $O/levels_fresh512.err
tail -1 $O/levels_fresh512.jsonl
summ() { python -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1])
r=d['roofline']; s=d.get('steady_state') or {}
print('$1'.split('/')[-1], 'value %.3e steady %.3e ratio %.3f pc %.3f steady_pc %.3f after %d frac %.3f kernel %.2f refill %.1f' % (d['value'], s.get('value',0), s.get('ratio_to_value',0), d['window']['produced_over_consumed'], s.get('produced_over_consumed',0), d['steps_after_reset'], r['frac'], r['avg_launch_us'], (r.get('refill') or {}).get('avg_launch_us',0)))
for k in ('compact_layout','sb3_layout'):
    if k in d: print('  ', k, '%.3e' % d[k]['value'], 'frac %.3f' % d[k]['roofline']['frac'])
"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_k20_$i.json 2> $O/bench_k20_$i.err
  summ $O/bench_k20_$i.json
done
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > $O/bench_default.json 2> $O/bench_default.err
summ $O/bench_default.json
timeout -k 10 300 python -u bench.py --config 4 --cpu-seconds 0 --both-layouts 0 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
summ $O/bench_cfg4.json
timeout -k 10 300 python -u bench.py --config 5 --cpu-seconds 0 --both-layouts 0 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
summ $O/bench_cfg5.json
