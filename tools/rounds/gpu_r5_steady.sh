#!/bin/bash
# Round 5: the driver's command and the default command with the steady-state window (bench.py --steady-ms)
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r5steady
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/k20.err || { tail -20 $O/k20.err; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
for f in $O/bench_k20.json $O/bench.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{\"metric')][0]); s=d.get('steady_state') or {}
print('$f'.split('/')[-1], 'value %.3e' % d['value'], 'paid %.3e' % d['value_resets_paid'], 'steady %.3e' % s.get('value', 0), 'p/c %.3f' % s.get('produced_over_consumed', 0), s.get('after_steps'), s.get('timed_steps'))"; done
