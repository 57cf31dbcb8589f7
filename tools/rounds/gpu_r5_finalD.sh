#!/bin/bash
# Round 5, last: the bench lines of the final bench.py (headline window + steady_state) -> gpurun_out/r5final/
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r5final
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/k20.err || { tail -20 $O/k20.err; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --config 4 --cpu-seconds 0 > $O/bench_cfg4.json 2> $O/cfg4.err || { tail -20 $O/cfg4.err; exit 1; }
timeout -k 10 300 python bench.py --config 5 --cpu-seconds 0 > $O/bench_cfg5.json 2> $O/cfg5.err || { tail -20 $O/cfg5.err; exit 1; }
for f in $O/bench*.json; do python3 -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{\"metric')][0]); s=d.get('steady_state') or {}; r=d['roofline']
print('$f'.split('/')[-1], 'value %.3e' % d['value'], 'frac %.3f' % r['frac'], 'paid %.3e' % d['value_resets_paid'], 'steady %.3e' % s.get('value', 0), 'p/c %.3f' % s.get('produced_over_consumed', 0), 'rocprof_timed', (r.get('rocprof') or {}).get('timed_frac'))"; done
