#!/bin/bash
# Round 6: the slide beside the refill (fork_end) and the refill publishing its own tails -- the GPU suite, smoke, the
# driver's line x2, the default line, configs 4 / 5.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6e
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
summ() { python -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1])
r=d['roofline']; s=d.get('steady_state') or {}
print('$1'.split('/')[-1], 'value %.3e steady %.3e ratio %.3f pc %.3f after %d frac %.3f kernel %.2f refill %.1f slide %.1f gpu_ms %.3f' % (d['value'], s.get('value',0), s.get('ratio_to_value',0), d['window']['produced_over_consumed'], d['steps_after_reset'], r['frac'], r['avg_launch_us'], (r.get('refill') or {}).get('avg_launch_us',0), (r.get('refill') or {}).get('slide_avg_launch_us') or 0, d['gpu_time_ms']))
for k in ('compact_layout','sb3_layout'):
    if k in d: print('  ', k, '%.3e' % d[k]['value'], 'frac %.3f' % d[k]['roofline']['frac'])
"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts $((i-1)) > $O/k20_$i.json 2> $O/k20_$i.err
  summ $O/k20_$i.json
done
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --both-layouts 0 > $O/default.json 2> $O/default.err
summ $O/default.json
timeout -k 10 300 python -u bench.py --config 4 --cpu-seconds 0 --both-layouts 0 > $O/cfg4.json 2> $O/cfg4.err
summ $O/cfg4.json
timeout -k 10 300 python -u bench.py --config 5 --cpu-seconds 0 --both-layouts 0 > $O/cfg5.json 2> $O/cfg5.err
summ $O/cfg5.json
