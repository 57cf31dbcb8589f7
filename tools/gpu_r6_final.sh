#!/bin/bash
# Round 6 final lines on the final build -> gpurun_out/r6final/ (copied to profiles/r06_bench/final/): the driver's
# command exactly as it runs it (x2: its cpu_baseline leg and the second layouts included), the default line,
# configs 4 and 5, and the PPO loop at horizon 16.  Each run has its own time limit; the first failure ends the call.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6final
mkdir -p $O
cd $R
python3 -c "import hashlib; print(hashlib.sha256(open('minigrid-rl_amd/mgx/libmgx.so','rb').read()).hexdigest()[:16])" > $O/lib_sha16.txt
summ() { python -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1])
r=d['roofline']; s=d.get('steady_state') or {}
if 'window' not in d: print('$1'.split('/')[-1], 'value %.3e' % d['value']); sys.exit(0)
print('$1'.split('/')[-1], 'value %.3e steady %.3e ratio %.3f pc %.3f after %d frac %.3f kernel %.2f refill %.1f gpu_ms %.3f traffic %s' % (d['value'], s.get('value',0), s.get('ratio_to_value',0), d['window']['produced_over_consumed'], d['steps_after_reset'], r['frac'], r['avg_launch_us'], (r.get('refill') or {}).get('avg_launch_us',0), d['gpu_time_ms'], r.get('traffic')))
for k in ('compact_layout','sb3_layout'):
    if k in d: print('  ', k, '%.3e' % d[k]['value'], 'frac %.3f' % d[k]['roofline']['frac'])
"; }
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || { tail -20 $O/driver_$i.err; exit 1; }
  summ $O/driver_$i.json
done
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --both-layouts 0 > $O/default.json 2> $O/default.err || { tail -20 $O/default.err; exit 1; }
summ $O/default.json
timeout -k 10 300 python -u bench.py --config 4 --cpu-seconds 0 --both-layouts 0 > $O/cfg4.json 2> $O/cfg4.err || { tail -20 $O/cfg4.err; exit 1; }
summ $O/cfg4.json
timeout -k 10 300 python -u bench.py --config 5 --cpu-seconds 0 --both-layouts 0 > $O/cfg5.json 2> $O/cfg5.err || { tail -20 $O/cfg5.err; exit 1; }
summ $O/cfg5.json
timeout -k 10 400 python -u bench.py --workload ppo --steps 2 --warmup 1 --horizon 16 --cpu-seconds 0 > $O/ppo16.json 2> $O/ppo16.err || { tail -20 $O/ppo16.err; exit 1; }
summ $O/ppo16.json
