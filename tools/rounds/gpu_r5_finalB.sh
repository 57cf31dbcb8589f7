#!/bin/bash
# Round 5 closing pass B (after pass A's profiles are committed under profiles/r05_pmc/): the bench lines -- the
# driver's command, the default command, configs 4 and 5, the PPO workload at horizon 16 -> gpurun_out/r5bench/.
# Then the N > 1 rehearsal (tools/gpu_dp_rehearsal.sh: gloo ranks on the one GPU).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r5bench
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/k20.err || { tail -20 $O/k20.err; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --config 4 --cpu-seconds 0 > $O/bench_cfg4.json 2> $O/cfg4.err || { tail -20 $O/cfg4.err; exit 1; }
timeout -k 10 300 python bench.py --config 5 --cpu-seconds 0 > $O/bench_cfg5.json 2> $O/cfg5.err || { tail -20 $O/cfg5.err; exit 1; }
timeout -k 10 500 python bench.py --workload ppo --steps 2 --warmup 1 --horizon 16 > $O/bench_ppo16.json 2> $O/ppo16.err || { tail -20 $O/ppo16.err; exit 1; }
for f in $O/bench*.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{\"metric')][0]); r=d.get('roofline') or {}
print('$f'.split('/')[-1], '%.3e' % d['value'], d['ms_per_step'], 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'rocprof', (r.get('rocprof') or {}).get('timed_frac'))"; done
bash $R/tools/gpu_dp_rehearsal.sh
