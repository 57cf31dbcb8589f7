#!/bin/bash
# Round-3 closing pass, part 2: configs 4 and 5 (default layouts) and config 3 (PPO, horizon 16,
# with the deterministic success-rate evaluation).  -> gpurun_out/final/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench2.json 2> $O/bench2.err || { tail -20 $O/bench2.err; exit 1; }
grep '^{"metric' $O/bench2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['config']['layout'], '%.4e' % d['value'], d['ms_per_step'], d['warmup'], d['roofline']['frac'], {k: '%.3e' % d[k]['value'] for k in d if k.endswith('_layout')})"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench2_k20.json 2> $O/bench2_k20.err || { tail -20 $O/bench2_k20.err; exit 1; }
grep '^{"metric' $O/bench2_k20.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k20', d['config']['layout'], '%.4e' % d['value'], d['ms_per_step'], d['warmup'], d['roofline']['frac'])"
for C in 4 5; do
  timeout -k 10 300 python bench.py --config $C --cpu-seconds 0 > $O/bench_cfg$C.json 2> $O/bench_cfg$C.err || { tail -20 $O/bench_cfg$C.err; exit 1; }
  grep '^{"metric' $O/bench_cfg$C.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg$C', d['config']['layout'], '%.4e' % d['value'], d['ms_per_step'], d['roofline']['frac'], {k: '%.3e' % d[k]['value'] for k in d if k.endswith('_layout')})"
done
timeout -k 10 600 python -u bench.py --workload ppo > $O/bench_ppo16.json 2> $O/bench_ppo16.err || { tail -20 $O/bench_ppo16.err; exit 1; }
grep '^{"metric' $O/bench_ppo16.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ppo', '%.4e' % d['value'], d['phases_s_per_iter'], d['eval'])"
