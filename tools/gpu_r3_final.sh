#!/bin/bash
# Round-3 closing pass, part 1: GPU tests + smoke, the driver's default bench line and its 20-step
# shape, and the rocprofv3 kernel stats of the default command.  -> gpurun_out/final/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
bash tools/gpu_tests.sh
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep '^{"metric' $O/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['config']['layout'], '%.4e' % d['value'], d['ms_per_step'], d['roofline']['frac'], {k: '%.3e' % d[k]['value'] for k in d if k.endswith('_layout')})"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err || { tail -20 $O/bench_k20.err; exit 1; }
grep '^{"metric' $O/bench_k20.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k20', d['config']['layout'], '%.4e' % d['value'], d['ms_per_step'], d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -2
