#!/bin/bash
# Round 4 closing pass 2: every profile shape (gpu_r4_profiles.sh -> gpurun_out/r4prof/), then the driver's line
# again with the profiles in place (bench.py reads profiles/r04_pmc/ only when they are committed: this line
# shows the fields it would then carry).
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_r4_profiles.sh
mkdir -p profiles/r04_pmc && cp gpurun_out/r4prof/kernel_stats_*.csv gpurun_out/r4prof/pmc_*.json profiles/r04_pmc/
O=$R/gpurun_out/r4bench
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20b.json 2> $O/k20b.err || { tail -20 $O/k20b.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench_k20b.json') if l.startswith('{\"metric')][0]); r=d['roofline']
print('%.3e' % d['value'], 'avg_launch_us', r['avg_launch_us'], 'frac', r['frac'], 'traffic', r['traffic'], 'rocprof', r['rocprof'])"
