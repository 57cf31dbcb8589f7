#!/bin/bash
# Round-3 measurement refresh at HEAD: PMC + kernel stats per config / layout (gpu_r3_profiles.sh),
# copied into the box's profiles/r03_pmc so that the bench lines that follow price `traffic` with them;
# then the default bench, its 20-step shape, configs 4 and 5, config 3 (PPO, horizon 16), the rocprofv3
# kernel stats of the default command, the refill's SQ counters.  -> gpurun_out/rf/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rf
mkdir -p $O
[ -n "$SKIP_PROF" ] || { bash tools/gpu_r3_profiles.sh > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }; }
[ -n "$SKIP_PROF" ] || cp $R/gpurun_out/r3prof/pmc_*.json $R/profiles/r03_pmc/
SKIP_TESTS=1 bash tools/gpu_r3_check2.sh
cp $R/gpurun_out/c2/*.json $O/
timeout -k 10 600 python -u bench.py --workload ppo > $O/bench_ppo16.json 2> $O/bench_ppo16.err || { tail -20 $O/bench_ppo16.err; exit 1; }
grep '^{"metric' $O/bench_ppo16.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ppo', '%.4e' % d['value'], d['phases_s_per_iter'], d['eval'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py > $O/prof_default.log 2>&1 || { tail -20 $O/prof_default.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -2
cd $R && bash tools/gpu_refill_pmc.sh > $O/refill_sq.log 2>&1 || { tail -20 $O/refill_sq.log; exit 1; }
tail -3 $O/refill_sq.log
