#!/bin/bash
# One gpurun call that regenerates every committed measurement of the current build:
# GPU parity tests -> smoke -> default bench (BASELINE config 2) -> configs 4/5 -> rocprofv3
# kernel stats of the default bench -> FETCH_SIZE / WRITE_SIZE PMC passes of the step kernel.
# Every GPU step has its own time limit; the first failing step ends the call.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --config 4 --cpu-seconds 0 > $O/bench_cfg4.json 2>$O/bench_cfg4.err || { tail -20 $O/bench_cfg4.err; exit 1; }
timeout -k 10 300 python bench.py --config 5 --cpu-seconds 0 > $O/bench_cfg5.json 2>$O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof/run_kernel_stats.csv')))[:6]:
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
"
P="timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv"
$P --pmc FETCH_SIZE -d $O/pmcF -o run -- python3 $R/bench.py --steps 256 --warmup 64 --cpu-seconds 0 --probe 0 --graph 0 > $O/pmcF.log 2>&1 || { tail -20 $O/pmcF.log; exit 1; }
$P --pmc WRITE_SIZE -d $O/pmcW -o run -- python3 $R/bench.py --steps 256 --warmup 64 --cpu-seconds 0 --probe 0 --graph 0 > $O/pmcW.log 2>&1 || { tail -20 $O/pmcW.log; exit 1; }
python3 $R/tools/_pmc_summarize.py $O/pmcF/run_counter_collection.csv $O/pmcW/run_counter_collection.csv > $O/pmc_step_kernel.json
cat $O/pmc_step_kernel.json
