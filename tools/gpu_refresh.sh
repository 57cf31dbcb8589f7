#!/bin/bash
# One gpurun call that regenerates every committed measurement of the current build:
# default bench (BASELINE config 2: compact headline + SB3-stack line + CPU baseline) -> the
# driver-shaped line (--steps 20 --warmup 5) -> configs 4/5 -> rocprofv3 kernel stats of the
# default bench -> FETCH_SIZE / WRITE_SIZE PMC passes of both step-kernel variants.
# Every GPU step has its own time limit; the first failing step ends the call.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_k20.json 2>$O/bench_k20.err || { tail -20 $O/bench_k20.err; exit 1; }
timeout -k 10 300 python bench.py --config 4 --cpu-seconds 0 > $O/bench_cfg4.json 2>$O/bench_cfg4.err || { tail -20 $O/bench_cfg4.err; exit 1; }
timeout -k 10 300 python bench.py --config 5 --cpu-seconds 0 > $O/bench_cfg5.json 2>$O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
echo configs done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof/run_kernel_stats.csv')))[:6]:
    print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])
"
# refill kernel alone (serial on the caller's stream), BASELINE config 2 shape
MGX_SERIAL_REFILL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_serial -o run --output-format csv -- python3 $R/tools/refill_cost.py > $O/prof_serial.log 2>&1 || { tail -20 $O/prof_serial.log; exit 1; }
P="timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv"
for L in compact sb3; do
  $P --pmc FETCH_SIZE -d $O/pmcF_$L -o run -- python3 $R/bench.py --layout $L --steps 256 --warmup 64 --cpu-seconds 0 --probe 0 --graph 0 --both-layouts 0 > $O/pmcF_$L.log 2>&1 || { tail -20 $O/pmcF_$L.log; exit 1; }
  $P --pmc WRITE_SIZE -d $O/pmcW_$L -o run -- python3 $R/bench.py --layout $L --steps 256 --warmup 64 --cpu-seconds 0 --probe 0 --graph 0 --both-layouts 0 > $O/pmcW_$L.log 2>&1 || { tail -20 $O/pmcW_$L.log; exit 1; }
done
python3 $R/tools/pmc_summarize.py $O/pmcF_compact/run_counter_collection.csv $O/pmcW_compact/run_counter_collection.csv "mgx_step_kernel<int, true>" > $O/pmc_step_kernel_compact.json
python3 $R/tools/pmc_summarize.py $O/pmcF_sb3/run_counter_collection.csv $O/pmcW_sb3/run_counter_collection.csv "mgx_step_kernel<int, false>" > $O/pmc_step_kernel.json
cat $O/pmc_step_kernel_compact.json $O/pmc_step_kernel.json
