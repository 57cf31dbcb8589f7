#!/bin/bash
# SB3-stack vs compact layout: rollout bench lines and PMC HBM traffic of each step kernel variant.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for L in sb3 compact; do
  timeout -k 10 300 python bench.py --steps 1024 --cpu-seconds 0 --layout $L > $O/bench_$L.json 2>$O/bench_$L.err || { tail -20 $O/bench_$L.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_$L.json')); r=d['roofline']
print('$L value %.4g  ms/step %.5f  step kernel %.2f us  pipeline %.2f us  frac %.3f' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us'], r['frac']))"
done
cd /tmp && export TMPDIR=/tmp
P="timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv"
$P --pmc FETCH_SIZE -d $O/pmcFc -o run -- python3 $R/bench.py --layout compact --steps 256 --warmup 64 --cpu-seconds 0 --probe 0 --graph 0 > $O/pmcFc.log 2>&1 || { tail -20 $O/pmcFc.log; exit 1; }
$P --pmc WRITE_SIZE -d $O/pmcWc -o run -- python3 $R/bench.py --layout compact --steps 256 --warmup 64 --cpu-seconds 0 --probe 0 --graph 0 > $O/pmcWc.log 2>&1 || { tail -20 $O/pmcWc.log; exit 1; }
python3 $R/tools/pmc_summarize.py $O/pmcFc/run_counter_collection.csv $O/pmcWc/run_counter_collection.csv "mgx_step_kernel<int, true>" > $O/pmc_step_kernel_compact.json
cat $O/pmc_step_kernel_compact.json
