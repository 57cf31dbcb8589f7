#!/bin/bash
# Parity tests (engine only) + refill section clocks + default bench + refill-alone profile.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_vec_env.py -x -q --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_gstamps.so timeout -k 10 200 python tools/diag_gen.py > $O/diag_gen.json 2>$O/diag_gen.err || { tail -20 $O/diag_gen.err; exit 1; }
cat $O/diag_gen.json
timeout -k 10 300 python bench.py --steps 1024 --cpu-seconds 0 > $O/bench1k.json 2>$O/bench1k.err || { tail -20 $O/bench1k.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench1k.json')); r=d['roofline']
print('value %.4g  ms/step %.5f  step kernel %.2f us  pipeline %.2f us  gae %s' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us'], [round(g['avg_launch_us'],1) for g in d['gae'].values()]))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_q -o run --output-format csv -- python3 $R/bench.py --steps 1024 --cpu-seconds 0 > $O/prof_q.log 2>&1 || { tail -20 $O/prof_q.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof_q/run_kernel_stats.csv')))[:4]:
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'], r['Percentage'])
"
