#!/bin/bash
# Refill change check incl. S = 16 (NW = 4 path): engine parity, default bench, config 5 bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_compact.py tests/test_vec_env.py -x -q -m gpu --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for C in 2 5; do
  timeout -k 10 300 python bench.py --config $C --cpu-seconds 0 --both-layouts 0 > $O/bench_c$C.json 2>$O/bench_c$C.err || { tail -20 $O/bench_c$C.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_c$C.json')); r=d['roofline']
print('config $C value %.4g  ms/step %.5f  step kernel %.2f us  pipeline %.2f us' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us']))"
done
