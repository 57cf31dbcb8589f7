#!/bin/bash
# Refill change check: engine parity, refill alone per epoch (default kernel and, for A/B, the
# all-problems kernel via MGX_REFILL_GENERIC=1), default bench line.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_compact.py tests/test_vec_env.py -x -q -m gpu --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/gpu_refill_cfgs.sh "4 5 0 multi" "4 None 0 multi"
MGX_REFILL_GENERIC=1 bash tools/gpu_refill_cfgs.sh "4 5 0 multi"
cd $R
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value %.4g  ms/step %.5f  step kernel %.2f us  pipeline %.2f us' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us']))"
