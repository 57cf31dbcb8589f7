#!/bin/bash
# Step-kernel change check: engine parity (fixtures, reset paths, compact gather), phase clocks
# (compact, step kernel alone), default bench line.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_compact.py tests/test_vec_env.py -x -q -m gpu --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_stamps1.so N=65536 MGX_SERIAL_REFILL=1 timeout -k 10 120 python tools/diag_step_phases.py 2>$O/sp.err || { tail -20 $O/sp.err; exit 1; }
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value %.4g  ms/step %.5f  step kernel %.2f us  pipeline %.2f us  alone %s' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us'], r.get('alone_us')))"
