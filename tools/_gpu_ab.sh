#!/bin/bash
# One gpurun call: GPU parity tests on the current build, then A/B bench of libmgx.so vs
# libmgx_prev.so (and the current build with the refill serialised).  Every GPU step has its
# own time limit; the first failing step ends the call.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
B="timeout -k 10 200 python bench.py --steps 2048 --warmup 128 --cpu-seconds 0"
$B > gpurun_out/ab_new.json 2>gpurun_out/ab_new.err
MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_prev.so $B > gpurun_out/ab_prev.json 2>gpurun_out/ab_prev.err
$B > gpurun_out/ab_new2.json 2>gpurun_out/ab_new2.err
MGX_SERIAL_REFILL=1 $B > gpurun_out/ab_new_serial.json 2>gpurun_out/ab_new_serial.err
for f in ab_new ab_prev ab_new2 ab_new_serial; do
  python3 -c "import json,sys; d=json.load(open('gpurun_out/$f.json')); r=d['roofline']; print('$f', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step', 'kernel', round(r['avg_launch_us'],2), 'us')"
done
