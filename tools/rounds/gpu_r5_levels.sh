#!/bin/bash
# Round 5: the refill's ring-level feedback (MtCtl.round_extra) -- the rollout / parity tests, the refill rounds
# over 20,000 steps (tools/diag_refill_steady.py, -DMGX_REFILL_CLOCK build) and the driver's line after a short
# (transient) and a 300-ms (steady-state) warm-up.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
[ -n "$NO_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_rollout.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/levels_tests.log 2>&1 || { tail -40 gpurun_out/levels_tests.log; exit 1; }
[ -n "$NO_TESTS" ] || tail -2 gpurun_out/levels_tests.log
MGX_LIB_PATH=$R/ab_libs/libmgx_rclock_np.so WINDOWS=20 timeout -k 10 400 python -u tools/diag_refill_steady.py > gpurun_out/steady2.jsonl 2> gpurun_out/steady2.err || { tail -20 gpurun_out/steady2.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/steady2.jsonl'):
    d=json.loads(l)
    if d['window'] % 4 == 3: print(d['window'], round(d['rounds_per_wave'],3), round(d['queued_per_env'],1), max(int(k) for k in d['rounds_hist']))"
VARIANTS="--warmup-ms 300|--warmup-ms 0" BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" ROUNDS=2 TAG=lv bash tools/gpu_ab_args.sh
