#!/bin/bash
# Quick A/B: the compact parity tests, then the default bench and the phase clocks at 65,536 envs.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-quick}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_compact.py -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value %.4e kernel %.2f us pipeline %.2f us frac %.3f sb3 %.4e' % (d['value'], r['avg_launch_us'], r['step_pipeline_us'], r['frac'], d['sb3_layout']['value']))"
L=$R/minigrid-rl_amd/mgx
for s in 1 0; do
  MGX_LIB_PATH=$L/libmgx_stamps1.so N=65536 MGX_SERIAL_REFILL=$s timeout -k 10 120 python tools/diag_step_phases.py >> $O/phases.jsonl 2>$O/sp.err || { tail -20 $O/sp.err; exit 1; }
done
cat $O/phases.jsonl
