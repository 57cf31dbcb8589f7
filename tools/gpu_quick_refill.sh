#!/bin/bash
# Generator change check: the parity tests that replay reference fixtures and oracle cases through every
# reset path, then wave clocks per attempt round and the config-2 pipeline.  -> gpurun_out/qr/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/qr
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_describe.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_rclock.so NS="1 64 65536" timeout -k 10 200 python tools/diag_refill_lanes.py
for CL in "2 compact" "2 fused"; do
  set -- $CL
  timeout -k 10 200 python bench.py --config $1 --layout $2 --both-layouts 0 --cpu-seconds 0 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -5 $O/b_$1_$2.err; exit 1; }
  python3 -c "
import json
for l in open('$O/b_$1_$2.json'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']
        print('cfg$1 $2', 'value %.4e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'kernel %.2f' % r['avg_launch_us'])"
done
