#!/bin/bash
# Full GPU tests + smoke, then config 2 (compact, fused) and 5 (fused) bench lines.  -> gpurun_out/chk/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/chk
mkdir -p $O
bash tools/gpu_tests.sh
for CL in "2 compact" "2 fused" "5 fused" "4 fused"; do
  set -- $CL
  timeout -k 10 200 python bench.py --config $1 --layout $2 --both-layouts 0 --cpu-seconds 0 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -5 $O/b_$1_$2.err; exit 1; }
  python3 -c "
import json
for l in open('$O/b_$1_$2.json'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']
        print('cfg$1 $2', 'value %.4e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'kernel %.2f' % r['avg_launch_us'], 'frac %.3f' % r['frac'])"
done
