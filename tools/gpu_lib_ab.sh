#!/bin/bash
# A/B of two builds (MGX_LIB_PATH): default bench line, alternating, 3 rounds.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
A=${LIB_A:-$R/minigrid-rl_amd/mgx/libmgx_prev.so}
B=${LIB_B:-$R/minigrid-rl_amd/mgx/libmgx.so}
for rep in 1 2 3; do for L in $A $B; do
  MGX_LIB_PATH=$L timeout -k 10 200 python bench.py --cpu-seconds 0 --both-layouts 0 ${BENCH_ARGS} > $O/ab.json 2>$O/ab.err || { tail -5 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/ab.json')); r=d['roofline']
print('$(basename $L) value %.4g step %.2f pipeline %.2f' % (d['value'], r['avg_launch_us'], r['step_pipeline_us']))"
done; done
