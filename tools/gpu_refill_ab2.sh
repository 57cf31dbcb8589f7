#!/bin/bash
# Refill A/B: default build vs the 16-group MT window build (libmgx_wg16.so), configs 2 (compact, fused)
# and 5 (fused); then the wave-clock histogram and a serial-refill kernel trace (kernel duration vs
# the mean wave's time).  -> gpurun_out/ab2/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab2
mkdir -p $O
summ() {
  python3 -c "
import json
for l in open('$1'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']
        print('$2', 'value %.4e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'kernel %.2f' % r['avg_launch_us'])"
}
for rep in 1 2; do
for LIB in libmgx.so libmgx_wg16.so; do
  for CL in "2 compact" "2 fused" "5 fused"; do
    set -- $CL
    MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/$LIB timeout -k 10 200 python bench.py --config $1 --layout $2 --both-layouts 0 --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    summ $O/b.json "$LIB cfg$1 $2"
  done
done
done
MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_rclock.so NS="64 65536" timeout -k 10 200 python tools/diag_refill_lanes.py
cd /tmp && export TMPDIR=/tmp
MGX_SERIAL_REFILL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/refill_cost.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -h "refill\|Name" $(find $O/prof -name "*kernel_stats.csv") | head -5
