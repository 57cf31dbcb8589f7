#!/bin/bash
# Fused vs compact pipeline against envs per GPU (config 2 workload): co-residency of the rollout
# workgroups and the refill waves (LDS: 4 rollout workgroups + 4 refill waves per CU do not fit at 65,536).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fn
mkdir -p $O
for N in ${NS:-49152 65536}; do
  for L in fused compact; do
    timeout -k 10 200 python bench.py --n-envs $N --layout $L --both-layouts 0 --cpu-seconds 0 > $O/b_${N}_$L.json 2> $O/b_${N}_$L.err || { tail -5 $O/b_${N}_$L.err; exit 1; }
    python3 -c "
import json
for l in open('$O/b_${N}_$L.json'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']
        print('N=$N $L value %.4e us/step %.2f kernel %.2f' % (d['value'], d['ms_per_step']*1e3, r['avg_launch_us']))"
  done
done
