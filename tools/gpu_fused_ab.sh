#!/bin/bash
# A/B of the rollout layouts on config 2 (+ 4, 5): fused (one launch per refill epoch) vs per-step compact; rocprof stats of the fused bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-fused}
mkdir -p $O
for cfg in 2 4 5; do
  for lay in fused compact; do
    timeout -k 10 300 python bench.py --config $cfg --layout $lay --both-layouts 0 --cpu-seconds 0 > $O/b_${cfg}_$lay.json 2> $O/b_${cfg}_$lay.err || { tail -20 $O/b_${cfg}_$lay.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/b_${cfg}_$lay.json')); r=d['roofline']
print('cfg $cfg $lay value %.4e ms/step %.4f kernel/step %.2f us frac %.3f window %s' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['window']))"
  done
done
timeout -k 10 300 python bench.py --layout fused --both-layouts 0 --cpu-seconds 0 --steps 20 --warmup 5 > $O/b_k20_fused.json 2> $O/b_k20.err || { tail -20 $O/b_k20.err; exit 1; }
python -c "
import json; d=json.load(open('$O/b_k20_fused.json')); print('k20 fused value %.4e ms/step %.4f' % (d['value'], d['ms_per_step']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --layout fused --both-layouts 0 --cpu-seconds 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof/run_kernel_stats.csv')))[:6]: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])"
