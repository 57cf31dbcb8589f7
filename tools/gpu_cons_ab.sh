#!/bin/bash
# A/B of the refill production cap: consumption-based (MGX_REFILL_MEAN=2, default) vs mean-deficit (1),
# both with mgx_reset filling every ring to D; configs 2/4/5 in the compact and fused layouts, then the
# driver-shaped 20-step window at three minimum warm-ups.  -> gpurun_out/cons/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/cons
mkdir -p $O
summ() {
  python3 -c "
import json,sys
for l in open('$1'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']; w=d['window']
        print('$2', 'value %.4e' % d['value'], 'ms/step %.2f us' % (d['ms_per_step']*1e3), 'kernel %.2f us' % r['avg_launch_us'],
              'frac %.3f' % r['frac'], 'prod/cons %.3f' % (w['episodes_produced']/max(1,w['episodes_consumed'])), 'warmup', d['warmup'])"
}
for CFG in 2 4 5; do
  for L in compact fused; do
    for M in 2 1; do
      MGX_REFILL_MEAN=$M timeout -k 10 200 python bench.py --config $CFG --layout $L --both-layouts 0 --cpu-seconds 0 > $O/b_${CFG}_${L}_$M.json 2> $O/b_${CFG}_${L}_$M.err || { tail -5 $O/b_${CFG}_${L}_$M.err; exit 1; }
      summ $O/b_${CFG}_${L}_$M.json "cfg$CFG $L mean=$M"
    done
  done
done
for MW in 0 256 2048; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --min-warmup $MW --both-layouts 0 --cpu-seconds 0 > $O/k20_$MW.json 2> $O/k20_$MW.err || { tail -5 $O/k20_$MW.err; exit 1; }
  summ $O/k20_$MW.json "k20 min-warmup $MW"
done
