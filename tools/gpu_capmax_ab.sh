#!/bin/bash
# Refill production ceiling (MGX_REFILL_CAPMAX): attempt rounds per wave (histogram, slowest wave) at
# config 2, then the fused / compact pipelines of configs 2, 4 and 5 with and without the ceiling.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/capmax
mkdir -p $O
MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_rclock.so CAPMAX="${CAPMAXS:-0 5}" timeout -k 10 300 python -u tools/diag_refill_clock.py > $O/rounds.jsonl 2> $O/rounds.err || { tail -5 $O/rounds.err; exit 1; }
cat $O/rounds.jsonl
summ() {
  python3 -c "
import json
for l in open('$1'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']; w=d['window']
        print('$2', 'value %.4e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'kernel %.2f' % r['avg_launch_us'], 'prod/cons %.4f' % (w['episodes_produced']/w['episodes_consumed']))"
}
for rep in 1 2; do
for CL in ${CONFIGS:-"2 fused" "4 fused" "5 fused"}; do
  set -- $CL
  for M in ${BENCH_CAPMAXS:-0 5}; do
    MGX_REFILL_CAPMAX=$M timeout -k 10 200 python bench.py --config $1 --layout $2 --both-layouts 0 --cpu-seconds 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    summ $O/b.json "capmax=$M cfg$1 $2"
  done
done
done
