#!/bin/bash
# Round 5: the driver's exact command, N times back to back on one box (the spread of its one-launch window)
# -> gpurun_out/r5rep/k20_<i>.json.  Then the evaluations of the resumed GTO / PKP models (test() protocol).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r5rep
mkdir -p $O
for i in $(seq 1 ${N:-5}); do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/k20_$i.json 2> $O/k20_$i.err || { tail -20 $O/k20_$i.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/k20_$i.json') if l.startswith('{\"metric')][0]); r=d['roofline']; print($i, '%.3e' % d['value'], 'kern %.2f frac %.3f' % (r['avg_launch_us'], r['frac']), 'refill', (r.get('refill') or {}).get('avg_launch_us'))"
done
for m in ${EVALS:-}; do
  CKPT=eval_ck/${m}_ck.pt NAME=$m COLS=$(echo $m | tr -d 0-9 | tr a-z A-Z),ALL NO_SQ=1 bash tools/gpu_r5_closeC.sh
done
