#!/bin/bash
# bench.py's window shapes with the fused default: odd step counts (K = 7, 37, 100) and the 2-rank gloo
# rehearsal of the N > 1 path.  -> gpurun_out/shapes/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/shapes
mkdir -p $O
for K in 7 37 100; do
  timeout -k 10 200 python bench.py --steps $K --warmup 3 --cpu-seconds 0 --both-layouts 0 > $O/k$K.json 2> $O/k$K.err || { tail -10 $O/k$K.err; exit 1; }
  grep '^{"metric' $O/k$K.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('K=$K', d['config']['layout'], 'E', d['config']['refill_every'], 'H', d['config']['horizon'], '%.3e' % d['value'], d['config']['timed'])"
done
bash tools/gpu_dp_rehearsal.sh
cp $R/gpurun_out/dp/dp2.line.json $O/dp2.line.json
cp $R/gpurun_out/dp/dp4.line.json $O/dp4.line.json
