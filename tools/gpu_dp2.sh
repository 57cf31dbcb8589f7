#!/bin/bash
# New graph-replay parity test, then a 2-rank rehearsal of bench.py's N > 1 path on one GPU (gloo).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_compact.py -x -q -m gpu -k graph --timeout 200 --timeout-method thread -rf > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
MGX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 64 --warmup 5 --cpu-seconds 0 > $O/dp2.json 2>$O/dp2.err || { tail -20 $O/dp2.err; exit 1; }
grep metric $O/dp2.json | cut -c1-400
