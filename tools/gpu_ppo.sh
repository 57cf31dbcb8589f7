#!/bin/bash
# Full PPO loop (BASELINE config 3) on the compact layout: horizon 16 and the reference horizon 1024.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 500 python bench.py --workload ppo --steps 2 --warmup 1 --horizon 16 > $O/ppo16.json 2>$O/ppo16.err || { tail -20 $O/ppo16.err; exit 1; }
cat $O/ppo16.json; tail -3 $O/ppo16.err
timeout -k 10 500 python bench.py --workload ppo --steps 1 --warmup 1 --horizon 1024 --batch-size 65536 > $O/ppo1024.json 2>$O/ppo1024.err || { tail -20 $O/ppo1024.err; exit 1; }
cat $O/ppo1024.json; tail -3 $O/ppo1024.err
