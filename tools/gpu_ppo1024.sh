#!/bin/bash
# BASELINE config 3 at the reference's horizon (algorithm/ppo.yaml:30 n_steps = 1024): 3 timed PPO
# iterations after 1 warm-up, 65,536 envs, minibatch 65,536, 4 epochs.  -> gpurun_out/ppo1024/
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/ppo1024
mkdir -p $O
timeout -k 10 900 python -u bench.py --workload ppo --horizon 1024 --steps 3 --warmup 1 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
cat $O/b.json
