#!/bin/bash
# Kernel timeline of the fused rollout bench (config 2): rollout / slide / refill start and end per
# epoch, to see how much the refill overlaps the rollout launch.  -> gpurun_out/ft/ (rocpd database)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ft
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 $R/bench.py --config 2 --layout fused --both-layouts 0 --cpu-seconds 0 --steps 512 --probe 64 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
ls -la $O/prof
