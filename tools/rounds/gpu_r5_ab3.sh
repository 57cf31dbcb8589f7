#!/bin/bash
# Round 5 A/B 3: the per-step compact kernel with wave 0's logic at issue priority 3 vs the product (the
# policy-in-the-loop line, 256 timed steps); then SQ counters of the fused rollout and the refill on the
# driver's line (product), and config 4's line.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TAG=r5cmp ROUNDS=3 LIBS="- ab_libs/libmgx_slprio3.so" BENCH_ARGS="--layout compact --steps 256 --warmup 256" bash tools/gpu_ab.sh
TAG=r5_roll KERNEL=mgx_rollout_kernel bash tools/gpu_sq.sh
TAG=r5_refill KERNEL=mgx_refill bash tools/gpu_sq.sh
timeout -k 10 300 python -u bench.py --config 4 --cpu-seconds 0 --both-layouts 0 > gpurun_out/r5_cfg4.json 2> gpurun_out/r5_cfg4.err || { tail -20 gpurun_out/r5_cfg4.err; exit 1; }
echo done
