#!/bin/bash
# Round 4 call B (diagnostics): kernel timelines with the refill serialised (each kernel alone; MT window 8 vs
# 16 groups), fused-rollout phase clocks (-DMGX_RSTAMPS) at configs 2 and 5, SQ counters of the rollout and
# refill kernels on the driver's line, refill cost by elimination (wave clocks, -DMGX_GEN_SKIP builds).
set -e
R=$GRAFT_REPO_ROOT
L=$R/minigrid-rl_amd/mgx
cd $R
for V in serial wg16_serial; do
  MGX_LIB_PATH=$L/libmgx_$V.so TAG=$V BENCH_ARGS="--gpus 1 --steps 256 --warmup 5 --cpu-seconds 0 --both-layouts 0" bash tools/gpu_trace.sh | tail -3
done
for lib in rstamps rstamps_serial; do
  MGX_LIB_PATH=$L/libmgx_$lib.so timeout -k 10 120 python tools/diag_rollout_phases.py > gpurun_out/ph_${lib}_c2.json
  MGX_LIB_PATH=$L/libmgx_$lib.so N=131072 MISSION=1 S=16 timeout -k 10 180 python tools/diag_rollout_phases.py > gpurun_out/ph_${lib}_c5.json
done
cat gpurun_out/ph_*.json
TAG=roll20 KERNEL=mgx_rollout_kernel bash tools/gpu_sq.sh
TAG=refill20 KERNEL=mgx_refill bash tools/gpu_sq.sh
for V in rclock skip1 skip2 skip4 skip8 skip32; do
  MGX_LIB_PATH=$L/libmgx_$V.so NS="64 65536" timeout -k 10 120 python tools/diag_refill_lanes.py | sed "s/^/$V /" | tee -a gpurun_out/elim.txt
done
