#!/bin/bash
# Round 4, final build: SQ counters of the rollout and refill kernels on the driver's line, rollout phase
# clocks (-DMGX_RSTAMPS) at configs 2 and 5 with the refill beside it and alone -> gpurun_out/.
set -e
R=$GRAFT_REPO_ROOT
L=$R/minigrid-rl_amd/mgx
cd $R
TAG=roll20 KERNEL=mgx_rollout_kernel bash tools/gpu_sq.sh
TAG=refill20 KERNEL=mgx_refill bash tools/gpu_sq.sh
for lib in rstamps rstamps_serial; do
  MGX_LIB_PATH=$L/libmgx_$lib.so timeout -k 10 120 python tools/diag_rollout_phases.py > gpurun_out/ph_${lib}_c2.json
  MGX_LIB_PATH=$L/libmgx_$lib.so N=131072 MISSION=1 S=16 timeout -k 10 180 python tools/diag_rollout_phases.py > gpurun_out/ph_${lib}_c5.json
done
cat gpurun_out/ph_*.json
