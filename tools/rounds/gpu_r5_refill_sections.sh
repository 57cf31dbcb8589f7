#!/bin/bash
# Round 5 ("find the 34 % wait"): SQ counters of the refill on the driver's line for the
# product build and the generator-section elimination builds (MGX_GEN_SKIP 1 keys + objects, 2 door positions,
# 4 goal + agent, 32 object choice draw; ab_libs/libmgx_gskip*.so) -> gpurun_out/sq_gs*.json.
set -e
R=$GRAFT_REPO_ROOT
cd $R
KERNEL=mgx_refill TAG=gs0 bash tools/gpu_sq.sh
for k in 1 2 4 32; do
  MGX_LIB_PATH=$R/ab_libs/libmgx_gskip$k.so KERNEL=mgx_refill TAG=gs$k bash tools/gpu_sq.sh
done
