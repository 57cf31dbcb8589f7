#!/bin/bash
# One gpurun call: phase clocks of the step kernel (stamps builds), refill concurrent and serialised.
set -e
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
for v in stamps stamps2 stamps3; do
  for sr in 0 1; do
    MGX_SERIAL_REFILL=$sr MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_$v.so timeout -k 10 120 python tools/_diag_phases.py > gpurun_out/ph_${v}_$sr.txt 2>&1
    echo "$v serial=$sr $(tail -1 gpurun_out/ph_${v}_$sr.txt)"
  done
done
