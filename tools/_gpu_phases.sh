#!/bin/bash
# One gpurun call: phase clocks of the step kernel (stamps builds 1-3) at the env counts given.
set -e
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
for n in "$@"; do
  for v in 1 2 3; do
    N=$n MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_stamps$v.so timeout -k 10 120 python tools/_diag_phases.py > gpurun_out/ph_${v}_$n.txt 2>&1
    echo "n=$n stamps$v $(tail -1 gpurun_out/ph_${v}_$n.txt)"
  done
done
