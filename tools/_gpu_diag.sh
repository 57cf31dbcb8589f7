#!/bin/bash
# Phase-stamp diagnostics of mgx_step_kernel (concurrent and serialised refill).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
for v in "" 2 3; do
  for ser in 0 1; do
    MGX_SERIAL_REFILL=$ser MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_stamps$v.so timeout -k 10 200 python tools/_diag_phases.py > $O/diag$v_$ser.log 2>&1 || { tail -5 $O/diag$v_$ser.log; exit 1; }
    echo "stamps$v serial=$ser $(tail -1 $O/diag$v_$ser.log)"
  done
done
