#!/bin/bash
# Step-kernel phase clocks (compact layout), beside the refill and alone, at two env counts.  Builds
# (mgx_diag.h): libmgx_stamps1.so = EXTRA="-DMGX_STAMPS=1", libmgx_stamps1_serial.so = the same with
# -DMGX_SERIAL_REFILL=1 (the refill on the caller's stream: the step kernel alone).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
L=$R/minigrid-rl_amd/mgx
for n in 65536 16384; do
  for lib in libmgx_stamps1_serial.so libmgx_stamps1.so; do
    MGX_LIB_PATH=$L/$lib N=$n timeout -k 10 120 python tools/diag_step_phases.py 2>$O/sp.err || { tail -20 $O/sp.err; exit 1; }
  done
done
