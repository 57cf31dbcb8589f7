#!/bin/bash
# Step-kernel phase clocks (compact layout), alone (serial refill) and beside the refill, at two env counts.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
L=$R/minigrid-rl_amd/mgx
for n in 65536 16384; do
  for s in 1 0; do
    MGX_LIB_PATH=$L/libmgx_stamps1.so N=$n MGX_SERIAL_REFILL=$s timeout -k 10 120 python tools/diag_step_phases.py 2>$O/sp.err || { tail -20 $O/sp.err; exit 1; }
  done
done
MGX_LIB_PATH=$L/libmgx_stamps2.so N=65536 MGX_SERIAL_REFILL=1 timeout -k 10 120 python tools/diag_step_phases.py 2>$O/sp.err || { tail -20 $O/sp.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
for n in 65536 16384; do
  N=$n MGX_SERIAL_REFILL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/sp_$n -o run --output-format csv -- python3 $R/tools/diag_step_phases.py > $O/sp_$n.log 2>&1 || { tail -20 $O/sp_$n.log; exit 1; }
  python3 -c "
import csv
for r in list(csv.DictReader(open('$O/sp_$n/run_kernel_stats.csv')))[:3]:
    print('$n', r['Name'][:50], r['Calls'], r['AverageNs'], r['MinNs'])
"
done
