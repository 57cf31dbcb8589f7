#!/bin/bash
# Refill kernel alone (MGX_SERIAL_REFILL=1) for library variants given as arguments (default build first).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MGX_SERIAL_REFILL=1
for V in libmgx.so "$@"; do
  MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/var -o run --output-format csv -- python3 $R/tools/refill_cost.py > $O/var.log 2>&1 || { tail -20 $O/var.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$O/var/run_kernel_stats.csv')):
    if 'refill' in r['Name']: print('$V', 'refill per epoch (excl. initial fill) %.1f us' % ((float(r['TotalDurationNs']) - float(r['MaxNs'])) / (int(r['Calls']) - 1) / 1e3))
"
done
