#!/bin/bash
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MGX_SERIAL_REFILL=1
for cfg in "4 5" "0 5" "2 5" "8 5" "4 None" "4 2"; do
  set -- $cfg
  NOBJ=$1 MISSION=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rc -o run --output-format csv -- python3 $R/tools/refill_cost.py > $O/rc.log 2>&1 || { tail -20 $O/rc.log; exit 1; }
  grep nobj $O/rc.log
  python3 -c "
import csv
for r in csv.DictReader(open('$O/rc/run_kernel_stats.csv')):
    if 'refill' in r['Name'] or 'step_kernel' in r['Name']: print('   ', r['Name'][40:75], r['Calls'], r['TotalDurationNs'], r['MaxNs'])
"
done
