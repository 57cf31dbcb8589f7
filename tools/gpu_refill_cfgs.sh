#!/bin/bash
# Refill kernel alone (MGX_SERIAL_REFILL=1) per 32-step epoch for configs given as "NOBJ MISSION ADO PROBLEM".
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MGX_SERIAL_REFILL=1
for cfg in "$@"; do
  set -- $cfg
  NOBJ=$1 MISSION=$2 ADO=$3 PROBLEM=$4 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/var -o run --output-format csv -- python3 $R/tools/refill_cost.py > $O/var.log 2>&1 || { tail -20 $O/var.log; exit 1; }
  python3 -c "
import csv
res = [l for l in open('$O/var.log') if l.startswith('nobj')][0].split()
for r in csv.DictReader(open('$O/var/run_kernel_stats.csv')):
    if 'refill' in r['Name']:
        per = (float(r['TotalDurationNs']) - float(r['MaxNs'])) / (int(r['Calls']) - 1) / 1e3
        print('$cfg', 'refill per epoch %.1f us, resets per epoch per env %.2f' % (per, int(res[5]) / 65536 / 32))
"
done
