#!/bin/bash
# Refill cost by elimination (diagnostic builds libmgx_skip<k>.so, MGX_GEN_SKIP=k): refill alone per
# epoch with generator sections skipped.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MGX_SERIAL_REFILL=1
for k in ${SKIPS:-"" 1 2 4 8}; do
  L=$R/minigrid-rl_amd/mgx/libmgx${k:+_skip$k}.so
  MGX_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/skip$k -o run --output-format csv -- python3 $R/tools/refill_cost.py > $O/skip$k.log 2>&1 || { tail -20 $O/skip$k.log; exit 1; }
  python3 -c "
import csv
res = [l for l in open('$O/skip$k.log') if l.startswith('nobj')][0].split()
for r in csv.DictReader(open('$O/skip$k/run_kernel_stats.csv')):
    if 'refill' in r['Name']:
        per = (float(r['TotalDurationNs']) - float(r['MaxNs'])) / (int(r['Calls']) - 1) / 1e3
        print('skip=${k:-0}', 'refill per epoch %.1f us, resets per epoch per env %.2f' % (per, int(res[5]) / 65536 / 32))
"
done
