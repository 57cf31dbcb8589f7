#!/bin/bash
# Refill cost by elimination: refill alone per epoch (serial refill) with generator sections skipped.
# Builds (mgx_diag.h): libmgx_serial.so = EXTRA="-DMGX_SERIAL_REFILL=1", libmgx_skip<k>.so =
# EXTRA="-DMGX_REFILL_CLOCK=1 -DMGX_SERIAL_REFILL=1 -DMGX_GEN_SKIP=<k>" (tools/build_diag_libs.sh).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in ${SKIPS:-"" 1 2 4 8}; do
  L=$R/minigrid-rl_amd/mgx/libmgx_serial.so
  [ -n "$k" ] && L=$R/minigrid-rl_amd/mgx/libmgx_skip$k.so
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
