#!/bin/bash
# Refill-kernel diagnostics: generator section clocks (-DMGX_GEN_STAMPS build), the refill
# alone (MGX_SERIAL_REFILL=1: on the step stream, not overlapped) under rocprofv3, a short bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_gstamps.so timeout -k 10 200 python tools/_diag_gen.py > $O/diag_gen.json 2>$O/diag_gen.err || { tail -20 $O/diag_gen.err; exit 1; }
cat $O/diag_gen.json
timeout -k 10 300 python bench.py --steps 512 --cpu-seconds 0 > $O/bench512.json 2>$O/bench512.err || { tail -20 $O/bench512.err; exit 1; }
cat $O/bench512.json
cd /tmp && export TMPDIR=/tmp
MGX_SERIAL_REFILL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_serial -o run --output-format csv -- python3 $R/bench.py --steps 512 --cpu-seconds 0 --graph 0 > $O/prof_serial.log 2>&1 || { tail -20 $O/prof_serial.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof_serial/run_kernel_stats.csv')))[:5]:
    print(r['Name'][:70], r['Calls'], r['AverageNs'], r['MinNs'], r['Percentage'])
"
