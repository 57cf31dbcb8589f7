#!/bin/bash
# Refill kernel alone (MGX_SERIAL_REFILL=1: on the step stream, not overlapped): kernel stats and
# one SQ counter pass; compact-layout bench workload.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MGX_SERIAL_REFILL=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ser -o run --output-format csv -- python3 $R/bench.py --steps 1024 --cpu-seconds 0 --graph 0 --both-layouts 0 > $O/prof_ser.log 2>&1 || { tail -20 $O/prof_ser.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof_ser/run_kernel_stats.csv')))[:4]:
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'], r['Percentage'])
"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY -d $O/pmc_ref -o run -- python3 $R/bench.py --steps 256 --warmup 64 --cpu-seconds 0 --graph 0 --probe 0 --both-layouts 0 > $O/pmc_ref.log 2>&1 || { tail -20 $O/pmc_ref.log; exit 1; }
python3 - <<PY
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open('$O/pmc_ref/run_counter_collection.csv')):
    k = 'refill' if 'refill' in r['Kernel_Name'] else ('step' if 'step_kernel' in r['Kernel_Name'] else None)
    if k is None: continue
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Dispatch_Id'])] += 1
for k, d in acc.items():
    nd = len({dk for (kk, dk) in n if kk == k})
    print(k, nd, {c: round(v / nd) for c, v in d.items()})
PY
