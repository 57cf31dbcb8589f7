#!/bin/bash
# SQ counters of the refill kernel alone (MGX_SERIAL_REFILL=1), one rocprofv3 pass per argument
# (each a space-separated counter list, <= 8 SQ counters); default: the two issue/stall passes.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MGX_SERIAL_REFILL=1
if [ $# -eq 0 ]; then
  set -- "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
         "SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_INST_CYCLES_VMEM"
fi
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv --pmc $C -d $O/rp$i -o run -- python3 $R/tools/refill_cost.py > $O/rp$i.log 2>&1 || { tail -20 $O/rp$i.log; exit 1; }
  python3 - <<PY
import csv, collections
acc = collections.defaultdict(float); ids = set()
for r in csv.DictReader(open('$O/rp$i/run_counter_collection.csv')):
    if 'refill' not in r['Kernel_Name']: continue
    ids.add(r['Dispatch_Id']); acc[r['Counter_Name']] += float(r['Counter_Value'])
nd = len(ids)
print({k: round(v / nd / 1024) for k, v in acc.items()}, 'per wave per launch,', nd, 'launches')
PY
done
