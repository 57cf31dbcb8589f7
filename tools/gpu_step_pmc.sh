#!/bin/bash
# SQ counters of the compact step kernel (tools/diag_step_phases.py, MGX_SERIAL_REFILL=1 so the step
# kernel runs alone), one rocprofv3 pass per argument (<= 8 SQ counters each); per wave per launch.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MGX_SERIAL_REFILL=1
if [ $# -eq 0 ]; then
  set -- "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
fi
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv --pmc $C -d $O/sp$i -o run -- python3 $R/tools/diag_step_phases.py > $O/sp$i.log 2>&1 || { tail -20 $O/sp$i.log; exit 1; }
  python3 - <<PY
import csv, collections
acc = collections.defaultdict(float); ids = set()
for r in csv.DictReader(open('$O/sp$i/run_counter_collection.csv')):
    if 'step_kernel' not in r['Kernel_Name']: continue
    ids.add(r['Dispatch_Id']); acc[r['Counter_Name']] += float(r['Counter_Value'])
nd = len(ids)
print({k: round(v / nd / 4096, 1) for k, v in acc.items()}, 'per wave per launch,', nd, 'launches')
PY
done
