#!/bin/bash
# SQ counters of the refill kernel alone (MGX_SERIAL_REFILL=1), one rocprofv3 pass per argument
# (each a space-separated counter list, <= 8 SQ counters); default: the two issue/stall passes.
# The first refill dispatch (mgx_reset's fill to D) is dropped.  -> gpurun_out/refill_sq.json
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export MGX_SERIAL_REFILL=1
if [ $# -eq 0 ]; then
  set -- "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
         "SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_VALU SQ_INSTS_SALU"
fi
i=0
rm -f $O/refill_sq.parts
for C in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $C -d $O/rp$i -o run -- python3 $R/tools/refill_cost.py > $O/rp$i.log 2>&1 || { tail -20 $O/rp$i.log; exit 1; }
  python3 - <<PY
import csv, collections, json
rows = [r for r in csv.DictReader(open('$O/rp$i/run_counter_collection.csv')) if 'refill' in r['Kernel_Name']]
ids = sorted({int(r['Dispatch_Id']) for r in rows})[1:]          # drop mgx_reset's fill
acc = collections.defaultdict(float)
for r in rows:
    if int(r['Dispatch_Id']) in ids: acc[r['Counter_Name']] += float(r['Counter_Value'])
waves = 65536 // 64
d = {k: v / len(ids) / waves for k, v in acc.items()}
open('$O/refill_sq.parts', 'a').write(json.dumps(d) + '\n')
print({k: round(v) for k, v in d.items()}, 'per wave per launch,', len(ids), 'launches')
PY
done
python3 - <<PY
import json
d = {}
for l in open('$O/refill_sq.parts'): d.update(json.loads(l))
cyc = d.get('SQ_WAVE_CYCLES')
out = {"kernel": "mgx_refill_multi_kernel<1> (config 2: GTG 8x8, 65,536 envs, 32-step epochs)",
       "method": "rocprofv3 --kernel-trace --pmc (one pass per counter group), MGX_SERIAL_REFILL=1 (refill alone), "
                 "tools/refill_cost.py; per wave per launch, mgx_reset's fill dropped",
       "per_wave_per_launch": d}
if cyc:
    out["fractions_of_wave_cycles"] = {k: d[k] / cyc for k in d if k.startswith(("SQ_WAIT", "SQ_ACTIVE"))}
json.dump(out, open('$O/refill_sq.json', 'w'), indent=1)
print(json.dumps(out.get("fractions_of_wave_cycles")))
PY
