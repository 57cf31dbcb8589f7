#!/bin/bash
# SQ counters of kernel $KERNEL (substring) over one bench command ($BENCH_ARGS), one rocprofv3 --pmc pass
# per counter group (<= 8 SQ counters each, its own run and time limit) -> gpurun_out/sq_$TAG.json
# (tools/sq_summary.py).  MGX_LIB_PATH may select a build.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sq_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
P2="SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_VALU SQ_INSTS_SALU"
i=0
files=""
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $C -d $O/p$i -o run -- python3 $R/bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0} > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  files="$files $O/p$i/run_counter_collection.csv"
done
python3 $R/tools/sq_summary.py "${KERNEL:-mgx_rollout_kernel}" $R/gpurun_out/sq_${TAG:-x}.json $files
rm -rf $O
