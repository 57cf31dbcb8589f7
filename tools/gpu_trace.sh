#!/bin/bash
# rocprofv3 kernel trace + stats of one bench command ($BENCH_ARGS; default: the driver's line
# `--gpus 1 --steps 20 --warmup 5`), the epoch table of tools/trace_epochs.py, and the kernel stats ->
# gpurun_out/trace_$TAG/.  MGX_LIB_PATH may select a diagnostic build.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -o run -- python3 $R/bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
F=$(find $O/raw -name '*kernel_trace.csv' | head -1)
S=$(find $O/raw -name '*kernel_stats.csv' | head -1)
cp $S $O/kernel_stats.csv
python3 $R/tools/trace_epochs.py $F > $O/epochs.txt
tail -40 $O/epochs.txt
gzip -c $F > $O/kernel_trace.csv.gz
rm -rf $O/raw
