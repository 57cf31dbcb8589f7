#!/bin/bash
# Round 6: kernel + HIP runtime trace of the driver's command with the region marked (bench.py --mark-region 1);
# tools/trace_window.py prints the region's timeline, its HIP API calls and the back-to-back replay period.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6trace${TAG:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/t -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --both-layouts 0 --cpu-seconds 0 --mark-region 1 ${BENCH_ARGS:-} > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
K=$(find $O/t -name "*kernel_trace.csv" | head -1)
A=$(find $O/t -name "*hip_api_trace.csv" | head -1)
python3 $R/tools/trace_window.py $K $A > $O/window.txt
gzip -c $K > $O/kernel_trace.csv.gz
rm -rf $O/t
cat $O/window.txt | head -80
tail -1 $O/t.log | cut -c1-300
