#!/bin/bash
# Round-3 measurement pass: default bench, driver-shaped bench, rocprofv3 kernel stats of the bench
# (compact layout only), step-kernel phase clocks (stamps build) at three env counts.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r3base}
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json | head -c 600; echo
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0 > $O/bench_k20.json 2> $O/bench_k20.err || { tail -20 $O/bench_k20.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --both-layouts 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R
L=$R/minigrid-rl_amd/mgx
for n in 65536 32768 16384; do
  for s in 1 0; do
    MGX_LIB_PATH=$L/libmgx_stamps1.so N=$n MGX_SERIAL_REFILL=$s timeout -k 10 120 python tools/diag_step_phases.py >> $O/phases.jsonl 2>$O/sp.err || { tail -20 $O/sp.err; exit 1; }
  done
done
cat $O/phases.jsonl
