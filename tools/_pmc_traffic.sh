#!/bin/bash
# HBM traffic of mgx_step_kernel per launch (MI355X_MICROARCH.md HBM/rocprofv3 recipe):
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes, kernel-trace only (no sys/runtime
# trace), FETCH_SIZE doubled (gfx950 reports half of wide streaming reads).
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P="timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv"
$P --pmc FETCH_SIZE -d $R/gpurun_out/pmcF -o run -- python3 $R/bench.py --steps 256 --warmup 64 --cpu-seconds 0 --probe 0 --graph 0 > $R/gpurun_out/pmcF.log 2>&1
$P --pmc WRITE_SIZE -d $R/gpurun_out/pmcW -o run -- python3 $R/bench.py --steps 256 --warmup 64 --cpu-seconds 0 --probe 0 --graph 0 > $R/gpurun_out/pmcW.log 2>&1
python3 $R/tools/_pmc_summarize.py $R/gpurun_out/pmcF/run_counter_collection.csv $R/gpurun_out/pmcW/run_counter_collection.csv > $R/gpurun_out/pmc_step_kernel.json
cat $R/gpurun_out/pmc_step_kernel.json
