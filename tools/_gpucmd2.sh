#!/bin/bash
# One gpurun call: GPU parity tests -> phase stamps (N=512 serial, full) -> bench -> rocprof stats.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -rf > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
N=512 MGX_SERIAL_REFILL=1 MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_stamps3.so timeout -k 10 200 python tools/_diag_phases.py > gpurun_out/diag3_512.log 2>&1
tail -1 gpurun_out/diag3_512.log
MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_stamps3.so timeout -k 10 200 python tools/_diag_phases.py > gpurun_out/diag3.log 2>&1
tail -1 gpurun_out/diag3.log
timeout -k 10 300 python bench.py --steps 2048 --warmup 128 --cpu-seconds 0 > gpurun_out/bench.json 2>gpurun_out/bench.err
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 1024 --warmup 64 --cpu-seconds 0 > $R/gpurun_out/prof.log 2>&1
python3 -c "
import csv
for r in list(csv.DictReader(open('$R/gpurun_out/prof/run_kernel_stats.csv')))[:5]:
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
"
