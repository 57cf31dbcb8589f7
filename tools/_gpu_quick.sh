#!/bin/bash
# One gpurun call: GPU parity tests, then a bench line without the CPU leg.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/gpu_tests.log | tail -30; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
