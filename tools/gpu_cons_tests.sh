#!/bin/bash
# GPU tests that exercise the refill's production rule and the reset fill.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/cons
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_rollout.py tests/test_compact.py -k "refill or ring or bench_shape or rollout or graph or max_consumption or mt_stream or fixture" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
