#!/bin/bash
# Quick GPU round trip: GPU parity tests -> smoke -> default bench -> driver-shaped bench
# (--steps 20 --warmup 5).  Each GPU step has its own time limit; the first failure ends the call.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_k20.json 2>$O/bench_k20.err || { tail -20 $O/bench_k20.err; exit 1; }
cat $O/bench_k20.json
