#!/bin/bash
# GPU tests (optionally a subset: PYTEST_ARGS, e.g. "tests/test_compact.py -k graph") + smoke.
# Each GPU step has its own time limit; the first failure ends the call.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
