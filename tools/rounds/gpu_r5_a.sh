#!/bin/bash
# Round 5, first GPU call: the changed GPU tests first (ring rows, kernel clock, bench shape), then the whole
# -m gpu suite + smoke, then the driver's bench command and the default one.  Each step time-limited; the
# first failure ends the call.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_rollout.py::test_kernel_clock_records_every_launch tests/test_compact.py \
  "tests/test_gpu_parity.py::test_bench_shape_graph_matches_oracle" -m gpu -x -v --timeout 300 --timeout-method thread -rf \
  > $O/t_changed.log 2>&1 || { tail -60 $O/t_changed.log; exit 1; }
tail -2 $O/t_changed.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_k20.json 2> $O/b_k20.err || { tail -30 $O/b_k20.err; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > $O/t_all.log 2>&1 || { tail -60 $O/t_all.log; exit 1; }
tail -2 $O/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $O/b_default.json 2> $O/b_default.err || { tail -30 $O/b_default.err; exit 1; }
echo done
