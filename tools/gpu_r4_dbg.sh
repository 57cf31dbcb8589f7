#!/bin/bash
# Round 4 debug: the fused rollout at the bench shape, eager and graph-replayed, against the oracle (details of
# the first mismatch), with the product build and the generic (non-S=8) rollout kernel; then the fused-vs-
# per-step and fixture tests with both.
R=$GRAFT_REPO_ROOT
cd $R
for L in libmgx.so libmgx_nos8.so; do
  echo "== $L"
  MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/$L timeout -k 10 120 python -u tools/dbg_fused_graph.py 2>&1 | tail -8
done
for L in libmgx.so libmgx_nos8.so; do
  echo "== $L"
  MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/$L timeout -k 10 300 python -u -m pytest tests/test_rollout.py -k "equals_per_step or fixture" -m gpu -q --timeout 120 --timeout-method thread 2>&1 | tail -4
done
