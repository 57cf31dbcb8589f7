#!/bin/bash
# Refill production overhead: attempt rounds per wave per epoch vs episodes consumed per env, for a sweep
# of production caps, with and without the mean-deficit cap (wave-clock build libmgx_rclock.so).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rounds
mkdir -p $O
export MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_rclock.so
for M in ${MEANS:-2 1 0}; do
  MGX_REFILL_MEAN=$M CAPS="${CAPS:-4 5 6 7}" timeout -k 10 300 python -u tools/diag_refill_clock.py > $O/mean$M.jsonl 2> $O/mean$M.err || { tail -5 $O/mean$M.err; exit 1; }
  echo "MGX_REFILL_MEAN=$M"; cat $O/mean$M.jsonl
done
