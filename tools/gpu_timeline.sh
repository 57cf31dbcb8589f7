#!/bin/bash
# Per-epoch kernel timeline (tools/epoch_timeline.py) of the fused rollout bench under rocprofv3
# --kernel-trace, for each MGX_REFILL_CAPMAX in $CAPMAXS and config in $CONFIGS.  -> gpurun_out/tl/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in ${CONFIGS:-2}; do
for M in ${CAPMAXS:-0 5}; do
  rm -rf $O/c${C}m$M
  MGX_REFILL_CAPMAX=$M timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c${C}m$M -o run -- python3 $R/bench.py --config $C --layout fused --both-layouts 0 --cpu-seconds 0 --steps ${STEPS:-512} > $O/b_c${C}m$M.json 2> $O/b_c${C}m$M.err || { tail -20 $O/b_c${C}m$M.err; exit 1; }
  F=$(find $O/c${C}m$M -name '*kernel_trace.csv' | head -1)
  echo "config $C capmax $M: $(python3 $R/tools/epoch_timeline.py $F)"
  rm -f $F
done
done
