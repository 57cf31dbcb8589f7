#!/bin/bash
# Round 5: the GTO single-task model under the reference's test() protocol (GTO and ALL columns), then the SQ
# counters of the final build's rollout and refill on the driver's line (tools/gpu_sq.sh -> gpurun_out/sq_*.json).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/eval_protocol.py --ckpt ${CKPT:-gpurun_out/learn/gto_ck.pt} --columns ${COLS:-GTO,ALL} --fresh 0 --out gpurun_out/eval_${NAME:-gto}.json 2> gpurun_out/eval_${NAME:-gto}.err || { tail -20 gpurun_out/eval_${NAME:-gto}.err; exit 1; }
if [ -z "$NO_SQ" ]; then
  KERNEL=mgx_rollout_kernel TAG=r5b_roll bash tools/gpu_sq.sh
  KERNEL=mgx_refill TAG=r5b_refill bash tools/gpu_sq.sh
fi
