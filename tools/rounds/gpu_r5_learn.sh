#!/bin/bash
# Round 5: a single-task PPO model (README.md:59-64 rows GTG / GTO / TGL were never trained before): one segment
# of tools/ppo_learn.py on MISSION, checkpoint into gpurun_out/ (merged back), no evaluation (tools/eval_protocol.py
# evaluates it under the reference's test() protocol in a later call).  Usage: MISSION=5 NAME=gtg SECONDS_=900
# [TOTAL=3.2e8: the lr schedule's total steps] [FROM=eval_ck/gtg_ck.pt: resume]
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/learn
mkdir -p $O
cd $R
RESUME=""
[ -n "$FROM" ] && RESUME="--resume $FROM"
timeout -k 10 $((SECONDS_ + 240)) python -u tools/ppo_learn.py --mission $MISSION --timesteps ${TOTAL:-2e9} --max-seconds $SECONDS_ \
  --no-eval --save $O/${NAME}_ck.pt --progress $O/${NAME}_progress.jsonl $RESUME > $O/${NAME}.json 2> $O/${NAME}.err \
  || { tail -30 $O/${NAME}.err; exit 1; }
cat $O/${NAME}.json
