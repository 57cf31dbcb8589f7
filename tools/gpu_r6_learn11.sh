#!/bin/bash
# Round 6: the mixed-task ALL model trained at 11x11 -- the size the reference's training and
# test() configs default to (hydra_configs/single.yaml:24, testing.yaml:26) -- in segments of SECONDS_ (one gpurun call
# each; FROM = the previous segment's checkpoint, copied into the tree).  TOTAL is the whole run's env-steps (the lr
# schedule's length).  Then EVAL=1: the reference's test() protocol at 11x11 on the ALL column.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/learn11
mkdir -p $O
cd $R
NAME=${NAME:-all11}
if [ -z "$EVAL" ]; then
  RESUME=""
  [ -n "$FROM" ] && RESUME="--resume $FROM"
  timeout -k 10 $((SECONDS_ + 200)) python -u tools/ppo_learn.py --mission None --size 11 --timesteps ${TOTAL:-4.6e8} \
    --max-seconds $SECONDS_ --no-eval --save $O/${NAME}_ck.pt --progress $O/${NAME}_progress.jsonl $RESUME \
    > $O/${NAME}.json 2> $O/${NAME}.err || { tail -30 $O/${NAME}.err; exit 1; }
  cat $O/${NAME}.json
else
  for col in ${COLS:-ALL}; do
    timeout -k 10 420 python -u tools/eval_protocol.py --ckpt $FROM --size 11 --columns $col --fresh 0 \
      --out $O/eval11_${NAME}_$col.json 2> $O/eval11_${NAME}_$col.err || { tail -20 $O/eval11_${NAME}_$col.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/eval11_${NAME}_$col.json')); print('$col', d['columns']['$col']['overall'])"
  done
fi
