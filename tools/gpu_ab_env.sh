#!/bin/bash
# A/B of HIP runtime settings on one box (the product library, the driver's command): for each round r, for each
# variant in $VARIANTS ('|'-separated space-separated VAR=value lists; "-" = none), one line of
# `python bench.py $BENCH_ARGS` with those variables exported.  The variant order rotates from round to round.
# Lines -> gpurun_out/abe_<tag>.txt / .jsonl.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
IFS='|' read -ra ARR <<< "$VARIANTS"
NL=${#ARR[@]}
for r in $(seq 1 ${ROUNDS:-3}); do
  for i in $(seq 0 $((NL - 1))); do
    V=${ARR[$(( (i + r - 1) % NL ))]}
    ( [ "$V" != "-" ] && export $V
      timeout -k 10 ${BENCH_TIMEOUT:-240} python bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} --cpu-seconds 0 --both-layouts 0 \
        > $O/abe_line.json 2> $O/abe_err.log ) || { tail -20 $O/abe_err.log; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/abe_line.json')); r=d['roofline']; f=r.get('refill') or {}; s=d.get('steady_state') or {}; print('[$V]', '%.3e'%d['value'], 'steady %.3e'%s.get('value',0), 'gpu_ms=%s'%d.get('gpu_time_ms'), 'kern_us=%.2f'%r['avg_launch_us'], 'refill_us=%.1f'%f.get('avg_launch_us', 0))" | tee -a $O/abe_${TAG:-x}.txt
    python -c "import json; d=json.load(open('$O/abe_line.json')); d['variant']='$V'; print(json.dumps(d))" >> $O/abe_${TAG:-x}.jsonl
  done
done
