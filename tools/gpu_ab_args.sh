#!/bin/bash
# A/B of bench.py options on one box (the product library): for each round r, for each variant in $VARIANTS
# ('|'-separated extra bench arguments; "-" = none), one line `python bench.py $BENCH_ARGS <variant>`.
# The variant order rotates from round to round.  Lines -> gpurun_out/abx_<tag>.txt / .jsonl.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
IFS='|' read -ra ARR <<< "$VARIANTS"
NL=${#ARR[@]}
for r in $(seq 1 ${ROUNDS:-2}); do
  for i in $(seq 0 $((NL - 1))); do
    V=${ARR[$(( (i + r - 1) % NL ))]}
    [ "$V" = "-" ] && VA="" || VA="$V"
    timeout -k 10 ${BENCH_TIMEOUT:-240} python bench.py $BENCH_ARGS $VA --cpu-seconds 0 --both-layouts 0 > $O/abx_line.json 2> $O/abx_err.log || { tail -20 $O/abx_err.log; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/abx_line.json')); r=d['roofline']; f=r.get('refill') or {}; print('[$V]', '%.3e'%d['value'], 'ms/step=%.5f'%d['ms_per_step'], 'gpu_ms=%s'%d.get('gpu_time_ms'), 'kern_us=%.2f'%r['avg_launch_us'], 'refill_us=%.1f'%f.get('avg_launch_us', 0), 'pipe_us=%.2f'%r['step_pipeline_us'])" | tee -a $O/abx_${TAG:-x}.txt
    python -c "import json; d=json.load(open('$O/abx_line.json')); d['variant']='$V'; print(json.dumps(d))" >> $O/abx_${TAG:-x}.jsonl
  done
done
