#!/bin/bash
# A/B of engine builds on one box: for each round r, for each library L in $LIBS (paths relative to the
# repo, "-" = the product libmgx.so), one bench line `python bench.py $BENCH_ARGS` with MGX_LIB_PATH=L.
# Lines -> gpurun_out/ab_<tag>.jsonl (tag = $TAG).  The library order rotates from round to round.  Optional first step: GPU tests ($PYTEST_ARGS, -k $PYTEST_K).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
if [ -n "$PYTEST_ARGS" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST_ARGS ${PYTEST_K:+-k "$PYTEST_K"} -m gpu -x -q --timeout 300 --timeout-method thread > $O/ab_tests.log 2>&1 || { tail -40 $O/ab_tests.log; exit 1; }
  tail -2 $O/ab_tests.log
fi
ARR=($LIBS)
NL=${#ARR[@]}
for r in $(seq 1 ${ROUNDS:-2}); do
  # the order rotates every round: the first run of a round measured slower in round 5's first A/B
  for i in $(seq 0 $((NL - 1))); do
    L=${ARR[$(( (i + r - 1) % NL ))]}
    if [ "$L" = "-" ]; then LP=$R/minigrid-rl_amd/mgx/libmgx.so; else LP=$R/$L; fi
    MGX_LIB_PATH=$LP timeout -k 10 ${BENCH_TIMEOUT:-240} python bench.py $BENCH_ARGS --cpu-seconds 0 --both-layouts 0 > $O/ab_line.json 2> $O/ab_err.log || { tail -20 $O/ab_err.log; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/ab_line.json')); r=d['roofline']; f=r.get('refill') or {}; print('$L', '%.3e'%d['value'], 'paid=%.3e'%d.get('value_resets_paid', 0), 'kern_us=%.2f'%r['avg_launch_us'], 'refill_us=%.1f'%f.get('avg_launch_us', 0), 'pipe_us=%.2f'%r['step_pipeline_us'], 'prod/cons=%s/%s'%(d['window']['episodes_produced'],d['window']['episodes_consumed']))" | tee -a $O/ab_${TAG:-x}.txt
    python -c "import json; d=json.load(open('$O/ab_line.json')); d['lib']='$L'; print(json.dumps(d))" >> $O/ab_${TAG:-x}.jsonl
  done
done
