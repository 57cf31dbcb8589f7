#!/bin/bash
# Round-6 profile pass -> gpurun_out/r6prof/ (copied to profiles/r06_pmc/): for each (config, layout, steps)
# shape in $SHAPES (default: the driver's `--steps 20` line at config 2, the default 2048-step lines of configs
# 2, 4, 5, and the per-step compact line), the rocprofv3 --kernel-trace --stats summary of the bench command
# and the two HBM-byte PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs), summarised per launch by
# tools/pmc_summary.py for the step kernel and the refill.  manifest.json records the libmgx.so hash these
# were collected with: bench.py reports committed rocprof figures only for that build.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6prof
mkdir -p $O
python3 -c "import hashlib,json,subprocess; print(json.dumps({'lib_sha16': hashlib.sha256(open('$R/minigrid-rl_amd/mgx/libmgx.so','rb').read()).hexdigest()[:16], 'what': 'rocprofv3 summaries of bench.py commands (tools/gpu_r6_profiles.sh)'}))" > $O/manifest.json
cd /tmp && export TMPDIR=/tmp
declare -A N=( [2]=65536 [4]=32768 [5]=131072 ) S=( [2]=8 [4]=8 [5]=16 ) M=( [2]=5 [4]=None [5]=1 )
for shape in ${SHAPES:-2:fused:20 2:fused:2048 2:compact:20 4:fused:2048 5:fused:2048}; do
  IFS=: read cfg lay steps <<< "$shape"
  if [ $steps -eq 20 ]; then E=20; else E=64; fi
  tag=${cfg}_${lay}_e$E
  B="$R/bench.py --config $cfg --layout $lay --both-layouts 0 --cpu-seconds 0 --steps $steps --warmup 5"
  # the driver's own command, unchanged, for its line (config 2, fused, 20 steps)
  [ "$shape" = "2:fused:20" ] && B="$R/bench.py --gpus 1 --steps 20 --warmup 5"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s_$tag -o run --output-format csv -- python3 $B > $O/s_$tag.log 2>&1 || { tail -20 $O/s_$tag.log; exit 1; }
  cp $(find $O/s_$tag -name '*kernel_stats.csv' | head -1) $O/kernel_stats_$tag.csv
  gzip -c $(find $O/s_$tag -name '*kernel_trace.csv' | head -1) > $O/kernel_trace_$tag.csv.gz
  grep '^{"metric"' $O/s_$tag.log > $O/bench_$tag.json || true
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/f_$tag -o run -- python3 $B > $O/f_$tag.log 2>&1 || { tail -20 $O/f_$tag.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/w_$tag -o run -- python3 $B > $O/w_$tag.log 2>&1 || { tail -20 $O/w_$tag.log; exit 1; }
  if [ $lay = fused ]; then K=mgx_rollout_kernel; SPL=$E; else K="mgx_step_kernel<int, true"; SPL=1; fi
  python3 $R/tools/pmc_summary.py $(find $O/f_$tag -name '*counter_collection.csv' | head -1) $(find $O/w_$tag -name '*counter_collection.csv' | head -1) "$K" ${N[$cfg]} ${S[$cfg]} ${M[$cfg]} $SPL $O/pmc_$tag.json
  python3 $R/tools/pmc_summary.py $(find $O/f_$tag -name '*counter_collection.csv' | head -1) $(find $O/w_$tag -name '*counter_collection.csv' | head -1) "mgx_refill" ${N[$cfg]} ${S[$cfg]} ${M[$cfg]} $E $O/pmc_refill_$tag.json
  rm -rf $O/s_$tag $O/f_$tag $O/w_$tag
done
ls $O
