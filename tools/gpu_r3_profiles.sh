#!/bin/bash
# Round-3 profile pass: for configs 2 / 4 / 5 and the compact per-step and fused layouts, the
# rocprofv3 kernel-trace stats and the two HBM-byte PMC passes of the bench command; refill SQ
# counters alone (config 2).  Outputs under gpurun_out/r3prof/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
declare -A N=( [2]=65536 [4]=32768 [5]=131072 ) S=( [2]=8 [4]=8 [5]=16 ) M=( [2]=5 [4]=None [5]=1 )
for cfg in ${CFGS:-2 4 5}; do
  for lay in ${LAYS:-compact fused}; do
    B="$R/bench.py --config $cfg --layout $lay --both-layouts 0 --cpu-seconds 0 --steps 256 --probe 64"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/s_${cfg}_$lay -o run --output-format csv -- python3 $B > $O/s_${cfg}_$lay.log 2>&1 || { tail -20 $O/s_${cfg}_$lay.log; exit 1; }
    timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/f_${cfg}_$lay -o run -- python3 $B > $O/f_${cfg}_$lay.log 2>&1 || { tail -20 $O/f_${cfg}_$lay.log; exit 1; }
    timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/w_${cfg}_$lay -o run -- python3 $B > $O/w_${cfg}_$lay.log 2>&1 || { tail -20 $O/w_${cfg}_$lay.log; exit 1; }
    if [ $lay = fused ]; then K=mgx_rollout_kernel; SPL=64; else K="mgx_step_kernel<int, true>"; SPL=1; fi
    python3 $R/tools/pmc_summary.py $O/f_${cfg}_$lay/run_counter_collection.csv $O/w_${cfg}_$lay/run_counter_collection.csv "$K" ${N[$cfg]} ${S[$cfg]} ${M[$cfg]} $SPL $O/pmc_${cfg}_$lay.json
    python3 $R/tools/pmc_summary.py $O/f_${cfg}_$lay/run_counter_collection.csv $O/w_${cfg}_$lay/run_counter_collection.csv "mgx_refill" ${N[$cfg]} ${S[$cfg]} ${M[$cfg]} 64 $O/pmc_refill_${cfg}_$lay.json
  done
done
