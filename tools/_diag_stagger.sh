R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for st in 0 8000 16000 24000; do
  MGX_STAGGER=$st MGX_SERIAL_REFILL=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/stg$st -o run --output-format csv -- python3 $R/bench.py --steps 512 --warmup 64 --cpu-seconds 0 --probe 0 > $R/gpurun_out/stg$st.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/stg$st/run_kernel_stats.csv')):
    if 'step_kernel' in r['Name']: print('stagger $st', r['AverageNs'])
"
done
