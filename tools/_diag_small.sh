R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for n in 512 8192 32768 65536; do
  MGX_SERIAL_REFILL=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/sm$n -o run --output-format csv -- python3 $R/bench.py --n-envs $n --steps 512 --warmup 64 --cpu-seconds 0 --probe 0 > $R/gpurun_out/sm$n.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/sm$n/run_kernel_stats.csv')):
    if 'step_kernel' in r['Name'] or 'refill' in r['Name']: print('n=$n', r['Name'][:45], r['AverageNs'], r['MinNs'])
"
done
