# step-kernel duration (serial refill, rocprof) for store-skipping diagnostic builds
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for L in libmgx.so libmgx_skip1.so libmgx_skip2.so libmgx_skip4.so libmgx_skip16.so libmgx_skip7.so; do
  MGX_SERIAL_REFILL=1 MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/skip_$L -o run --output-format csv -- python3 $R/bench.py --steps 512 --warmup 64 --cpu-seconds 0 --probe 0 > $R/gpurun_out/skip_$L.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/skip_$L/run_kernel_stats.csv')):
    if 'step_kernel' in r['Name']: print('$L', r['AverageNs'])
"
done
