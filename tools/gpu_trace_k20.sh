set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tk20
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --both-layouts 0 --cpu-seconds 0 --host-wait spin > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
gzip -c $(find $O/t -name "*kernel_trace.csv" | head -1) > $O/kernel_trace.csv.gz
rm -rf $O/t
