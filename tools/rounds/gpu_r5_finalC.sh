#!/bin/bash
# Round 5 closing pass C: the TGL single-task model under the reference's test() protocol, the N > 1
# rehearsal (tools/gpu_dp_rehearsal.sh, gloo on one GPU), and a HIP runtime-API + kernel trace of the driver's
# command (where the 20-step region's time goes outside the kernels: graph launch, synchronize).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r5api
timeout -k 10 600 python -u tools/eval_protocol.py --ckpt eval_ck/tgl_ck.pt --columns TGL,ALL --fresh 0 --out gpurun_out/eval_tgl.json 2> gpurun_out/eval_tgl.err || { tail -20 gpurun_out/eval_tgl.err; exit 1; }
bash tools/gpu_dp_rehearsal.sh
O=$R/gpurun_out/r5api
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/t -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --both-layouts 0 --cpu-seconds 0 > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
for k in kernel_trace hip_api_trace; do gzip -c $(find $O/t -name "*${k}.csv" | head -1) > $O/$k.csv.gz; done
rm -rf $O/t
ls -la $O
