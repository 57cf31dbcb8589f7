#!/bin/bash
# Round 5 closing pass C: the TGL single-task model under the reference's test() protocol, then the N > 1
# rehearsal (tools/gpu_dp_rehearsal.sh, gloo on one GPU).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/eval_protocol.py --ckpt eval_ck/tgl_ck.pt --columns TGL,ALL --fresh 0 --out gpurun_out/eval_tgl.json 2> gpurun_out/eval_tgl.err || { tail -20 gpurun_out/eval_tgl.err; exit 1; }
bash tools/gpu_dp_rehearsal.sh
