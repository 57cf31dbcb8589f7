#!/bin/bash
# Round 4: the randbelow_seq generator build (libmgx_seq.so) through the reference fixtures, then A/B
# against the product build on the driver's line, the default line and config 4; refill cost by
# elimination (wave clocks per attempt round, one wave alone and the full grid).
set -e
R=$GRAFT_REPO_ROOT
L=$R/minigrid-rl_amd/mgx
cd $R
MGX_LIB_PATH=$L/libmgx_seq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_rollout.py -k "fixture or oracle_1024 or full_size" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/seq_tests.log 2>&1 || { tail -30 gpurun_out/seq_tests.log; exit 1; }
tail -2 gpurun_out/seq_tests.log
TAG=seq20 ROUNDS=3 LIBS="- minigrid-rl_amd/mgx/libmgx_seq.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=seq2048 ROUNDS=2 LIBS="- minigrid-rl_amd/mgx/libmgx_seq.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=seqc4 ROUNDS=1 LIBS="- minigrid-rl_amd/mgx/libmgx_seq.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
for V in rclock skip1 skip2 skip4 skip8 skip32; do
  MGX_LIB_PATH=$L/libmgx_$V.so NS="64 65536" timeout -k 10 120 python tools/diag_refill_lanes.py | sed "s/^/$V /" | tee -a gpurun_out/elim.txt
done
