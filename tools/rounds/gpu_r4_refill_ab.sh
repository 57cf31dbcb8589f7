#!/bin/bash
# Round 4: which change moved the refill at the driver's 20-step epochs.  A/B of the product build against
# the generic-multi refill (nos8r), the refill-first launch order (reffirst) and round 3's library; then the
# refill alone (serial builds) per epoch: product, generic-multi refill, round 3 (its env knob).
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
TAG=rf20 ROUNDS=2 LIBS="- $L/libmgx_nos8r.so $L/libmgx_reffirst.so $L/libmgx_r3.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
BA="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0"
MGX_LIB_PATH=$R/$L/libmgx_serial.so TAG=ser_prod BENCH_ARGS="$BA" bash tools/gpu_trace.sh | sed -n 8,12p
MGX_LIB_PATH=$R/$L/libmgx_nos8r_serial.so TAG=ser_nos8r BENCH_ARGS="$BA" bash tools/gpu_trace.sh | sed -n 8,12p
MGX_SERIAL_REFILL=1 MGX_LIB_PATH=$R/$L/libmgx_r3.so TAG=ser_r3 BENCH_ARGS="$BA" bash tools/gpu_trace.sh | sed -n 8,12p
