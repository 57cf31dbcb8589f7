#!/bin/bash
# Round 4: every GPU test with the product build (S = 8 per-step kernel), fused parity tests with the
# bounded-barrier and 16-env-refill builds, then A/B: per-step kernel S = 8 vs generic (compact layout),
# bounded rollout barriers (MGX_ROLL_VMKEEP) on the driver's / default line and config 5, 16-env refill
# waves at config 4.
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
bash tools/gpu_tests.sh
for V in vm6 epw16; do
  MGX_LIB_PATH=$R/$L/libmgx_$V.so timeout -k 10 600 python -u -m pytest tests/test_rollout.py tests/test_gpu_parity.py -k "rollout or fused or bench_shape or refill or ring" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/vm_$V.log 2>&1 || { tail -30 gpurun_out/vm_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/vm_$V.log)"
done
TAG=st8 ROUNDS=2 LIBS="- $L/libmgx_nostep8.so" BENCH_ARGS="--layout compact --steps 256 --warmup 256 --both-layouts 0" bash tools/gpu_ab.sh
TAG=vm20 ROUNDS=2 LIBS="- $L/libmgx_vm0.so $L/libmgx_vm6.so $L/libmgx_vm12.so" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_ab.sh
TAG=vm2048 ROUNDS=1 LIBS="- $L/libmgx_vm6.so $L/libmgx_vm12.so" BENCH_ARGS="" bash tools/gpu_ab.sh
TAG=vmc5 ROUNDS=1 LIBS="- $L/libmgx_vm6.so $L/libmgx_vm12.so" BENCH_ARGS="--config 5" bash tools/gpu_ab.sh
TAG=e16c4 ROUNDS=2 LIBS="- $L/libmgx_epw16.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh
