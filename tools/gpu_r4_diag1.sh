set -e
R=$GRAFT_REPO_ROOT
L=$R/minigrid-rl_amd/mgx
MGX_LIB_PATH=$L/libmgx_serial.so TAG=serial20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0" bash tools/gpu_trace.sh > /dev/null
MGX_LIB_PATH=$L/libmgx_serial.so TAG=serial64 BENCH_ARGS="--gpus 1 --steps 256 --warmup 5 --cpu-seconds 0 --both-layouts 0" bash tools/gpu_trace.sh > /dev/null
for lib in rstamps rstamps_serial; do
  MGX_LIB_PATH=$L/libmgx_$lib.so timeout -k 10 120 python tools/diag_rollout_phases.py > gpurun_out/ph_${lib}_c2.json
  MGX_LIB_PATH=$L/libmgx_$lib.so N=131072 MISSION=1 S=16 timeout -k 10 180 python tools/diag_rollout_phases.py > gpurun_out/ph_${lib}_c5.json
done
cat gpurun_out/ph_*.json
TAG=roll20 KERNEL=mgx_rollout_kernel bash tools/gpu_sq.sh
TAG=refill20 KERNEL=mgx_refill bash tools/gpu_sq.sh
TAG=prod20 BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0" bash tools/gpu_trace.sh
