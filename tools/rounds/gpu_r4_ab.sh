#!/bin/bash
# Round 4's A/B experiments (DESIGN §5 "Round-4 changes"), one per EXP, each the interleaved bench lines of
# tools/gpu_ab.sh over builds made by tools/build_diag_libs.sh ("-" = the product libmgx.so).
#   EXP=order   refill enqueued first (product) vs rollout first                        (rollfirst)
#   EXP=epw     32-env refill waves at config 4 (product auto) vs 64 / 16                (epw64, epw16)
#   EXP=vm      rollout barrier bound 8 (product) vs __syncthreads / 4 / 12 / 16         (vmsync, vm4, vm12, vm16)
#   EXP=defer   rows copied out a step late (product) vs at the end of the step          (nodefer)
#   EXP=step8   per-step kernel compiled for S = 8 (product) vs generic                  (nostep8)
#   EXP=refill  refill priority 3, MT top-ups, token copy                                (prio3, topup2, topup4, notok)
#   EXP=prio    refill issue priority 2 (product) vs 1 / 0                               (prio1, prio0)
#   EXP=pop     resets by ballot + popcount (product) vs per-pop LDS atomics              (popatomic)
#   EXP=gae     the driver's line with the GAE fused into the rollout launch (bench.py --gae-fused 1) vs not
set -e
R=$GRAFT_REPO_ROOT
L=minigrid-rl_amd/mgx
cd $R
K20="--steps 20 --warmup 5"
case "${EXP:?set EXP}" in
  order)  TAG=order20 ROUNDS=2 LIBS="- $L/libmgx_rollfirst.so" BENCH_ARGS="$K20" bash tools/gpu_ab.sh ;;
  epw)    TAG=epw_c4 ROUNDS=2 LIBS="- $L/libmgx_epw64.so $L/libmgx_epw16.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh ;;
  vm)     TAG=vm2048 ROUNDS=2 LIBS="- $L/libmgx_vmsync.so $L/libmgx_vm4.so $L/libmgx_vm12.so $L/libmgx_vm16.so" BENCH_ARGS="" bash tools/gpu_ab.sh
          TAG=vm20 ROUNDS=3 LIBS="- $L/libmgx_vmsync.so $L/libmgx_vm12.so" BENCH_ARGS="$K20" bash tools/gpu_ab.sh ;;
  defer)  TAG=df2048 ROUNDS=2 LIBS="- $L/libmgx_nodefer.so" BENCH_ARGS="" bash tools/gpu_ab.sh
          TAG=df20 ROUNDS=3 LIBS="- $L/libmgx_nodefer.so" BENCH_ARGS="$K20" bash tools/gpu_ab.sh
          TAG=dfc5 ROUNDS=1 LIBS="- $L/libmgx_nodefer.so" BENCH_ARGS="--config 5" bash tools/gpu_ab.sh ;;
  step8)  TAG=st8 ROUNDS=2 LIBS="- $L/libmgx_nostep8.so" BENCH_ARGS="--layout compact --steps 256 --warmup 256" bash tools/gpu_ab.sh ;;
  refill) TAG=rf20 ROUNDS=2 LIBS="- $L/libmgx_prio3.so $L/libmgx_topup2.so $L/libmgx_topup4.so $L/libmgx_notok.so" BENCH_ARGS="$K20" bash tools/gpu_ab.sh ;;
  prio)   TAG=pr20 ROUNDS=3 LIBS="- $L/libmgx_prio1.so $L/libmgx_prio0.so" BENCH_ARGS="$K20" bash tools/gpu_ab.sh
          TAG=pr2048 ROUNDS=1 LIBS="- $L/libmgx_prio1.so $L/libmgx_prio0.so" BENCH_ARGS="" bash tools/gpu_ab.sh
          TAG=prc4 ROUNDS=1 LIBS="- $L/libmgx_prio1.so $L/libmgx_prio0.so" BENCH_ARGS="--config 4" bash tools/gpu_ab.sh ;;
  pop)    TAG=pc2048 ROUNDS=2 LIBS="- $L/libmgx_popatomic.so" BENCH_ARGS="" bash tools/gpu_ab.sh ;;
  gae)    for r in 1 2 3; do for g in 1 0; do
            timeout -k 10 240 python bench.py $K20 --cpu-seconds 0 --both-layouts 0 --gae-fused $g > gpurun_out/gae_line.json 2> gpurun_out/gae_err.log || { tail -20 gpurun_out/gae_err.log; exit 1; }
            python -c "import json; d=json.load(open('gpurun_out/gae_line.json')); print('gae_fused=$g', '%.3e' % d['value'])"
          done; done ;;
  *) echo "unknown EXP=$EXP"; exit 1 ;;
esac
