#!/bin/bash
# Rehearsal of bench.py's N > 1 path on ONE GPU with the gloo backend (RCCL refuses two ranks on one
# GPU; the driver's 8-GPU run uses RCCL): 2 and 4 ranks, each its own shard of 65,536 envs
# (env_index_offset = rank * n), barrier + max-over-ranks timing, the adv-stat all-reduce per horizon,
# ranks_seen from a collective.  Output lines -> gpurun_out/dp/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dp
mkdir -p $O
for np in 2 4; do
  MGX_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port $((29500 + np)) bench.py --gpus $np --steps ${STEPS:-20} --warmup 5 --cpu-seconds 0 > $O/dp$np.json 2>$O/dp$np.err || { tail -20 $O/dp$np.err; exit 1; }
  # gloo prints its connection banner on stdout (RCCL does not): keep the bench's JSON line only
  grep '^{"metric"' $O/dp$np.json > $O/dp$np.line.json
  python -c "
import json; d=json.load(open('$O/dp$np.line.json'))
s = d.get('steady_state') or {}
print('np $np n_gpus', d['n_gpus'], 'ranks_seen', d['ranks_seen'], 'backend', d['dist_backend'], 'value %.3e' % d['value'], 'steady %.3e' % s.get('value', 0), 'after', d.get('steps_after_reset'), d['config']['timed'])"
done
# the PPO workload (BASELINE config 3's loop) at 2 ranks: gradient + adv-stat all-reduces over gloo, each rank
# its own 16,384-env shard
MGX_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29510 bench.py --gpus 2 --workload ppo --n-envs 16384 --steps 2 --warmup 1 --eval-episodes 0 > $O/ppo2.json 2>$O/ppo2.err || { tail -20 $O/ppo2.err; exit 1; }
grep '^{"metric"' $O/ppo2.json > $O/ppo2.line.json
python -c "
import json; d=json.load(open('$O/ppo2.line.json'))
print('ppo np 2 n_gpus', d['n_gpus'], 'ranks_seen', d['ranks_seen'], d['dist_backend'], 'value %.3e' % d['value'], d['phases_s_per_iter'], d['config']['parallelism'])"
