#!/bin/bash
# Round 5: record-layout ring (coalesced refill writes) -- parity first (fixtures through all three step paths,
# the bench shape, full-size oracle compares), then the benches, then the test() protocol evaluation.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5c
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_rollout.py tests/test_evaluation.py tests/test_compact.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -rf > $O/t.log 2>&1 || { tail -60 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_k20.json 2> $O/b_k20.err || { tail -30 $O/b_k20.err; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --both-layouts 0 > $O/b_default.json 2> $O/b_default.err || { tail -30 $O/b_default.err; exit 1; }
timeout -k 10 600 python -u tools/eval_protocol.py --ckpt eval_ck/all_ck3.pt --out $O/eval_all.json 2> $O/eval_all.err || { tail -30 $O/eval_all.err; exit 1; }
timeout -k 10 600 python -u tools/eval_protocol.py --random --fresh 0 --out $O/eval_random.json 2> $O/eval_random.err || { tail -30 $O/eval_random.err; exit 1; }
echo done
