#!/bin/bash
# Round 5: kernel clock re-check, the driver's bench line, then the test() protocol evaluation of the round-4 ALL
# checkpoint (eval_ck/all_ck3.pt) and of a random policy.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_rollout.py::test_kernel_clock_records_every_launch \
  tests/test_evaluation.py -m gpu -x -v --timeout 300 --timeout-method thread -rf > $O/t.log 2>&1 || { tail -60 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/b_k20.json 2> $O/b_k20.err || { tail -30 $O/b_k20.err; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --both-layouts 0 > $O/b_default.json 2> $O/b_default.err || { tail -30 $O/b_default.err; exit 1; }
timeout -k 10 600 python -u tools/eval_protocol.py --ckpt eval_ck/all_ck3.pt --out $O/eval_all.json 2> $O/eval_all.err || { tail -30 $O/eval_all.err; exit 1; }
timeout -k 10 600 python -u tools/eval_protocol.py --random --fresh 0 --out $O/eval_random.json 2> $O/eval_random.err || { tail -30 $O/eval_random.err; exit 1; }
echo done
