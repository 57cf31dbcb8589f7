#!/bin/bash
# Round 6: the round-5 checkpoints (trained at 8x8) under the reference's test() protocol at 11x11 -- the
# size src/hydra_configs/testing.yaml and single.yaml default to -- each model on its own task column, the ALL model on
# ALL -> gpurun_out/eval11_<name>.json.  Each evaluation has its own time limit; each takes 4-6 min (one env, as the
# reference's test() steps it), so run them in two calls (SPECS="tgl_ck:TGL" ...).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in ${SPECS:-all_ck3:ALL gtg2_ck:GTG gto2_ck:GTO pkp2_ck:PKP tgl_ck:TGL}; do
  ck=${spec%%:*}; col=${spec##*:}
  timeout -k 10 420 python -u tools/eval_protocol.py --ckpt eval_ck/$ck.pt --size 11 --columns $col --fresh 0 --out gpurun_out/eval11_$ck.json 2> gpurun_out/eval11_$ck.err || { tail -20 gpurun_out/eval11_$ck.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/eval11_$ck.json')); c=d['columns']['$col']
print('$ck', '$col', c['overall'], 'seconds', c.get('seconds'))"
done
