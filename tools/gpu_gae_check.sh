#!/bin/bash
# GAE change check: GAE / PPO GPU tests, then the driver-shaped line twice and the default bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "gae or ppo or collector or compact" > $O/gae_tests.log 2>&1 || { tail -40 $O/gae_tests.log; exit 1; }
tail -2 $O/gae_tests.log
for rep in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --both-layouts 0 > $O/g20.json 2>$O/g20.err || { tail -5 $O/g20.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/g20.json')); r=d['roofline']
print('K20 value %.4g ms/step %.5f step %.2f pipeline %.2f gae %s' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us'], d['gae']['horizon']['avg_launch_us']))"
done
timeout -k 10 300 python bench.py --cpu-seconds 0 --both-layouts 0 > $O/gdef.json 2>$O/gdef.err || { tail -5 $O/gdef.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/gdef.json')); r=d['roofline']
print('default value %.4g ms/step %.5f step %.2f pipeline %.2f gae %s' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['step_pipeline_us'], d['gae']['horizon']['avg_launch_us']))"
