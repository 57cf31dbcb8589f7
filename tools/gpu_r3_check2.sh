#!/bin/bash
# Round-3 check after the refill changes: GPU tests + smoke, the default bench (all layouts, CPU
# baseline), the driver-shaped 20-step line, configs 4 and 5.  -> gpurun_out/c2/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c2
mkdir -p $O
[ -n "$SKIP_TESTS" ] || bash tools/gpu_tests.sh
show() {
  python3 -c "
import json
for l in open('$1'):
    if l.startswith('{\"metric'):
        d=json.loads(l); r=d['roofline']; w=d['window']
        print('$2', d['config']['layout'], 'E', d['config']['refill_every'], 'value %.4e' % d['value'], 'us/step %.2f' % (d['ms_per_step']*1e3), 'kernel %.2f frac %.3f' % (r['avg_launch_us'], r['frac']), 'prod/cons %.4f' % (w['episodes_produced']/w['episodes_consumed']), {k: '%.3e' % d[k]['value'] for k in d if k.endswith('_layout')})"
}
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
show $O/bench.json default
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err || { tail -20 $O/bench_k20.err; exit 1; }
show $O/bench_k20.json k20
for C in 4 5; do
  timeout -k 10 300 python bench.py --config $C --cpu-seconds 0 > $O/bench_cfg$C.json 2> $O/bench_cfg$C.err || { tail -20 $O/bench_cfg$C.err; exit 1; }
  show $O/bench_cfg$C.json cfg$C
done
