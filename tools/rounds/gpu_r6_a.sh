#!/bin/bash
# Round 6, first call: is round 5's "steady-state drain" the bench's fixed action replay?
# tools/diag_ring_levels.py with the same action slice every replay (rounds 2-5) vs fresh actions (round 6), then the
# driver's command with the round-6 bench.py (fresh actions, timed region >= 20,480 steps after the reset).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6a
mkdir -p $O
cd $R
timeout -k 10 240 env ACTIONS=fixed WINDOWS=${WINDOWS:-20} python -u tools/diag_ring_levels.py > $O/levels_fixed.jsonl 2> $O/levels_fixed.err
timeout -k 10 240 env ACTIONS=fresh WINDOWS=${WINDOWS:-20} python -u tools/diag_ring_levels.py > $O/levels_fresh.jsonl 2> $O/levels_fresh.err
tail -2 $O/levels_fixed.jsonl
tail -2 $O/levels_fresh.jsonl
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds ${CPU_S:-2} > $O/bench_k20.json 2> $O/bench_k20.err
python -c "
import json; d=json.loads(open('$O/bench_k20.json').read().strip().splitlines()[-1])
print('value %.3e steady %.3e ratio %.3f pc %.3f steady_pc %.3f after %d frac %.3f refill %.1f' % (d['value'], d['steady_state']['value'], d['steady_state']['ratio_to_value'], d['window']['produced_over_consumed'], d['steady_state']['produced_over_consumed'], d['steps_after_reset'], d['roofline']['frac'], d['roofline']['refill']['avg_launch_us']))
print('compact %.3e sb3 %.3e' % (d['compact_layout']['value'], d['sb3_layout']['value']))"
