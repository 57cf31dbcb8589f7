#!/bin/bash
# Refill cost by elimination (round 3): wave clocks per attempt round at n = 1 and 64 (one wave alone)
# for the full generator and builds that skip one section (-DMGX_GEN_SKIP=k: 1 keys + objects, 2 door
# positions, 4 goal + agent, 8 walls + door draws, 16 MT top-up in the task loop, 32 object choice draw).
# Timing only: a skipped section changes the episodes.
set -e
R=$GRAFT_REPO_ROOT
for L in rclock skip1 skip2 skip4 skip8 skip16 skip32; do
  MGX_LIB_PATH=$R/minigrid-rl_amd/mgx/libmgx_$L.so NS="1 64" timeout -k 10 120 python tools/diag_refill_lanes.py | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$L', 'n', d['n'], 'clocks/round %.0f' % d['clocks_per_round'], 'rounds %.2f' % d['rounds_per_wave_launch'])"
done
