"""Refill wave clocks (libmgx_rclock.so, -DMGX_REFILL_CLOCK): s_memtime cycles per wave per refill
launch and attempt rounds per wave (the busiest lane's) -- run under rocprofv3 --kernel-trace with a
build that also has -DMGX_SERIAL_REFILL=1 to put the clocks beside the launch durations (mgx_diag.h).

Env: MISSION (default 5), CAPS (space-separated production caps to sweep, default "0" = the engine's
default), REFILL_EVERY (default 32).  One JSON line per cap: rounds per wave-launch against the
episodes each env consumed per launch (their ratio is the production overhead)."""
import os, sys, json
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "minigrid-rl_amd")]
import torch
from mgx import MgxEngine
n = 65536
E = int(os.environ.get("REFILL_EVERY", 32))
acts = torch.randint(0, 7, (2048, n), device="cuda", dtype=torch.int32)
for cap in [int(c) for c in os.environ.get("CAPS", "0").split()]:
    e = MgxEngine(problem="multi", mission=int(os.environ.get("MISSION", 5)), size=8, num_objects=4, n_envs=n,
                  terminal_mode="none", refill_every=E, refill_cap=cap)
    e.reset()
    for i in range(1024):
        e.step(acts[i])
    torch.cuda.synchronize()
    c0 = e.debug_counters(); s0 = e.stats()
    for i in range(1024, 2048):
        e.step(acts[i])
    torch.cuda.synchronize()
    c1 = e.debug_counters(); s1 = e.stats()
    waves = c1[28] - c0[28]
    launches = s1["refill_launches"] - s0["refill_launches"]
    eps = (s1["resets"] - s0["resets"]) / n / launches
    rounds = (c1[27] - c0[27]) / waves
    hist = {r: c1[8 + r] - c0[8 + r] for r in range(16) if c1[8 + r] - c0[8 + r]}
    print(json.dumps(dict(cap=cap, refill_every=E, rounds_hist=hist,
                          slowest_wave_clocks=c1[29], queued_per_env=(s0["queued"] / n, s1["queued"] / n), launches=launches, clocks_per_wave_launch=(c1[26] - c0[26]) / waves,
                          rounds_per_wave_launch=rounds, episodes_per_env_launch=eps,
                          overhead=rounds / eps)), flush=True)
    e.close()
