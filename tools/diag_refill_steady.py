"""Refill attempt rounds per wave over time (libmgx_rclock*.so, -DMGX_REFILL_CLOCK): config 2 at the driver's
20-step refill epochs, the rounds histogram and the queued episodes per env in windows of 1,000 steps after the
reset -- does the epoch's refill cost stay where the first windows put it?"""
import os, sys, json
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "minigrid-rl_amd")]
import torch
from mgx import MgxEngine
n = 65536
E = int(os.environ.get("REFILL_EVERY", 20))
acts = torch.randint(0, 7, (1000, n), device="cuda", dtype=torch.int32)
e = MgxEngine(problem="multi", mission=int(os.environ.get("MISSION", 5)), size=8, num_objects=4, n_envs=n,
              terminal_mode="none", refill_every=E)
e.reset()
for w in range(int(os.environ.get("WINDOWS", 20))):
    torch.cuda.synchronize()
    c0 = e.debug_counters(); s0 = e.stats()
    for i in range(1000):
        e.step(acts[i])
    torch.cuda.synchronize()
    c1 = e.debug_counters(); s1 = e.stats()
    waves = c1[28] - c0[28]
    hist = {r: c1[8 + r] - c0[8 + r] for r in range(16) if c1[8 + r] - c0[8 + r]}
    print(json.dumps(dict(window=w, steps=(w + 1) * 1000, rounds_per_wave=(c1[27] - c0[27]) / max(waves, 1), rounds_hist=hist,
                          queued_per_env=s1["queued"] / n, resets_per_env_epoch=(s1["resets"] - s0["resets"]) / n / (1000 / E),
                          clocks_per_wave=(c1[26] - c0[26]) / max(waves, 1))), flush=True)
