"""Refill wave clocks per attempt round against the number of envs (lanes) a wave generates for
(libmgx_rclock.so, -DMGX_REFILL_CLOCK): n = 1 times one lane's path alone, n = 64 one full wave, n = 65,536
the production grid beside the steps.  Cycles per round at n = 1 vs n = 64 is the cost of divergence
(a wave runs the union of its lanes' paths)."""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "minigrid-rl_amd")]
import torch  # noqa: E402

from mgx import MgxEngine  # noqa: E402

for n in [int(v) for v in os.environ.get("NS", "1 8 64 65536").split()]:
    e = MgxEngine(problem="multi", mission=int(os.environ.get("MISSION", 5)), size=8, num_objects=4, n_envs=n,
                  terminal_mode="none", refill_every=32)
    acts = torch.randint(0, 7, (2048, n), device="cuda", dtype=torch.int32)
    e.reset()
    for i in range(512):
        e.step(acts[i])
    torch.cuda.synchronize()
    c0, s0 = e.debug_counters(), e.stats()
    for i in range(512, 2048):
        e.step(acts[i])
    torch.cuda.synchronize()
    c1, s1 = e.debug_counters(), e.stats()
    waves, rounds, clocks = c1[28] - c0[28], c1[27] - c0[27], c1[26] - c0[26]
    print(json.dumps(dict(n=n, waves=waves, rounds_per_wave_launch=rounds / waves,
                          clocks_per_round=clocks / max(rounds, 1),
                          clocks_per_wave_launch=clocks / waves, max_wave_clocks=c1[29],
                          rounds_histogram={r: c1[8 + r] - c0[8 + r] for r in range(16) if c1[8 + r] - c0[8 + r]},
                          episodes_per_env_launch=(s1["resets"] - s0["resets"]) / n /
                          max(1, s1["refill_launches"] - s0["refill_launches"]))), flush=True)
    e.close()
