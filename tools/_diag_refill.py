"""Refill-kernel cost per generated episode, single lane vs full waves (run under rocprofv3 --pmc)."""
import os, sys, json
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'minigrid-rl_amd')]
import torch
from mgx import MgxEngine
out = {}
for n in (1, 64, 65536):
    e = MgxEngine(problem="multi", mission=5, size=8, n_envs=n)
    acts = torch.randint(0, 7, (96, n), device="cuda", dtype=torch.int32)
    e.reset()
    s0 = e.stats()
    for i in range(96):
        e.step(acts[i])
    torch.cuda.synchronize()
    s1 = e.stats()
    out[n] = dict(resets=s1["resets"] - s0["resets"], steps=s1["steps"] - s0["steps"])
    del e
    torch.cuda.synchronize()
print(json.dumps(out))
