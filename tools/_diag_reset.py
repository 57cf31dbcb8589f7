import sys, time, json
import os; sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'minigrid-rl_amd')]
import torch
from mgx import MgxEngine
res = {}
for n in (1, 8, 64, 256, 4096, 65536):
    e = MgxEngine(problem="multi", mission=5, size=8, n_envs=n)
    e.reset(); torch.cuda.synchronize()
    ts = []
    for rep in range(5):
        ev0 = torch.cuda.Event(enable_timing=True); ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(); e.reset(); ev1.record(); torch.cuda.synchronize()
        ts.append(ev0.elapsed_time(ev1) * 1e3)
    res[n] = min(ts)
    del e
print(json.dumps({"reset_kernel_us_by_n": res}))
for size in (8, 16):
  for mission in (5, None):
    e = MgxEngine(problem="multi", mission=mission, size=size, n_envs=64)
    e.reset(); torch.cuda.synchronize()
    ts=[]
    for rep in range(5):
        ev0 = torch.cuda.Event(enable_timing=True); ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(); e.reset(); ev1.record(); torch.cuda.synchronize()
        ts.append(ev0.elapsed_time(ev1) * 1e3)
    print("size", size, "mission", mission, "64 envs reset us", min(ts))
