import sys
import os; sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'minigrid-rl_amd')]
import torch
from mgx import MgxEngine
n = 65536
e = MgxEngine(problem="multi", mission=5, size=8, n_envs=n)
acts = torch.randint(0, 7, (96, n), device="cuda", dtype=torch.int32)
e.reset()
for i in range(96): e.step(acts[i])
torch.cuda.synchronize()
print("done")
