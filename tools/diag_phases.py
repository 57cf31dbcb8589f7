import sys, time, json
import os; sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'minigrid-rl_amd')]
import torch
from mgx import MgxEngine
n = int(os.environ.get("N", 65536))
import sys as _s
e = MgxEngine(problem="multi", mission=5, size=8, n_envs=n)
acts = torch.randint(0, 7, (256, n), device="cuda", dtype=torch.int32)
torch.cuda.synchronize(); t=time.perf_counter()
e.reset(); torch.cuda.synchronize(); print("reset_kernel_s", time.perf_counter()-t)
for i in range(64): e.step(acts[i])
s0 = e.stats()
t=time.perf_counter()
for i in range(64, 256): e.step(acts[i])
torch.cuda.synchronize(); dt=time.perf_counter()-t
s1 = e.stats()
nblk = n // 64; steps = 192
ph = [(b-a)/nblk/steps for a,b in zip(s0['phase_clocks'], s1['phase_clocks'])]
print(json.dumps(dict(us_per_step=dt/steps*1e6, clocks_per_block_step=ph, resets_per_step=(s1['resets']-s0['resets'])/steps)))
