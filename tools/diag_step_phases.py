"""Step-kernel phase clocks (libmgx_stamps.so, -DMGX_STAMPS=N): s_memtime cycles per workgroup per
compact step, by phase (counters 4..7; their meaning depends on N, see mgx_step_kernel's tail).
Env: N envs, a -DMGX_SERIAL_REFILL=1 build runs the refill on the caller's stream (step kernel alone)."""
import os, sys, json, time
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'minigrid-rl_amd')]
import torch
from mgx import MgxEngine
from mgx.compact import CompactBuffer
n = int(os.environ.get("N", 65536))
T = 256
e = MgxEngine(problem="multi", mission=5, size=8, n_envs=n, n_stack=4)
buf = CompactBuffer(e, T)
acts = torch.randint(0, 7, (T, n), device="cuda", dtype=torch.int32)
e.reset(); buf.observe(0)
for t in range(128): buf.step(t, acts[t])
torch.cuda.synchronize()
c0 = e.debug_counters()
t0 = time.perf_counter()
for t in range(128, 256): buf.step(t, acts[t])
torch.cuda.synchronize()
dt = time.perf_counter() - t0
c1 = e.debug_counters()
nblk = (n + 63) // 64
ph = [round((c1[k] - c0[k]) / nblk / 128) for k in range(4, 8)]
print(json.dumps(dict(n=n, lib=os.path.basename(os.environ.get("MGX_LIB_PATH", "libmgx.so")), us_per_step=round(dt / 128 * 1e6, 2),
                      clocks_per_block_step=ph, total=sum(ph))))
