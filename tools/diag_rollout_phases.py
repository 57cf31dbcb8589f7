"""Fused-rollout phase clocks (libmgx_rstamps.so, -DMGX_RSTAMPS): s_memtime cycles per workgroup per
step, wave 0's view -- step logic, wait at the post-logic barrier, terminal rows + render, rows out + the
end-of-step barrier.  Env: N envs (65,536), MISSION (5), S (8); a -DMGX_SERIAL_REFILL=1 build (with -DMGX_RSTAMPS=1) runs the refill on the
caller's stream (the rollout alone), else beside it."""
import json
import os
import sys
import time
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "minigrid-rl_amd")]
import torch  # noqa: E402
from mgx import MgxEngine  # noqa: E402
from mgx.compact import CompactBuffer  # noqa: E402

n = int(os.environ.get("N", 65536))
mission = os.environ.get("MISSION", "5")
e = MgxEngine(problem="multi", mission=None if mission == "None" else int(mission), size=int(os.environ.get("S", 8)),
              n_envs=n, n_stack=4)
E = e.refill_every
T = 16 * E
buf = CompactBuffer(e, T)
acts = torch.randint(0, 7, (T, n), device="cuda", dtype=torch.int32)
e.reset()
buf.observe(0)
for t in range(0, T // 2, E):
    buf.rollout(t, acts[t:t + E])
torch.cuda.synchronize()
c0 = e.debug_counters()
t0 = time.perf_counter()
for t in range(T // 2, T, E):
    buf.rollout(t, acts[t:t + E])
torch.cuda.synchronize()
dt = time.perf_counter() - t0
c1 = e.debug_counters()
nblk = (n + 63) // 64
steps = T // 2
ph = [round((c1[k] - c0[k]) / nblk / steps) for k in range(4, 8)]
print(json.dumps(dict(n=n, lib=os.path.basename(os.environ.get("MGX_LIB_PATH", "libmgx.so")), us_per_step=round(dt / steps * 1e6, 2),
                      clocks_per_block_step=dict(logic=ph[0], barrier_wait=ph[1], render=ph[2], rows_out_barrier=ph[3]),
                      total=sum(ph))))
