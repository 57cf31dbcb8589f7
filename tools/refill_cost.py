"""Refill-kernel cost per episode for a config (serial refill: run a -DMGX_SERIAL_REFILL=1 build under
rocprofv3 --kernel-trace --stats; the refill launches of the timed epochs are the kernel's calls minus
the initial fill).  Prints resets consumed so the per-episode cost can be formed."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "minigrid-rl_amd")]
import torch  # noqa: E402

from mgx import MgxEngine  # noqa: E402

nobj = int(os.environ.get("NOBJ", 4))
mission = os.environ.get("MISSION", "5")
mission = None if mission == "None" else int(mission)
n = int(os.environ.get("N", 65536))
e = MgxEngine(problem=os.environ.get("PROBLEM", "multi"), mission=mission, size=int(os.environ.get("S", 8)),
              num_objects=nobj, n_envs=n, terminal_mode="none", refill_every=32,
              all_doors_open=os.environ.get("ADO", "0") == "1")
acts = torch.randint(0, 7, (1024, n), device="cuda", dtype=torch.int32)
e.reset()
for i in range(1024):
    e.step(acts[i])
torch.cuda.synchronize()
st = e.stats()
print("nobj", nobj, "mission", mission, "resets", st["resets"], "refill_launches", st["refill_launches"], "n", n)
