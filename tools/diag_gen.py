"""Generator section clocks (libmgx_gstamps.so, -DMGX_GEN_STAMPS): wave clocks per section per epoch."""
import os, sys, json
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'minigrid-rl_amd')]
import torch
from mgx import MgxEngine
n = int(os.environ.get("N", 65536)); mission = os.environ.get("MISSION", "5")
mission = None if mission == "None" else int(mission)
e = MgxEngine(problem="multi", mission=mission, size=int(os.environ.get("S", 8)), n_envs=n,
              all_doors_open=os.environ.get("ADO", "0") == "1", num_objects=int(os.environ.get("NOBJ", 4)))
acts = torch.randint(0, 7, (256, n), device="cuda", dtype=torch.int32)
e.reset()
for i in range(64): e.step(acts[i])
torch.cuda.synchronize()
c0 = e.debug_counters(); s0 = e.stats()
for i in range(64, 256): e.step(acts[i])
torch.cuda.synchronize()
c1 = e.debug_counters(); s1 = e.stats()
names = {8: "copyout+loop", 9: "setup", 10: "mission+nr", 11: "walls+door draws", 12: "door pos",
         13: "goal+agent", 14: "keys+objects (last commit)", 15: "mission target", 16: "k+o: MT top-up",
         17: "k+o: task set-up", 18: "k+o: inner loop", 19: "k+o: commit+advance"}
waves = (n + 63) // 64; epochs = 192 // e.refill_every
res = {names[k]: round((c1[k] - c0[k]) / waves / epochs) for k in names}
res["total_per_wave_epoch"] = sum(res.values())
for k, nm in ((20, "room_task_iters"), (21, "randbelow_iters"), (24, "randbelow_calls"), (22, "free_cell_iters"), (23, "mt_refills"), (25, "mt_topups")):
    res[nm] = round((c1[k] - c0[k]) / waves / epochs, 1)
res["episodes_per_wave_epoch"] = (s1["resets"] - s0["resets"]) / waves / epochs
print(json.dumps(res))
