import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, 'minigrid-rl_amd'), os.path.join(R, 'oracle')]
import numpy as np, torch
import oracle as O
from mgx import MgxEngine
for S in (8, 11):
    n = 16
    e = MgxEngine(problem="multi", mission=None, size=S, n_envs=n)
    ov = O.OracleVec("multi", None, S, 4, n, 42)
    e.reset(); ov.reset()
    a = np.full(n, 6)
    o = ov.step(a.astype(np.int32))
    obs = e.step(torch.as_tensor(a, device="cuda"))
    img = obs["image"][:, -3:].permute(0, 2, 3, 1).cpu().numpy()
    d1, d2 = e.dump_state(), ov.dump()
    bad = [i for i in range(n) if not np.array_equal(img[i], o["r_image"][i])]
    print("S", S, "bad frames", bad, "grid eq", [np.array_equal(d1["grid"][i], d2["grid"][i]) for i in range(n)][:8],
          "agent eq", np.array_equal(d1["agent"], d2["agent"]))
    if bad:
        i = bad[0]
        print(" env", i, "agent", d1["agent"][i], d2["agent"][i])
        print(" got plane0\n", img[i][:, :, 0]); print(" want\n", o["r_image"][i][:, :, 0])
