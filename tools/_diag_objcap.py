"""Diagnose an engine-vs-oracle image mismatch: first differing env / step, with both views."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), d) for d in ("oracle", "minigrid-rl_amd", "tests")]
import numpy as np, torch
import oracle as O
from mgx import MgxEngine
from test_gpu_parity import EngineSource
problem, mission, size, nobj = sys.argv[1], None, int(sys.argv[2]), int(sys.argv[3])
n, T = 512, 16
ov = O.OracleVec(problem, mission, size, nobj, n, 42)
eng = MgxEngine(problem=problem, mission=mission, size=size, num_objects=nobj, n_envs=n, n_stack=4, terminal_mode="all", reward64=True)
r = ov.reset(); obs = eng.reset()
img, dr, mi = EngineSource.newest(obs)
print("reset image equal", np.array_equal(img, r["image"]))
acts = np.random.default_rng(7).integers(0, 7, (T, n))
for t in range(T):
    o = ov.step(acts[t]); obs = eng.step(torch.as_tensor(acts[t], device=eng.device))
    done = eng.done.cpu().numpy().astype(bool)
    img, dr, mi = EngineSource.newest(obs); timg, _, _ = EngineSource.newest(eng.terminal_obs)
    got = np.where(done[:, None, None, None], timg, img)
    bad = np.nonzero((got != o["image"]).any(axis=(1, 2, 3)))[0]
    if len(bad):
        e = bad[0]
        print("t", t, "n_bad", len(bad), "env", e, "action", acts[t][e], "done", done[e])
        print("engine types\n", got[e][..., 0].T); print("oracle types\n", o["image"][e][..., 0].T)
        a, b = eng.dump_state(), ov.dump()
        print("agent", a["agent"][e], b["agent"][e])
        print("grid eq", np.array_equal(a["grid"][e], b["grid"][e]))
        print("eng grid types\n", a["grid"][e][..., 0].T); print("orc grid types\n", b["grid"][e][..., 0].T)
        break
print("err", eng.stats() if hasattr(eng, "stats") else None)
