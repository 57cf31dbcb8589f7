import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, 'minigrid-rl_amd'), os.path.join(R, 'oracle')]
import numpy as np, torch
import oracle as O
from mgx import MgxEngine
n = 8
for ring in (0, -1):
    e = MgxEngine(problem="multi", mission=5, size=8, n_envs=n, ring_depth=ring)
    ov = O.OracleVec("multi", 5, 8, 4, n, 42)
    e.reset(); ov.reset()
    rng = np.random.default_rng(1)
    for t in range(20):
        a = rng.integers(0, 7, n)
        e.step(torch.as_tensor(a, device="cuda")); ov.step(a.astype(np.int32))
    a_, b_ = e.dump_state(), ov.dump()
    print("ring", ring, "before: mt", a_["mtwords"], b_["mtwords"], "pcg eq", np.array_equal(a_["pcg"], b_["pcg"]))
    e.reset(); ov.reset(None)
    a_, b_ = e.dump_state(), ov.dump()
    print(" after: mt", a_["mtwords"], b_["mtwords"])
    print(" agent", a_["agent"].tolist(), b_["agent"].tolist())
    print(" pcg eq", np.array_equal(a_["pcg"], b_["pcg"]), "grid eq", np.array_equal(a_["grid"], b_["grid"]))
