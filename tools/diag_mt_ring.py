"""Diagnostics for the device MT ring: GTG 8x8, N envs stepped against the C oracle; at the first
mismatch print the step, the env, both RNG cursors and the ring's generated length."""
import os, sys, json
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), p) for p in ("minigrid-rl_amd", "oracle")]
import numpy as np
import torch
import oracle as O
from mgx import MgxEngine
n = int(os.environ.get("N", 1024)); T = int(os.environ.get("T", 8000)); words = int(os.environ.get("WORDS", 1 << 16))
ring = int(os.environ.get("RING", 0))
ov = O.OracleVec("multi", 5, 8, 4, n, 42)
eng = MgxEngine(problem="multi", mission=5, size=8, n_envs=n, n_stack=4, terminal_mode="none", reward64=True,
                mt_table_words=words, ring_depth=ring)
ov.reset(); eng.reset()
acts = np.random.default_rng(31).integers(0, 7, (T, n)).astype(np.int32)
ad = torch.as_tensor(acts, device=eng.device)
for t in range(T):
    o = ov.step(acts[t]); obs = eng.step(ad[t])
    if t % 100 == 0 or t == T - 1:
        done = eng.done.cpu().numpy().astype(bool)
        img = obs["image"][:, -3:].permute(0, 2, 3, 1).cpu().numpy()
        want = np.where(done[:, None, None, None], o["r_image"], o["image"])
        bad = np.nonzero((img != want).reshape(n, -1).any(1) | (done != (o["terminated"] | o["truncated"]).astype(bool)))[0]
        st = eng.stats()
        a, b = eng.dump_state(), ov.dump()
        mw = b["mtwords"]
        line = dict(t=t, bad=len(bad), mt_generated=st["mt_generated"], max_cursor=st["max_mt_cursor"],
                    oracle_cursor_min=int(mw.min()), oracle_cursor_max=int(mw.max()))
        if len(bad):
            e = int(bad[0])
            line.update(env=e, eng_cursor=int(a["mtwords"][e]), oracle_cursor=int(mw[e]),
                        bad_cursor_envs=int((a["mtwords"] != mw).sum()))
        print(json.dumps(line), flush=True)
        if len(bad):
            break
try:
    eng.poll_error(); print("no device error")
except Exception as ex:
    print("device error:", ex)
