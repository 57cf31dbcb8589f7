"""Debug: the bench-shape fused graph (E = H = 20) at small N against the C oracle, printing the first
mismatching step's details (which envs, popped or not, where in the frame)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "minigrid-rl_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import oracle as O  # noqa: E402
from mgx import MgxEngine  # noqa: E402
from mgx.compact import CompactBuffer  # noqa: E402

n, E, W, reps = int(os.environ.get("N", 512)), 20, int(os.environ.get("W", 200)), 3
graph = os.environ.get("GRAPH", "1") == "1"
ov = O.OracleVec("multi", 5, 8, 4, n, 42)
eng = MgxEngine(problem="multi", mission=5, size=8, n_envs=n, n_stack=4, terminal_mode="truncated", refill_every=E)
dev = eng.device
buf = CompactBuffer(eng, E)
H = buf.H
rng = np.random.default_rng(77)
acts = rng.integers(0, 7, (W + reps * E, n)).astype(np.int32)
ov.reset(); eng.reset(); buf.observe(0)


def check(tag, t0):
    rows = buf.rows.cpu().numpy()
    for j in range(E):
        o = ov.step(acts[t0 + j])
        done = (o["terminated"] | o["truncated"]).astype(bool)
        img = rows[H + 1 + j][:, 1:].reshape(n, 3, 7, 7).transpose(0, 2, 3, 1)
        want = np.where(done[:, None, None, None], o["r_image"], o["image"])
        bad = np.nonzero((img != want).reshape(n, -1).any(1))[0]
        if bad.size:
            i = bad[0]
            print(tag, "step", t0 + j, "bad envs", bad.size, bad[:10].tolist(), "done", done[bad[:10]].tolist(),
                  "popped-frac", float(done[bad].mean()))
            print(" got  ch0", img[i, :, :, 0].tolist())
            print(" want ch0", want[i, :, :, 0].tolist())
            return False
    return True


ok = True
for t in range(0, W, E):
    if t:
        buf.carry_over()
    buf.rollout(0, torch.as_tensor(acts[t:t + E], device=dev))
    torch.cuda.synchronize()
    ok = check("eager", t) and ok
    if not ok:
        break
eng.join(); torch.cuda.synchronize()
print("eager warm-up ok" if ok else "eager warm-up FAILED")
if ok:
    static = torch.zeros((E, n), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        gr.capture_begin()
        buf.carry_over()
        buf.rollout(0, static)
        eng.join()
        gr.capture_end()
    torch.cuda.synchronize()
    for r in range(reps):
        static.copy_(torch.as_tensor(acts[W + r * E:W + (r + 1) * E], device=dev))
        gr.replay()
        torch.cuda.synchronize()
        if not check("graph r%d" % r, W + r * E):
            break
    else:
        print("graph replays ok")
eng.poll_error()
