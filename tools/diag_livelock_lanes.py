"""Round 5 steady-state question: do some envs' resets abandon hundreds of attempts in a row?  20,000
per-step launches at config 2 (20-step refill epochs); after every step, each env that started an episode reports
the abandoned attempts before it (MgxEngine.livelock, the header's live-lock count); the largest count per env is
kept.  Prints the histogram of the per-env maxima and the worst envs."""
import json, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "minigrid-rl_amd")]
import torch
from mgx import MgxEngine
n = 65536
e = MgxEngine(problem="multi", mission=5, size=8, num_objects=4, n_envs=n, terminal_mode="none", refill_every=20)
e.reset()
acts = torch.randint(0, 7, (1000, n), device="cuda", dtype=torch.int32)
mx = torch.zeros(n, dtype=torch.int32, device="cuda")
total = torch.zeros(n, dtype=torch.int64, device="cuda")
for w in range(int(os.environ.get("WINDOWS", 20))):
    for i in range(1000):
        e.step(acts[i])
        ll = torch.where(e.done, e.livelock, torch.zeros_like(e.livelock))
        mx = torch.maximum(mx, ll)
        total += ll.to(torch.int64)
    torch.cuda.synchronize()
    s = e.stats()
    print(json.dumps(dict(steps=(w + 1) * 1000, queued_per_env=s["queued"] / n, max_livelock=int(mx.max()),
                          envs_ge_10=int((mx >= 10).sum()), envs_ge_50=int((mx >= 50).sum()),
                          envs_ge_100=int((mx >= 100).sum()), abandoned_total=int(total.sum()))), flush=True)
v, i = torch.topk(mx, 10)
print(json.dumps(dict(worst=[(int(a), int(b)) for a, b in zip(i.tolist(), v.tolist())])))
