"""PPO loop timing at BASELINE config 3 scale (PKP 8x8, 65,536 envs): where the time goes."""
import json, os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'minigrid-rl_amd')]
import torch
from mgx import MgxEngine
from mgx.policy import ActorCriticPolicy
from mgx.ppo import PPOConfig, RolloutCollector, Trainer

n = int(os.environ.get("N", 65536)); T = int(os.environ.get("T", 16)); B = int(os.environ.get("B", 8192))
cache = bool(int(os.environ.get("CACHE", 0)))
cfg = PPOConfig(n_envs=n, horizon=T, batch_size=B, n_epochs=1, mission_cache=cache,
                env=dict(problem="multi", mission=2, size=8, num_objects=4))
eng = MgxEngine(n_envs=n, n_stack=4, terminal_mode="truncated", mission_dtype=torch.uint8, **cfg.env)
pol = ActorCriticPolicy(mission_cache=cache).cuda()
col = RolloutCollector(eng, pol, cfg); tr = Trainer(pol, cfg)
col.start()
res = {}
def timed(name, fn):
    torch.cuda.synchronize(); t0 = time.perf_counter(); r = fn(); torch.cuda.synchronize()
    res[name] = time.perf_counter() - t0; return r
with torch.no_grad():
    timed("policy_fwd_x4", lambda: [pol(eng.obs) for _ in range(4)])
timed("env_step_x64", lambda: [eng.step(torch.randint(0, 7, (n,), device="cuda")) for _ in range(64)])
buf = timed("collect", col.collect)
timed("collect2", col.collect)
timed("train", lambda: tr.train(buf, 1.0))
res.update(n=n, T=T, B=B, cache=cache, env_steps_per_s_collect=n * T / res["collect2"],
           env_steps_per_s_total=n * T / (res["collect2"] + res["train"]))
print(json.dumps(res))
