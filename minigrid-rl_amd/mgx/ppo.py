"""Device-resident PPO rollout + training loop over the engine (BASELINE config 3).

Mirrors what the reference runs through SB3 at src/ppo.py:83-159:
`PPO(CustomPPOPolicy, vec_env, **config).learn(total_timesteps)` with the
config of hydra_configs/algorithm/ppo.yaml.  The SB3 pieces restated here
(stable_baselines3 2.x, not vendored by the reference -> parity unpinned, see
DESIGN.md §6):

  OnPolicyAlgorithm.collect_rollouts   -> RolloutCollector.collect
      per step: policy(obs) -> actions/values/log_probs; env.step; for every
      done env with TimeLimit.truncated, reward += gamma * V(terminal_obs);
      buffer.add(last_obs, actions, rewards, last_episode_starts, values,
      log_probs); last_episode_starts = dones.  At the end: V(new_obs) and
      compute_returns_and_advantage(last_values, dones)  (-> mgx_gae).
  RolloutBuffer.get(batch_size)        -> minibatches over a random permutation
      of the env-major flattened (env, t) index (swap_and_flatten).
  PPO.train                            -> Trainer.train: per-minibatch advantage
      normalisation (A - mean) / (std_unbiased + 1e-8), clipped surrogate,
      clipped value loss, entropy bonus, grad-norm clip, Adam step.
  linear_schedule (ppo.py:35-40)       -> max(progress_remaining * lr0, lr_final).

Nothing leaves the GPU: observations stay in the engine's in-place stacks and
are copied into a compact uint8 buffer (image, direction, mission tokens < 32:
exact), actions are sampled on device and fed back to mgx_step directly.

Multi-GPU: pass `group` (a torch.distributed process group,
RCCL on GPUs, gloo on CPU).  Each rank owns its own env shard.  Per optimiser
step the gradients are all-reduced (mean) in one flat bucket; per rollout one
all-reduce of the f64 advantage statistics (sum A, sum A^2, n) produced by
mgx_gae gives the global advantage mean/std (logged; used for normalisation
only with adv_norm="global").
"""
import math
from dataclasses import dataclass, field

import numpy as np
import torch

from .compact import CompactBuffer
from .engine import MgxEngine, gae, gae_dones


@dataclass
class PPOConfig:
    """hydra_configs/algorithm/ppo.yaml (model_kwargs) + single.yaml network.optim_eps."""
    n_envs: int = 16
    horizon: int = 1024                 # n_steps
    batch_size: int = 256
    n_epochs: int = 4
    gamma: float = 0.8108071290665859
    gae_lambda: float = 0.9452281119742252
    clip_range: float = 0.1
    clip_range_vf: float = 0.08341734780140342     # <= 0 -> None
    normalize_advantage: bool = True
    ent_coef: float = 0.045732238989694494
    vf_coef: float = 0.8177283657817492
    max_grad_norm: float = 0.5215982006116593
    initial_learning_rate: float = 3e-4
    final_learning_rate: float = 3e-6
    optim_eps: float = 1e-8
    n_frames_stack: int = 4
    n_eval_episodes: int = 100          # algorithm/ppo.yaml: evaluate_policy after learn (src/ppo.py:161-165)
    seed: int = 42
    adv_norm: str = "minibatch"         # "minibatch" (reference) | "global" (all-reduced stats)
    mission_cache: bool = True          # policy.py: GRU once per distinct mission stack
    layout: str = "compact"             # rollout storage: "compact" (mgx/compact.py) | "sb3" (stacked obs)
    env: dict = field(default_factory=lambda: dict(problem="multi", mission=2, size=8, num_objects=4))


def linear_schedule(initial_value, final_value):
    """src/ppo.py:35-40."""
    def func(progress_remaining):
        return max(progress_remaining * initial_value, final_value)
    return func


class RolloutBuffer:
    """DictRolloutBuffer with compact integer observation storage, [T, N, ...]."""

    def __init__(self, T, N, n_stack, device):
        self.T, self.N = T, N
        u8 = torch.uint8
        self.image = torch.zeros((T, N, 3 * n_stack, 7, 7), dtype=u8, device=device)
        self.direction = torch.zeros((T, N, 4 * n_stack), dtype=u8, device=device)
        self.mission = torch.zeros((T, N, 32 * n_stack), dtype=u8, device=device)
        f32 = dict(dtype=torch.float32, device=device)
        self.actions = torch.zeros((T, N), dtype=torch.int64, device=device)
        self.rewards = torch.zeros((T, N), **f32)
        self.episode_starts = torch.zeros((T, N), **f32)
        self.values = torch.zeros((T, N), **f32)
        self.log_probs = torch.zeros((T, N), **f32)
        self.advantages = None
        self.returns = None
        self.adv_stats = torch.zeros(3, dtype=torch.float64, device=device)

    def add(self, t, obs, actions, rewards, episode_starts, values, log_probs):
        self.image[t].copy_(obs["image"])
        self.direction[t].copy_(obs["direction"])
        self.mission[t].copy_(obs["mission"])
        self.actions[t].copy_(actions)
        self.rewards[t].copy_(rewards)
        self.episode_starts[t].copy_(episode_starts)
        self.values[t].copy_(values)
        self.log_probs[t].copy_(log_probs)

    def compute_returns_and_advantage(self, last_values, dones, gamma, gae_lambda):
        self.adv_stats.zero_()
        self.advantages, self.returns = gae(self.rewards, self.values, self.episode_starts, last_values, dones,
                                            gamma, gae_lambda, stats=self.adv_stats)

    def minibatches(self, batch_size, perm):
        """perm: permutation of the env-major flat index i = env * T + t (SB3 swap_and_flatten)."""
        T = self.T
        for s in range(0, perm.numel(), batch_size):
            idx = perm[s:s + batch_size]
            env, t = idx // T, idx % T
            obs = {"image": self.image[t, env], "direction": self.direction[t, env], "mission": self.mission[t, env]}
            yield (obs, self.actions[t, env], self.values[t, env], self.log_probs[t, env],
                   self.advantages[t, env], self.returns[t, env])


class RolloutCollector:
    """OnPolicyAlgorithm.collect_rollouts over an MgxEngine, entirely on device."""

    def __init__(self, engine, policy, cfg):
        self.engine, self.policy, self.cfg = engine, policy, cfg
        self.buffer = RolloutBuffer(cfg.horizon, engine.n, cfg.n_frames_stack, engine.device)
        self.last_episode_starts = torch.ones(engine.n, dtype=torch.float32, device=engine.device)
        self.last_dones = torch.zeros(engine.n, dtype=torch.bool, device=engine.device)
        self.num_timesteps = 0
        self.ep_returns, self.ep_lens = [], []
        self.stopped = False           # a callback's on_step returned False (SB3 early stop)

    def start(self):
        self.engine.reset()
        self.last_episode_starts.fill_(1.0)

    @torch.no_grad()
    def collect(self, callback=None):
        e, pol, cfg, buf = self.engine, self.policy, self.cfg, self.buffer
        pol.train(False)
        gamma32 = torch.tensor(cfg.gamma, dtype=torch.float32)
        ep_r, ep_l = [], []
        for t in range(cfg.horizon):
            obs = e.obs
            actions, values, log_probs = pol(obs)
            # the engine updates the stacks in place: store the pre-step obs first
            buf.image[t].copy_(obs["image"])
            buf.direction[t].copy_(obs["direction"])
            buf.mission[t].copy_(obs["mission"])
            e.step(actions)
            self.num_timesteps += e.n
            rewards = e.reward.clone()
            boot = (e.truncated & ~e.terminated).nonzero().flatten()
            if boot.numel():
                t_obs = {k: v.index_select(0, boot) for k, v in e.terminal_obs.items()}
                tv = pol.predict_values(t_obs)
                rewards.index_put_((boot,), rewards.index_select(0, boot) + gamma32.to(tv.device) * tv)
            buf.actions[t].copy_(actions)
            buf.rewards[t].copy_(rewards)
            buf.episode_starts[t].copy_(self.last_episode_starts)
            buf.values[t].copy_(values)
            buf.log_probs[t].copy_(log_probs)
            self.last_episode_starts.copy_(e.done.float())
            d = e.done
            ep_r.append(torch.where(d, e.ep_return, torch.nan))
            ep_l.append(torch.where(d, e.ep_len.float(), torch.nan))
            if callback is not None:       # BaseCallback.on_step, once per vectorised step
                if callback.on_step(pol, self.num_timesteps) is False:
                    # SB3 collect_rollouts: return False at once (no GAE); learn() stops
                    self.stopped = True
                    return None
                pol.train(False)
        self.last_dones.copy_(e.done)
        last_values = pol.predict_values(e.obs)
        buf.compute_returns_and_advantage(last_values, self.last_dones, cfg.gamma, cfg.gae_lambda)
        r, l = torch.stack(ep_r), torch.stack(ep_l)
        m = ~torch.isnan(r)
        self.ep_returns, self.ep_lens = r[m], l[m]
        return buf


class CompactRollout:
    """The rollout of CompactRolloutCollector: observations in the compact layout (one 148-B row
    + mission id per env-step, stacks rebuilt by mgx_gather), per-step policy outputs, GAE."""

    def __init__(self, engine, T):
        self.buf = CompactBuffer(engine, T, ring=True)      # history rows read in place (no per-rollout copy)
        self.T, self.N = T, engine.n
        dev = engine.device
        self.actions = torch.zeros((T, self.N), dtype=torch.int64, device=dev)
        self.values = torch.zeros((T, self.N), dtype=torch.float32, device=dev)
        self.log_probs = torch.zeros((T, self.N), dtype=torch.float32, device=dev)
        self.advantages = torch.zeros((T, self.N), dtype=torch.float32, device=dev)
        self.returns = torch.zeros((T, self.N), dtype=torch.float32, device=dev)
        self.adv_stats = torch.zeros(3, dtype=torch.float64, device=dev)

    @property
    def rewards(self):
        return self.buf.rewards

    def compute_returns_and_advantage(self, last_values, gamma, gae_lambda):
        """SB3 GAE over the compact dones (mgx_gae_dones: next_non_terminal(t) = 1 - done(t))."""
        self.adv_stats.zero_()
        gae_dones(self.buf.rewards, self.values, self.buf.dones, last_values, gamma, gae_lambda,
                  stats=self.adv_stats, out=(self.advantages, self.returns))

    def minibatches(self, batch_size, perm):
        """perm: permutation of the env-major flat index i = env * T + t (SB3 swap_and_flatten);
        observations gathered straight into the policy's f32 input."""
        T = self.T
        for s in range(0, perm.numel(), batch_size):
            idx = perm[s:s + batch_size]
            env, t = idx // T, idx % T
            obs = self.buf.gather(self.buf.index(t, env), f32=True)
            yield (obs, self.actions[t, env], self.values[t, env], self.log_probs[t, env],
                   self.advantages[t, env], self.returns[t, env])


class CompactRolloutCollector:
    """OnPolicyAlgorithm.collect_rollouts over an MgxEngine with the compact layout: per step one
    gather builds the policy's f32 input (VecFrameStack + preprocess_obs fused), one
    mgx_step_compact writes the next observation row, reward and done straight into the rollout
    buffer (no stack roll, no buffer copy)."""

    def __init__(self, engine, policy, cfg):
        self.engine, self.policy, self.cfg = engine, policy, cfg
        self.rollout = CompactRollout(engine, cfg.horizon)
        self.num_timesteps = 0
        self.ep_returns, self.ep_lens = [], []
        self.stopped = False
        self._n_rollouts = 0
        n, k, dev = engine.n, engine.n_stack, engine.device
        self._obs = dict(image=torch.empty((n, 3 * k, 7, 7), dtype=torch.float32, device=dev),
                         direction=torch.empty((n, 4 * k), dtype=torch.float32, device=dev),
                         mission=torch.empty((n, 32 * k), dtype=torch.uint8, device=dev))

    def start(self):
        self.engine.reset()
        self.rollout.buf.observe(0)
        self._n_rollouts = 0

    @torch.no_grad()
    def collect(self, callback=None):
        e, pol, cfg, ro = self.engine, self.policy, self.cfg, self.rollout
        buf = ro.buf
        if self._n_rollouts:
            buf.carry_over()
        self._n_rollouts += 1
        pol.train(False)
        gamma32 = torch.tensor(cfg.gamma, dtype=torch.float32)
        ep_r, ep_l = [], []
        for t in range(cfg.horizon):
            obs = buf.gather_step(t, f32=True, out=self._obs)
            actions, values, log_probs = pol(obs)
            buf.step(t, actions)
            self.num_timesteps += e.n
            boot = (buf.truncated[t].bool() & ~buf.terminated[t].bool()).nonzero().flatten()
            if boot.numel():
                tv = pol.predict_values(buf.gather_step(t, terminal=True, envs=boot))
                r = buf.rewards[t]
                r.index_put_((boot,), r.index_select(0, boot) + gamma32.to(tv.device) * tv)
            ro.actions[t].copy_(actions)
            ro.values[t].copy_(values)
            ro.log_probs[t].copy_(log_probs)
            d = buf.dones[t].bool()
            ep_r.append(torch.where(d, e.ep_return, torch.nan))
            ep_l.append(torch.where(d, e.ep_len.float(), torch.nan))
            if callback is not None:
                if callback.on_step(pol, self.num_timesteps) is False:
                    self.stopped = True
                    return None
                pol.train(False)
        last_values = pol.predict_values(buf.gather_step(cfg.horizon, f32=True, out=self._obs))
        ro.compute_returns_and_advantage(last_values, cfg.gamma, cfg.gae_lambda)
        r, l = torch.stack(ep_r), torch.stack(ep_l)
        m = ~torch.isnan(r)
        self.ep_returns, self.ep_lens = r[m], l[m]
        return ro


class Trainer:
    """PPO.train (SB3) + the learn() loop; optional data-parallel group."""

    def __init__(self, policy, cfg, group=None):
        self.policy, self.cfg, self.group = policy, cfg, group
        self.lr_schedule = linear_schedule(cfg.initial_learning_rate, cfg.final_learning_rate)
        self.gen = torch.Generator(device=next(policy.parameters()).device)
        self.gen.manual_seed(cfg.seed)
        self.world = torch.distributed.get_world_size(group) if group is not None else 1

    def global_adv_stats(self, buf):
        s = buf.adv_stats.clone()
        if self.group is not None:
            torch.distributed.all_reduce(s, group=self.group)       # the one RCCL exchange per rollout
        n = s[2].clamp_min(1)
        mean = s[0] / n
        var = (s[1] - n * mean * mean) / (n - 1).clamp_min(1)
        return mean, var.clamp_min(0).sqrt(), s

    def _allreduce_grads(self):
        if self.group is None:
            return
        grads = [p.grad for p in self.policy.parameters() if p.grad is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        torch.distributed.all_reduce(flat, group=self.group)
        flat /= self.world
        o = 0
        for g in grads:
            g.copy_(flat[o:o + g.numel()].view_as(g))
            o += g.numel()

    def train(self, buf, progress_remaining, perm_fn=None):
        cfg, pol = self.cfg, self.policy
        pol.train(True)
        lr = self.lr_schedule(progress_remaining)
        for g in pol.optimizer.param_groups:
            g["lr"] = lr
        clip = cfg.clip_range
        clip_vf = cfg.clip_range_vf if cfg.clip_range_vf > 0 else None
        g_mean = g_std = None
        if cfg.adv_norm == "global":
            g_mean, g_std, _ = self.global_adv_stats(buf)
        n = buf.T * buf.N
        stats = dict(pg=[], vf=[], ent=[], kl=[], clipfrac=[])
        for epoch in range(cfg.n_epochs):
            perm = perm_fn(n) if perm_fn else torch.randperm(n, generator=self.gen, device=self.gen.device)
            for obs, actions, old_v, old_lp, adv, ret in buf.minibatches(cfg.batch_size, perm):
                values, log_prob, entropy = pol.evaluate_actions(obs, actions)
                if cfg.normalize_advantage and adv.numel() > 1:
                    if g_mean is not None:
                        adv = (adv - g_mean.float()) / (g_std.float() + 1e-8)
                    else:
                        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
                ratio = torch.exp(log_prob - old_lp)
                pl1 = adv * ratio
                pl2 = adv * torch.clamp(ratio, 1 - clip, 1 + clip)
                policy_loss = -torch.min(pl1, pl2).mean()
                values_pred = values if clip_vf is None else old_v + torch.clamp(values - old_v, -clip_vf, clip_vf)
                value_loss = torch.nn.functional.mse_loss(ret, values_pred)
                entropy_loss = -torch.mean(entropy)
                loss = policy_loss + cfg.ent_coef * entropy_loss + cfg.vf_coef * value_loss
                with torch.no_grad():
                    log_ratio = log_prob - old_lp
                    stats["kl"].append(torch.mean((torch.exp(log_ratio) - 1) - log_ratio))
                    stats["clipfrac"].append(torch.mean((torch.abs(ratio - 1) > clip).float()))
                stats["pg"].append(policy_loss.detach())
                stats["vf"].append(value_loss.detach())
                stats["ent"].append(entropy_loss.detach())
                pol.optimizer.zero_grad()
                loss.backward()
                self._allreduce_grads()
                torch.nn.utils.clip_grad_norm_(pol.parameters(), cfg.max_grad_norm)
                pol.optimizer.step()
        return {k: float(torch.stack(v).mean()) for k, v in stats.items()} | {"lr": lr}


def make_collector(engine, policy, cfg):
    """The rollout collector of cfg.layout ("compact": CompactRolloutCollector, "sb3": RolloutCollector)."""
    if cfg.layout == "compact":
        return CompactRolloutCollector(engine, policy, cfg)
    if cfg.layout == "sb3":
        return RolloutCollector(engine, policy, cfg)
    raise ValueError("layout must be 'compact' or 'sb3'")


def learn(cfg, total_timesteps, device="cuda", group=None, rank=0, log=None, callback=None, evaluate=False,
          init=None):
    """PPO(...).learn(total_timesteps, callback=callback) for one rank's env shard; returns
    (policy, history, engine).  evaluate=True then runs evaluate_policy(model, vec_env,
    n_eval_episodes) on the training engine as src/ppo.py:161-165 does (history[-1]
    gets mean_reward / std_reward).  init: continue a run (SB3's PPO.load(...) then
    learn(..., reset_num_timesteps=False)): {"policy": state_dict, "optimizer": state_dict,
    "timesteps": int, "seed_offset": int} -- the envs restart from fresh episodes seeded
    cfg.seed + seed_offset; the learning-rate schedule continues from `timesteps`."""
    from .policy import ActorCriticPolicy
    init = init or {}
    torch.manual_seed(cfg.seed + rank + init.get("seed_offset", 0))
    eng = MgxEngine(n_envs=cfg.n_envs, seed=cfg.seed + init.get("seed_offset", 0), env_index_offset=rank * cfg.n_envs,
                    n_stack=cfg.n_frames_stack, terminal_mode="truncated", mission_dtype=torch.uint8,
                    device=device, reward64=True, **cfg.env)
    pol = ActorCriticPolicy(n_stack=cfg.n_frames_stack, optim_eps=cfg.optim_eps, lr=cfg.initial_learning_rate,
                            mission_cache=cfg.mission_cache).to(eng.device)
    if "policy" in init:
        pol.load_state_dict(init["policy"])
        pol.optimizer.load_state_dict(init["optimizer"])
    if group is not None:   # identical initial weights on every rank
        for p in pol.parameters():
            torch.distributed.broadcast(p.data, 0, group=group)
    col = make_collector(eng, pol, cfg)
    tr = Trainer(pol, cfg, group)
    col.start()
    hist = []
    world = tr.world
    col.num_timesteps = int(init.get("timesteps", 0)) // world
    while col.num_timesteps * world < total_timesteps:
        buf = col.collect(callback)
        if buf is None:                # callback asked to stop (SB3: continue_training False)
            break
        progress = 1.0 - float(col.num_timesteps * world) / float(total_timesteps)
        mean, std, s = tr.global_adv_stats(buf)
        st = tr.train(buf, progress)
        st.update(timesteps=col.num_timesteps * world, adv_mean=float(mean), adv_std=float(std),
                  ep_rew_mean=float(col.ep_returns.mean()) if col.ep_returns.numel() else math.nan,
                  ep_len_mean=float(col.ep_lens.mean()) if col.ep_lens.numel() else math.nan)
        hist.append(st)
        if log:
            log(st)
    if evaluate:
        from .evaluation import evaluate_policy
        mean_r, std_r = evaluate_policy(pol, eng, cfg.n_eval_episodes)
        if hist:
            hist[-1].update(mean_reward=mean_r, std_reward=std_r)
        if log:
            log(dict(mean_reward=mean_r, std_reward=std_r, n_eval_episodes=cfg.n_eval_episodes))
    eng.poll_error()
    return pol, hist, eng
