"""Device-resident policy evaluation over an MgxEngine: SB3's `evaluate_policy`
and `EvalCallback` as the reference calls them (src/ppo.py:145-150, 161-165;
SURVEY.md §8(f) rank 3).

SB3 2.x semantics restated (not vendored by the reference -> parity unpinned at
that boundary, pinned here against the C oracle, tests/test_evaluation.py):

  evaluate_policy(model, env, n_eval_episodes=10, deterministic=True)
    * observations = env.reset()  (SB3 VecEnv.reset: seeded on the first call,
      later calls unseeded -- MgxEngine.reset follows the same rule)
    * env i must finish episode_count_targets[i] = (n_eval_episodes + i) // n_envs
      episodes; the loop runs while any env is below its target
    * a done env below its target contributes Monitor's info["episode"]:
      r = round(sum(episode rewards), 6), l = episode length; rewards are
      appended in step order, env index order within a step
    * returns (np.mean(rewards), np.std(rewards)) or, with
      return_episode_rewards=True, (rewards, lengths) lists.

Nothing leaves the GPU per step except one bool (is any env still below its
target), the loop condition SB3 evaluates every iteration.
"""
import os

import numpy as np
import torch


def _act_fn(model, deterministic):
    if hasattr(model, "predict"):
        return lambda obs: model.predict(obs, deterministic=deterministic)
    return model   # any callable obs -> actions [N] (int32/int64, on the engine's device)


@torch.no_grad()
def evaluate_policy(model, engine, n_eval_episodes=10, deterministic=True, return_episode_rewards=False,
                    reward_threshold=None):
    """SB3 `evaluate_policy` over `engine` (an MgxEngine).  `model` is an
    ActorCriticPolicy (its predict(obs, deterministic)) or a callable obs -> actions."""
    act = _act_fn(model, deterministic)
    n, dev = engine.n, engine.device
    idx = torch.arange(n, device=dev)
    targets = (n_eval_episodes + idx) // n            # episode_count_targets
    cap = max(1, (n_eval_episodes + n - 1) // n)
    counts = torch.zeros(n, dtype=torch.int64, device=dev)
    rew = torch.zeros((n, cap), dtype=torch.float64, device=dev)
    lens = torch.zeros((n, cap), dtype=torch.int64, device=dev)
    when = torch.full((n, cap), -1, dtype=torch.int64, device=dev)
    obs = engine.reset()
    t = 0
    while bool((counts < targets).any()):
        actions = act(obs)
        obs = engine.step(actions)
        rec = engine.done & (counts < targets)
        slot = counts.clamp(max=cap - 1)
        r = engine.reward64 if engine.reward64 is not None else engine.ep_return.double()
        # only the final step of an episode can pay (PlaygroundEnv.step), so the Monitor sum
        # of the episode's rewards is the last reward exactly
        rew[idx, slot] = torch.where(rec, r, rew[idx, slot])
        lens[idx, slot] = torch.where(rec, engine.ep_len.long(), lens[idx, slot])
        when[idx, slot] = torch.where(rec, torch.full_like(counts, t), when[idx, slot])
        counts += rec.long()
        t += 1
    w = when.cpu().numpy()
    sel = np.nonzero(w >= 0)
    order = np.lexsort((sel[0], w[sel]))                 # by step, then env index
    env_i, k = sel[0][order], sel[1][order]
    r_np, l_np = rew.cpu().numpy(), lens.cpu().numpy()
    episode_rewards = [round(float(r_np[i, j]), 6) for i, j in zip(env_i, k)]
    episode_lengths = [int(l_np[i, j]) for i, j in zip(env_i, k)]
    mean_reward = float(np.mean(episode_rewards)) if episode_rewards else float("nan")
    std_reward = float(np.std(episode_rewards)) if episode_rewards else float("nan")
    if reward_threshold is not None:
        assert mean_reward > reward_threshold, "Mean reward below threshold: %.2f < %.2f" % (
            mean_reward, reward_threshold)
    if return_episode_rewards:
        return episode_rewards, episode_lengths
    return mean_reward, std_reward


# minigrid OBJECT_TO_IDX['door'] (the type byte of mgx_dump_state's grid); PlaygroundEnv's multi layouts place
# 1 / 3 / 4 doors for 2 / 3 / 4 rooms (custom_env.py:617-649, 857-928, 1299-1389)
_DOOR = 4
_ROOMS_BY_DOORS = {1: 2, 3: 3, 4: 4}
TASKS = (("go to goal", "GTG"), ("go to", "GTO"), ("pick up", "PKP"), ("toggle", "TGL"), ("drop", "DRP"),
         ("move", "MOV"))


def task_of(mission_text):
    """README.md:54-65's task columns from a mission text ('go to goal' before 'go to')."""
    for prefix, name in TASKS:
        if mission_text.startswith(prefix):
            return name
    return mission_text


@torch.no_grad()
def evaluate_test_protocol(model, engine, n_episodes=1000, deterministic=True, progress=None):
    """The reference's benchmark protocol, `test()` (src/ppo.py:185-230; README.md:54-65 "Benchmark (1k ep)"):
    ONE env, make_vec_env(make_env, n_envs=1, seed=cfg.seed, vec_env_cls=DummyVecEnv) + VecTransposeImage +
    VecFrameStack, and per episode

        obs = vec_env.reset(); while not done: action = model.predict(obs, deterministic); obs, r, done = step

    with the episode's reward summed.  `engine` must be a fresh 1-env MgxEngine of the tested config (its first
    reset is make_vec_env's seeded one: PCG64(seed), CPython random = MT19937(seed) from PlaygroundEnv.__init__,
    custom_env.py:82).  The single MT19937 stream advances across the episodes, so missions and room counts vary
    from episode to episode, and every episode skips one generated episode: DummyVecEnv auto-resets the env when
    it is done (one episode generated), and test()'s next vec_env.reset() -- unseeded, both streams continuing --
    generates another (MgxEngine.reset after the first is that unseeded reset).
    Returns one dict per episode: reward (f64 sum), length, success (reward > 0: the mission was completed),
    mission_id, mission text, task (README's column), rooms (multi: 2 / 3 / 4 from the door count; else 0).
    `progress(k)`, if given, is called after every episode (k episodes done)."""
    from ._lib import mission_text
    if engine.n != 1:
        raise ValueError("the test() protocol steps ONE env (src/ppo.py:201-206: n_envs=1)")
    act = _act_fn(model, deterministic)
    out, texts = [], {}
    for _ in range(n_episodes):
        obs = engine.reset()
        st = engine.dump_state()
        mid = int(st["mission_id"][0])
        doors = int((st["grid"][0, :, :, 0] == _DOOR).sum())
        if mid not in texts:
            texts[mid] = mission_text(mid)
        total, length = 0.0, 0
        while True:
            obs = engine.step(act(obs))
            length += 1
            r = engine.reward64 if engine.reward64 is not None else engine.reward.double()
            total += float(r[0])
            if bool(engine.done[0]):
                break
        out.append(dict(reward=total, length=length, success=total > 0, mission_id=mid, mission=texts[mid],
                        task=task_of(texts[mid]), rooms=_ROOMS_BY_DOORS.get(doors, 0)))
        if progress is not None:
            progress(len(out))
    return out


def summarize_episodes(eps):
    """Success rate overall and per (task, rooms) cell, and the cell histogram, of evaluate_test_protocol's
    episodes."""
    import collections
    cells = collections.defaultdict(list)
    for e in eps:
        cells["%s/%d rooms" % (e["task"], e["rooms"])].append(e)
    per_task = collections.defaultdict(list)
    for e in eps:
        per_task[e["task"]].append(e)

    def stat(v):
        return {"episodes": len(v), "success_rate": float(np.mean([x["success"] for x in v])),
                "mean_reward": float(np.mean([x["reward"] for x in v])),
                "mean_length": float(np.mean([x["length"] for x in v]))}
    return {"overall": stat(eps), "per_task": {k: stat(v) for k, v in sorted(per_task.items())},
            "per_cell": {k: stat(v) for k, v in sorted(cells.items())},
            "cell_histogram": {k: len(v) for k, v in sorted(cells.items())},
            "distinct_missions": len({e["mission_id"] for e in eps})}


class EvalCallback:
    """SB3 EvalCallback(eval_env, best_model_save_path, eval_freq, n_eval_episodes,
    deterministic=True) for mgx.ppo.learn: every `eval_freq` vectorised steps of the
    training engine, evaluate on `eval_engine` and keep the best policy weights.

    The reference passes its training vec_env as eval_env (src/ppo.py:145), which makes
    SB3 reset the training envs mid-rollout; here evaluation runs on its own engine
    (SB3's documented usage) so the training rollout is not disturbed."""

    def __init__(self, eval_engine, best_model_save_path=None, eval_freq=10000, n_eval_episodes=5,
                 deterministic=True, log=None, callback_on_new_best=None):
        self.eval_engine = eval_engine
        self.callback_on_new_best = callback_on_new_best   # SB3: its on_step() False stops training
        self.best_model_save_path = best_model_save_path
        self.eval_freq = int(eval_freq)
        self.n_eval_episodes = int(n_eval_episodes)
        self.deterministic = deterministic
        self.log = log
        self.n_calls = 0
        self.best_mean_reward = -float("inf")
        self.last_mean_reward = -float("inf")
        self.evaluations = []      # (num_timesteps, mean_reward, std_reward, mean_ep_length)

    def on_step(self, policy, num_timesteps):
        self.n_calls += 1
        if self.eval_freq <= 0 or self.n_calls % self.eval_freq != 0:
            return True
        was_training = policy.training
        policy.train(False)
        rews, lens = evaluate_policy(policy, self.eval_engine, self.n_eval_episodes, self.deterministic,
                                     return_episode_rewards=True)
        policy.train(was_training)
        mean_r, std_r = float(np.mean(rews)), float(np.std(rews))
        self.last_mean_reward = mean_r
        self.evaluations.append((num_timesteps, mean_r, std_r, float(np.mean(lens))))
        if self.log:
            self.log(dict(eval_timesteps=num_timesteps, eval_mean_reward=mean_r, eval_std_reward=std_r,
                          eval_mean_ep_length=float(np.mean(lens))))
        if mean_r > self.best_mean_reward:
            self.best_mean_reward = mean_r
            if self.best_model_save_path is not None:
                os.makedirs(self.best_model_save_path, exist_ok=True)
                torch.save(policy.state_dict(), os.path.join(self.best_model_save_path, "best_model.pt"))
            if self.callback_on_new_best is not None:
                return bool(self.callback_on_new_best.on_step(self))
        return True


class StopTrainingOnRewardThreshold:
    """SB3 StopTrainingOnRewardThreshold, used as EvalCallback(callback_on_new_best=...):
    training stops once the best mean evaluation reward reaches `reward_threshold`."""

    def __init__(self, reward_threshold):
        self.reward_threshold = float(reward_threshold)

    def on_step(self, parent):
        return bool(parent.best_mean_reward < self.reward_threshold)
