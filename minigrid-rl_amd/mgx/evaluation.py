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
