"""MgxVecEnv: the SB3 `VecEnv` face of the engine (host numpy in/out).

This is the drop-in for the object the reference builds at src/ppo.py:118-126:

    vec_env = make_vec_env(make_env, n_envs, seed, SubprocVecEnv, env_kwargs=...)
    vec_env = VecTransposeImage(vec_env)
    vec_env = VecFrameStack(vec_env, n_frames_stack, channels_order='first')

It keeps SB3's VecEnv contract (stable_baselines3.common.vec_env.base_vec_env):

  * reset() -> obs dict; step_async(actions) / step_wait() -> (obs, rewards
    f32[N], dones bool[N], infos list[N]); step(actions); seed(seed);
    num_envs, observation_space, action_space; close(); get_attr / set_attr /
    env_method / env_is_wrapped for the few attributes the PPO loop reads;
  * obs arrays are COPIES owned by the caller (_obs_from_buf);
  * infos[i] of a done env carries 'terminal_observation' (the stacked,
    transposed final obs, VecFrameStack.step_wait), 'TimeLimit.truncated'
    (truncated and not terminated, SubprocVecEnv worker) and Monitor's
    'episode' {'r', 'l', 't'}.

The PPO loop of this package does not go through here: it keeps everything on
device (MgxEngine).  This class is for callers that want the reference's host
API unchanged, at the cost of a device->host copy of the observation per step.
"""
import time

import numpy as np
import torch

from .engine import MgxEngine
from .spaces import make_spaces


class MgxVecEnv:
    """SB3-compatible vectorised PlaygroundEnv on one GPU.

    cfg_env mirrors `cfg.env` of the reference (single.yaml: problem, mission,
    size, num_objects, all_doors_open, see_through_walls, obstacles)."""

    metadata = {"render_modes": []}

    def __init__(self, n_envs, seed=42, n_frames_stack=4, problem="multi", mission=5, size=8, num_objects=4,
                 all_doors_open=False, see_through_walls=True, obstacles=False, device="cuda",
                 env_index_offset=0, **engine_kw):
        self.num_envs = int(n_envs)
        self.n_stack = int(n_frames_stack)
        self.engine = MgxEngine(problem=problem, mission=mission, size=size, num_objects=num_objects,
                                n_envs=n_envs, seed=seed, env_index_offset=env_index_offset, n_stack=self.n_stack,
                                all_doors_open=all_doors_open, see_through_walls=see_through_walls,
                                obstacles=obstacles, terminal_mode="all", reward64=True, device=device,
                                **engine_kw)
        self.observation_space, self.action_space = make_spaces(self.n_stack)
        self.render_mode = None
        self._actions = None
        self._t_start = time.time()
        self._attrs = dict(problem=problem, mission=mission, size=size, num_objects=num_objects,
                           max_steps=size * size, all_doors_open=all_doors_open,
                           see_through_walls=see_through_walls)
        dev = self.engine.device
        self._act_dev = torch.zeros(self.num_envs, dtype=torch.int64, device=dev)
        pin = torch.cuda.is_available()
        self._host = {k: torch.empty(v.shape, dtype=v.dtype, pin_memory=pin) for k, v in self.engine.obs.items()}
        self._host_scalars = torch.empty((4, self.num_envs), dtype=torch.float64, pin_memory=pin)
        self._ep_start = np.full(self.num_envs, time.time())

    # ------------------------------------------------------------------ SB3 API
    def seed(self, seed=None):
        """VecEnv.seed: the next reset() seeds env i with seed + i (PCG64 only)."""
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 31 - 1))
        self.engine.set_seed(seed)
        return [seed + i for i in range(self.num_envs)]

    def reset(self):
        self.engine.reset()
        self._ep_start[:] = time.time()
        return self._obs_to_host(self.engine.obs)

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        a = self._actions
        if isinstance(a, torch.Tensor):
            self._act_dev.copy_(a.reshape(-1))
        else:
            self._act_dev.copy_(torch.from_numpy(np.asarray(a, dtype=np.int64).reshape(-1)))
        e = self.engine
        obs = e.step(self._act_dev)
        sc = self._host_scalars
        sc[0].copy_(e.reward64, non_blocking=True)
        sc[1].copy_(e.terminated, non_blocking=True)
        sc[2].copy_(e.truncated, non_blocking=True)
        sc[3].copy_(e.ep_len, non_blocking=True)
        obs_h = self._obs_to_host(obs)          # synchronises the stream
        e.poll_error()
        reward64 = sc[0].numpy().copy()
        term = sc[1].numpy() != 0
        trunc = sc[2].numpy() != 0
        ep_len = sc[3].numpy().astype(np.int64)
        dones = term | trunc
        infos = [{} for _ in range(self.num_envs)]
        idx = np.nonzero(dones)[0]
        if idx.size:
            sel = torch.as_tensor(idx, device=e.device)
            t_obs = {k: v.index_select(0, sel).cpu().numpy() for k, v in e.terminal_obs.items()}
            now = time.time()
            for j, i in enumerate(idx):
                infos[i]["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
                infos[i]["terminal_observation"] = {k: v[j] for k, v in t_obs.items()}
                # Monitor: only an episode's final step can pay a reward in PlaygroundEnv
                infos[i]["episode"] = {"r": round(float(reward64[i]), 6), "l": int(ep_len[i]),
                                       "t": round(now - self._t_start, 6)}
            self._ep_start[idx] = now
        return obs_h, reward64.astype(np.float32), dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.engine.close()

    def render(self, mode=None):
        raise NotImplementedError("rendering is outside the engine's scope (DESIGN.md §8)")

    def get_attr(self, attr_name, indices=None):
        if attr_name not in self._attrs:
            raise AttributeError(attr_name)
        return [self._attrs[attr_name] for _ in self._indices(indices)]

    def set_attr(self, attr_name, value, indices=None):
        raise AttributeError("env attributes are fixed at create time (%s)" % attr_name)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        raise AttributeError("per-env methods are not exposed (%s)" % method_name)

    def env_is_wrapped(self, wrapper_class, indices=None):
        # Every env is Monitor-wrapped (make_vec_env) with TokenizeVocab/Discrete2Box inside
        name = getattr(wrapper_class, "__name__", str(wrapper_class))
        return [name in ("Monitor", "TokenizeVocabWrapper", "Discrete2BoxWrapper")
                for _ in self._indices(indices)]

    def get_images(self):
        raise NotImplementedError("rendering is outside the engine's scope (DESIGN.md §8)")

    @property
    def unwrapped(self):
        return self

    # ------------------------------------------------------------------ helpers
    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    def _obs_to_host(self, obs):
        for k, v in obs.items():
            self._host[k].copy_(v, non_blocking=True)
        torch.cuda.current_stream(self.engine.device).synchronize()
        return {k: v.numpy().copy() for k, v in self._host.items()}
