"""MgxVecEnv: the SB3 `VecEnv` face of the engine (host numpy in/out).

This is the drop-in for the object the reference builds at src/ppo.py:118-126:

    vec_env = make_vec_env(make_env, n_envs, seed, SubprocVecEnv, env_kwargs=...)     # :118-122
    if cfg.algorithm.n_frames_stack > 1 and not cfg.algorithm.recurrent:               # :124
        vec_env = VecTransposeImage(vec_env)                                           # :125
        vec_env = VecFrameStack(vec_env, n_frames_stack, channels_order='first')       # :126
    model = algo(policy=policy, env=vec_env, **config)                                 # :134-136

Two modes:

  * raw (`raw=True`, the drop-in for line 118 alone): observations are exactly what
    make_vec_env's envs return -- image HWC (7,7,3), one-hot direction (4,), mission tokens
    (32,) int64 (environment.py:84-89,142) -- so lines 124-126 and SB3's own wrappers run
    unchanged on top, and `PPO(policy, env)` sees the same wrapper chain as in the reference
    (BaseAlgorithm._wrap_env finds its VecTransposeImage and adds nothing);
  * fused (default): the engine does VecTransposeImage + VecFrameStack(n, 'first') itself
    (stacked CHW image (3n,7,7), direction (4n,), mission (32n,)) -- the replacement for
    lines 118-126 together, for callers that do not pass the env through SB3's _wrap_env
    (which, not seeing a VecTransposeImage in the chain, would transpose the (3n,7,7) image
    space again: use raw mode with SB3's algorithms).

Raw mode follows make_env's wrapper rule (environment.py:28-29): the direction is the one-hot Box(4,)
of Discrete2BoxWrapper only when n_frames_stack > 1 and not recurrent; otherwise it is MiniGridEnv's
Discrete(4) (an int64 per env on the host).

Trajectories are SubprocVecEnv's (ppo.py:121, single_run): each env its own CPython `random`
(MT19937(seed), custom_env.py:82).  The reference's MULTIRUN branch (`DummyVecEnv`) runs every env in
one process, whose envs then draw from ONE process-global MT stream interleaved by env index; the
engine does not reproduce that interleaving (`vec_env_cls="dummy"` with n_envs > 1 warns).

When stable_baselines3 is importable the class subclasses its `VecEnv` (so `_wrap_env` does
not re-wrap it in a DummyVecEnv); otherwise it duck-types the same contract
(stable_baselines3.common.vec_env.base_vec_env):

  * reset() -> obs dict; step_async(actions) / step_wait() -> (obs, rewards
    f32[N], dones bool[N], infos list[N]); step(actions); seed(seed);
    num_envs, observation_space, action_space; close(); get_attr / set_attr /
    env_method / env_is_wrapped for the few attributes the PPO loop reads;
  * obs arrays are COPIES owned by the caller (_obs_from_buf);
  * infos[i] of a done env carries 'terminal_observation' (the final obs, stacked
    and transposed in fused mode as VecFrameStack.step_wait does), 'TimeLimit.truncated'
    (truncated and not terminated, SubprocVecEnv worker) and Monitor's 'episode'
    {'r', 'l', 't'}.

The PPO loop of this package does not go through here: it keeps everything on
device (MgxEngine).  This class is for callers that want the reference's host
API unchanged, at the cost of a device->host copy of the observation per step.
"""
import time
import warnings

import numpy as np
import torch

from .engine import MgxEngine
from .spaces import make_spaces

try:  # pragma: no cover - SB3 is absent in this image (parity of this layer is unpinned)
    from stable_baselines3.common.vec_env import VecEnv as _VecEnvBase
    HAVE_SB3 = True
except ImportError:  # pragma: no cover
    _VecEnvBase = object
    HAVE_SB3 = False


class MgxVecEnv(_VecEnvBase):
    """SB3-compatible vectorised PlaygroundEnv on one GPU.

    cfg_env mirrors `cfg.env` of the reference (single.yaml: problem, mission,
    size, num_objects, all_doors_open, see_through_walls, obstacles)."""

    metadata = {"render_modes": []}

    def __init__(self, n_envs, seed=42, n_frames_stack=4, problem="multi", mission=5, size=8, num_objects=4,
                 all_doors_open=False, see_through_walls=True, obstacles=False, device="cuda",
                 env_index_offset=0, raw=False, recurrent=False, vec_env_cls="subproc", **engine_kw):
        self.num_envs = int(n_envs)
        self.raw = bool(raw)
        self.n_stack = 1 if self.raw else int(n_frames_stack)
        if self.raw:
            # make_env wraps the direction in Discrete2BoxWrapper only when n_frames_stack > 1 and not
            # recurrent (environment.py:28-29); otherwise the env hands out MiniGridEnv's Discrete(4)
            self.dir_one_hot = int(n_frames_stack) > 1 and not recurrent
        else:
            if recurrent or int(n_frames_stack) <= 1:
                raise ValueError("fused mode is VecTransposeImage + VecFrameStack, which the reference applies only "
                                 "when n_frames_stack > 1 and not recurrent (ppo.py:124, environment.py:28): "
                                 "use raw=True")
            self.dir_one_hot = True
        if vec_env_cls not in ("subproc", "dummy"):
            raise ValueError("vec_env_cls must be 'subproc' or 'dummy'")
        if vec_env_cls == "dummy" and self.num_envs > 1:
            warnings.warn("MgxVecEnv reproduces SubprocVecEnv trajectories (one CPython random per env, "
                          "custom_env.py:82); the reference's DummyVecEnv branch (ppo.py:121, multirun) shares one "
                          "process-global MT19937 stream across its envs, so its trajectories differ for n_envs > 1",
                          RuntimeWarning, stacklevel=2)
        self.engine = MgxEngine(problem=problem, mission=mission, size=size, num_objects=num_objects,
                                n_envs=n_envs, seed=seed, env_index_offset=env_index_offset, n_stack=self.n_stack,
                                all_doors_open=all_doors_open, see_through_walls=see_through_walls,
                                obstacles=obstacles, terminal_mode="all", reward64=True, device=device,
                                **engine_kw)
        obs_space, act_space = make_spaces(self.n_stack, raw=self.raw, dir_one_hot=self.dir_one_hot)
        self.render_mode = None
        self._attrs = dict(problem=problem, mission=mission, size=size, num_objects=num_objects,
                           max_steps=size * size, all_doors_open=all_doors_open,
                           see_through_walls=see_through_walls, render_mode=None)
        if HAVE_SB3:
            _VecEnvBase.__init__(self, self.num_envs, obs_space, act_space)
        else:
            self.observation_space, self.action_space = obs_space, act_space
            self.reset_infos = [{} for _ in range(self.num_envs)]
        self._seeds = [None] * self.num_envs
        self._actions = None
        self._t_start = time.time()
        dev = self.engine.device
        self._act_dev = torch.zeros(self.num_envs, dtype=torch.int64, device=dev)
        pin = torch.cuda.is_available()
        self._host = {k: torch.empty(self._host_shape(k, v), dtype=self._layout(k, v[:1]).dtype, pin_memory=pin)
                      for k, v in self.engine.obs.items()}
        self._host_scalars = torch.empty((4, self.num_envs), dtype=torch.float64, pin_memory=pin)
        self._ep_start = np.full(self.num_envs, time.time())

    # ------------------------------------------------------------------ SB3 API
    def seed(self, seed=None):
        """VecEnv.seed: the next reset() seeds env i with seed + i (PCG64 only)."""
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 31 - 1))
        self.engine.set_seed(seed)
        self._seeds = [seed + i for i in range(self.num_envs)]
        return list(self._seeds)

    def reset(self):
        self.engine.reset()
        self._seeds = [None] * self.num_envs
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
            t_obs = {k: self._layout(k, v.index_select(0, sel)).cpu().numpy() for k, v in e.terminal_obs.items()}
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
        raise NotImplementedError("rendering is outside the engine's scope (DESIGN.md §9)")

    def get_attr(self, attr_name, indices=None):
        if attr_name not in self._attrs:
            raise AttributeError(attr_name)
        return [self._attrs[attr_name] for _ in self._indices(indices)]

    def set_attr(self, attr_name, value, indices=None):
        raise AttributeError("env attributes are fixed at create time (%s)" % attr_name)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        raise AttributeError("per-env methods are not exposed (%s)" % method_name)

    def env_is_wrapped(self, wrapper_class, indices=None):
        name = getattr(wrapper_class, "__name__", str(wrapper_class))
        # Every env is Monitor-wrapped (make_vec_env) with TokenizeVocabWrapper inside; Discrete2BoxWrapper only
        # where make_env adds it (n_frames_stack > 1 and not recurrent, environment.py:28-29)
        wrapped = ("Monitor", "TokenizeVocabWrapper") + (("Discrete2BoxWrapper",) if self.dir_one_hot else ())
        return [name in wrapped for _ in self._indices(indices)]

    def get_images(self):
        raise NotImplementedError("rendering is outside the engine's scope (DESIGN.md §9)")

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

    def _host_shape(self, key, v):
        if self.raw and key == "image":          # (N, 3, 7, 7) [c][vx][vy] -> the env's (N, 7, 7, 3)
            return (v.shape[0], 7, 7, 3)
        if key == "direction" and not self.dir_one_hot:
            return (v.shape[0],)
        return tuple(v.shape)

    def _layout(self, key, v):
        """Engine tensor -> the layout this VecEnv hands out (raw mode: the env's HWC image; the Discrete(4)
        direction where make_env adds no Discrete2BoxWrapper)."""
        if self.raw and key == "image":
            return v.permute(0, 2, 3, 1)
        if key == "direction" and not self.dir_one_hot:
            return v.argmax(1)                   # one-hot (4,) of the single frame -> int64 direction
        return v

    def _obs_to_host(self, obs):
        for k, v in obs.items():
            self._host[k].copy_(self._layout(k, v), non_blocking=True)
        torch.cuda.current_stream(self.engine.device).synchronize()
        return {k: v.numpy().copy() for k, v in self._host.items()}
