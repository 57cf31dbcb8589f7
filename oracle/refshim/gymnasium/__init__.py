"""Clean-room restatement of the tiny slice of the gymnasium API that the
reference's `src/custom_env.py` / `src/environment.py` touch.

TEST INFRASTRUCTURE ONLY.  gymnasium is not installed in this image and is not
vendored by the reference (`requirements.txt:8`, unpinned).  This module exists
so that `tests/golden/make_golden.py` can execute the reference's own
`custom_env.py` unchanged to produce golden fixtures.  It is never imported by
the product path and never travels a semantic decision into the engine.

Semantics restated (gymnasium >= 0.26, public API):
* `Env.reset(seed=s)` re-creates `self.np_random` as
  `numpy.random.Generator(PCG64(SeedSequence(s)))` (gymnasium.utils.seeding).
* `ObservationWrapper.step/reset` forward to the inner env and map the obs.
"""
import numpy as np

from . import spaces  # noqa: F401


class _Logger:
    ERROR = 40
    min_level = 30


logger = _Logger()


def _np_random(seed):
    ss = np.random.SeedSequence(seed)
    return np.random.Generator(np.random.PCG64(ss)), ss.entropy


class Env:
    metadata = {"render_modes": []}
    render_mode = None
    _np_random = None

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random, _ = _np_random(None)
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._np_random, _ = _np_random(seed)

    @property
    def unwrapped(self):
        return self


class Wrapper(Env):
    def __init__(self, env):
        self.env = env
        self._observation_space = None

    @property
    def observation_space(self):
        if self._observation_space is None:
            return self.env.observation_space
        return self._observation_space

    @observation_space.setter
    def observation_space(self, space):
        self._observation_space = space

    @property
    def action_space(self):
        return self.env.action_space

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def step(self, action):
        return self.env.step(action)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)


class ObservationWrapper(Wrapper):
    def reset(self, **kwargs):
        obs, info = self.env.reset(**kwargs)
        return self.observation(obs), info

    def step(self, action):
        obs, reward, terminated, truncated, info = self.env.step(action)
        return self.observation(obs), reward, terminated, truncated, info

    def observation(self, obs):
        raise NotImplementedError


def make(*args, **kwargs):
    raise RuntimeError("gymnasium.make is not available in the oracle shim")
