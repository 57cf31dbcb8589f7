"""Observation / action spaces of the wrapped PlaygroundEnv.

Uses gymnasium.spaces when gymnasium is importable (the reference's own
dependency); otherwise minimal duck-typed stand-ins with the attributes SB3 and
the policy read (shape, dtype, low, high, n, spaces).  Shapes are the ones the
reference's wrapper stack produces (environment.py:84-89,142 then SB3
VecTransposeImage + VecFrameStack(n, 'first'), ppo.py:124-126).
"""
import numpy as np

try:  # pragma: no cover - gymnasium is absent in this image
    from gymnasium import spaces as _gs
except ImportError:  # pragma: no cover
    _gs = None


class Box:
    def __init__(self, low, high, shape, dtype):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return "Box(%s, %s, %s, %s)" % (self.low.min(), self.high.max(), self.shape, self.dtype)


class Discrete:
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)

    def contains(self, x):
        return 0 <= int(x) < self.n

    def __repr__(self):
        return "Discrete(%d)" % self.n


class Dict:
    def __init__(self, spaces):
        self.spaces = dict(spaces)

    def __getitem__(self, k):
        return self.spaces[k]

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()

    def __repr__(self):
        return "Dict(%s)" % ", ".join("%s: %r" % kv for kv in self.spaces.items())


def make_spaces(n_stack, mission_dtype=np.int64, raw=False, dir_one_hot=True):
    """(observation_space, action_space) of the stacked, transposed env -- or, raw=True, of one
    wrapped env as make_vec_env hands it out (environment.py:84-89,142): image HWC (7,7,3).
    dir_one_hot (raw only): make_env applies Discrete2BoxWrapper only when n_frames_stack > 1 and not
    recurrent (environment.py:28-29); otherwise the direction is MiniGridEnv's own Discrete(4)."""
    mk_box = (lambda lo, hi, shape, dt: _gs.Box(lo, hi, shape, dt)) if _gs else Box
    mk_dict = _gs.Dict if _gs else Dict
    mk_disc = _gs.Discrete if _gs else Discrete
    if raw:
        obs = mk_dict({
            "direction": mk_box(0, 1, (4,), np.uint8) if dir_one_hot else mk_disc(4),   # Discrete2BoxWrapper | raw
            "image": mk_box(0, 255, (7, 7, 3), np.uint8),              # MiniGridEnv image, [vx][vy][c]
            "mission": mk_box(0, 32, (32,), mission_dtype),            # TokenizeVocabWrapper
        })
        return obs, mk_disc(7)
    obs = mk_dict({
        "direction": mk_box(0, 1, (4 * n_stack,), np.uint8),          # Discrete2BoxWrapper, stacked
        "image": mk_box(0, 255, (3 * n_stack, 7, 7), np.uint8),       # transposed to CHW, stacked
        "mission": mk_box(0, 32, (32 * n_stack,), mission_dtype),     # TokenizeVocabWrapper, stacked
    })
    return obs, mk_disc(7)                                            # MiniGridEnv.Actions (7)
