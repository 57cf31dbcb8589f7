"""Minimal gymnasium.spaces restatement (TEST INFRASTRUCTURE ONLY; see package doc)."""
import numpy as np


class Space:
    pass


class Discrete(Space):
    def __init__(self, n, start=0):
        self.n = int(n)
        self.start = int(start)
        self.shape = ()
        self.dtype = np.int64


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low)
        self.shape = tuple(shape)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)


class Dict(Space):
    def __init__(self, spaces=None):
        self.spaces = dict(spaces or {})

    def __getitem__(self, k):
        return self.spaces[k]

    def __setitem__(self, k, v):
        self.spaces[k] = v

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()


class Text(Space):
    def __init__(self, max_length=4096, **kw):
        self.max_length = max_length
