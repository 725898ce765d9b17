"""Minimal Discrete / Box spaces (the two gym.spaces classes othello.py:245-254 uses).

gym is not a dependency of this package; these expose the attributes the
reference's callers read (`n`, `shape`, `low`, `high`) plus sample/contains.
"""
import numpy as np


class Discrete(object):
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64

    def sample(self, rng=np.random):
        return int(rng.randint(self.n))

    def contains(self, x):
        try:
            x = int(x)
        except (TypeError, ValueError):
            return False
        return 0 <= x < self.n

    def __repr__(self):
        return "Discrete(%d)" % self.n


class Box(object):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low = np.asarray(low, dtype=dtype)
        self.high = np.asarray(high, dtype=dtype)
        self.shape = tuple(shape) if shape is not None else self.low.shape
        self.dtype = dtype

    def sample(self, rng=np.random):
        return rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return "Box(%s)" % (self.shape,)
