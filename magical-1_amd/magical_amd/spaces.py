"""Minimal gym.spaces stand-ins (gym is optional; used when it is importable)."""
import collections

import numpy as np

try:  # pragma: no cover - exercised only where gym is installed
    from gym.spaces import Box, Dict, Discrete  # noqa: F401
except Exception:  # gym absent in this image
    class Discrete:
        def __init__(self, n):
            self.n = n
            self.shape = ()
            self.dtype = np.int64
            self._rng = np.random.RandomState()

        def seed(self, seed=None):
            self._rng = np.random.RandomState(seed)
            return [seed]

        def sample(self):
            return int(self._rng.randint(self.n))

        def contains(self, x):
            return 0 <= int(x) < self.n

        def __repr__(self):
            return f"Discrete({self.n})"

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.shape = tuple(shape)
            self.dtype = np.dtype(dtype)
            self.low = np.full(self.shape, low, dtype=self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and x.dtype == self.dtype

        def __repr__(self):
            return f"Box({self.shape}, {self.dtype})"

    class Dict:
        def __init__(self, spaces):
            self.spaces = collections.OrderedDict(spaces)

        def __getitem__(self, k):
            return self.spaces[k]

        def keys(self):
            return self.spaces.keys()

        def __repr__(self):
            return f"Dict({dict(self.spaces)})"
