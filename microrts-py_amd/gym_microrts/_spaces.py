"""Observation / action spaces of MicroRTSGridModeVecEnv.

Uses gym.spaces when gym is importable (the reference constructs
gym.spaces.Box / MultiDiscrete at vec_env.py:242-252).  gym is not installed in
this image, so a minimal stand-in with the attributes the drivers read
(`shape`, `dtype`, `nvec`, `seed`, `sample`, `contains`) is provided.
"""
import numpy as np

try:  # pragma: no cover - depends on the environment
    import gym as _gym

    if getattr(_gym, "__microrts_compat__", False):  # our own stand-in (compat/gym) re-exports this module
        raise ImportError("gym stand-in")
    from gym.spaces import Box, Discrete, MultiDiscrete  # noqa: F401
except Exception:  # gym absent

    class _Space:
        def __init__(self, shape, dtype):
            self.shape = tuple(shape)
            self.dtype = np.dtype(dtype)
            self.np_random = np.random.default_rng()

        def seed(self, seed=None):
            self.np_random = np.random.default_rng(seed)
            return [seed]

    class Box(_Space):
        def __init__(self, low, high, shape, dtype=np.float32):
            super().__init__(shape, dtype)
            self.low = np.full(self.shape, low, dtype=self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype)

        def sample(self):
            return self.np_random.integers(self.low, self.high + 1, size=self.shape).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class MultiDiscrete(_Space):
        def __init__(self, nvec, dtype=np.int64):
            self.nvec = np.asarray(nvec, dtype=np.int64)
            super().__init__(self.nvec.shape, dtype)

        def sample(self):
            return (self.np_random.random(self.nvec.shape) * self.nvec).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= 0)) and bool(np.all(x < self.nvec))

        def __repr__(self):
            return f"MultiDiscrete({self.nvec})"

    class Discrete(_Space):
        """gym.spaces.Discrete(n) (MicroRTSBotVecEnv's dummy spaces, vec_env.py:1180-1181)"""

        def __init__(self, n):
            self.n = int(n)
            super().__init__((), np.int64)

        def sample(self):
            return int(self.np_random.integers(self.n))

        def contains(self, x):
            return 0 <= int(x) < self.n

        def __repr__(self):
            return f"Discrete({self.n})"
