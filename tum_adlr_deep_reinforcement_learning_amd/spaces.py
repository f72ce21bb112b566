"""Observation / action spaces.

Uses ``gym.spaces.Box`` when gym is installed (so SB3's space checks see the
real class), otherwise a minimal Box with the attributes SB3 0.10 reads
(``low``, ``high``, ``shape``, ``dtype``, ``sample``, ``contains``).
"""
import numpy as np

try:  # pragma: no cover - gym is not installed in the build image
    from gym.spaces import Box  # noqa: F401
except Exception:  # noqa: BLE001

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            if shape is not None and np.isscalar(low):
                low = np.full(shape, low)
                high = np.full(shape, high)
            self.low = np.asarray(low, dtype=self.dtype)
            self.high = np.asarray(high, dtype=self.dtype)
            self.shape = self.low.shape
            self._rng = np.random.RandomState()

        def seed(self, seed=None):
            self._rng = np.random.RandomState(seed)
            return [seed]

        def sample(self):
            lo = np.maximum(self.low.astype(np.float64), -1e6)
            hi = np.minimum(self.high.astype(np.float64), 1e6)
            return self._rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return "Box(%s, %s)" % (self.shape, self.dtype)

        def __eq__(self, other):
            return isinstance(other, Box) and self.shape == other.shape and np.allclose(self.low, other.low) and \
                np.allclose(self.high, other.high)
