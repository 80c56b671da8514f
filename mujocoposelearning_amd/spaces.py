"""gymnasium compatibility: use gymnasium's Env/Box when installed (the reference pins 0.28.1,
environment.yml:95), else a minimal stand-in with the attributes the reference and SB3 read."""
import numpy as np

try:  # pragma: no cover - exercised only where gymnasium is installed
    from gymnasium import Env
    from gymnasium.spaces import Box
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class Env:
        metadata = {}
        render_mode = None

        def close(self):
            pass

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.full(self.shape, low, dtype=self.dtype) if np.isscalar(low) else np.asarray(low, self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype) if np.isscalar(high) else np.asarray(high, self.dtype)
            self._rng = np.random.default_rng(seed)

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return self._rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"
