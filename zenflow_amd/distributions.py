"""Latent distributions — drop-in for ``zenflow.distributions``
(reference: src/zenflow/distributions.py).

``log_prob`` runs on the GPU (the same latent epilogue the fused flow kernel
uses).  ``sample`` draws on the host from a seeded numpy Generator: JAX's
threefry stream is not reproducible without JAX, so sampling parity is
statistical (moments), exactly as the reference tests check it."""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional

import numpy as np

from . import _lib as L
from .random import as_generator


class Distribution(ABC):
    """Distribution base class with lazy ``dim`` (distributions.py:11-47)."""

    _dim: Optional[int] = None

    def log_prob(self, x):
        """Log-probability of N samples (N, D) -> (N,)."""
        shape = x.shape if isinstance(x, L.DeviceArray) else np.shape(x)
        if self._dim is None:
            self._dim = int(shape[-1])
        return self._log_prob_impl(x)

    @property
    def dim(self):
        return self._dim

    def _log_prob_impl(self, x):
        from .engine import Program
        from .bijectors import Chain

        xd, was_dev = L.as_device(x)
        if xd.ndim != 2:
            raise ValueError("x must be (N, D)")
        prog = Program(Chain(()), {}, xd.shape[1], 0, latent=self)
        lp = prog.log_prob(xd)
        return lp if was_dev else lp.numpy()

    @abstractmethod
    def sample(self, nsamples: int, rngkey) -> np.ndarray: ...

    def __repr__(self):
        return f"{self.__class__.__name__}()"


class Normal(Distribution):
    """Multivariate normal, mean 0.5, standard deviation 0.1 (distributions.py:50-62)."""

    def sample(self, nsamples: int, rngkey) -> np.ndarray:
        g = as_generator(rngkey)
        return (0.5 + 0.1 * g.standard_normal((nsamples, self.dim))).astype(np.float32)


class TruncatedNormal(Distribution):
    """Normal truncated to [0, 1] (+-5 sigma) (distributions.py:65-78)."""

    def sample(self, nsamples: int, rngkey) -> np.ndarray:
        g = as_generator(rngkey)
        z = g.standard_normal((nsamples, self.dim))
        bad = np.abs(z) > 5
        while bad.any():
            z[bad] = g.standard_normal(int(bad.sum()))
            bad = np.abs(z) > 5
        return (0.5 + 0.1 * z).astype(np.float32)


class Beta(Distribution):
    """Symmetric multivariate beta; the default latent of ``Flow``
    (distributions.py:81-116)."""

    def __init__(self, peakness: float = 12.0):
        if peakness < 1:
            raise ValueError("peakness must be at least 1")
        self.peakness = peakness

    def sample(self, nsamples: int, rngkey) -> np.ndarray:
        g = as_generator(rngkey)
        return g.beta(self.peakness, self.peakness, (nsamples, self.dim)).astype(np.float32)

    def __repr__(self):
        return f"{self.__class__.__name__}(peakness={self.peakness})"


class Uniform(Distribution):
    """Multivariate uniform on [0, 1] (distributions.py:119-126)."""

    def sample(self, nsamples: int, rngkey) -> np.ndarray:
        g = as_generator(rngkey)
        return g.uniform(size=(nsamples, self.dim)).astype(np.float32)
