"""Latent distributions — drop-in for ``zenflow.distributions``
(reference: src/zenflow/distributions.py).

``log_prob`` runs on the GPU (the same latent epilogue the fused flow kernel
uses).  ``sample`` draws on the GPU too (``zf_latent_sample``: Philox4x32-10
keyed by the seed, counter = (row, dim), zf_random.h): JAX's threefry stream
is not reproducible without JAX, so sampling parity is statistical (KS tests,
moments), as the reference tests check it."""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional

import numpy as np

from . import _lib as L
from .random import key_to_seed


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

    def _device_sample(self, nsamples: int, rngkey) -> np.ndarray:
        """Draw (nsamples, dim) on the GPU (zf_latent_sample: Philox keyed by
        the key's 64-bit seed); the same z zf_flow_sample feeds the inverse."""
        from .engine import _latent_code

        if self.dim is None:
            raise ValueError("dim unknown: call log_prob first")
        code, param = _latent_code(self)
        L.ensure_device()
        z = L.DeviceArray((int(nsamples), self.dim))
        L.check(L.load_library().zf_latent_sample(code, param, key_to_seed(rngkey), z.ptr, int(nsamples),
                                                  self.dim, L.stream()), "zf_latent_sample")
        return z.numpy()

    def __repr__(self):
        return f"{self.__class__.__name__}()"


class Normal(Distribution):
    """Multivariate normal, mean 0.5, standard deviation 0.1 (distributions.py:50-62)."""

    def sample(self, nsamples: int, rngkey) -> np.ndarray:
        return self._device_sample(nsamples, rngkey)


class TruncatedNormal(Distribution):
    """Normal truncated to [0, 1] (+-5 sigma) (distributions.py:65-78)."""

    def sample(self, nsamples: int, rngkey) -> np.ndarray:
        return self._device_sample(nsamples, rngkey)


class Beta(Distribution):
    """Symmetric multivariate beta; the default latent of ``Flow``
    (distributions.py:81-116)."""

    def __init__(self, peakness: float = 12.0):
        if peakness < 1:
            raise ValueError("peakness must be at least 1")
        self.peakness = peakness

    def sample(self, nsamples: int, rngkey) -> np.ndarray:
        return self._device_sample(nsamples, rngkey)

    def __repr__(self):
        return f"{self.__class__.__name__}(peakness={self.peakness})"


class Uniform(Distribution):
    """Multivariate uniform on [0, 1] (distributions.py:119-126)."""

    def sample(self, nsamples: int, rngkey) -> np.ndarray:
        return self._device_sample(nsamples, rngkey)
