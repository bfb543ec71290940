"""Seeds for init / sample (stand-in for ``jax.random.PRNGKey``).

JAX's threefry stream cannot be reproduced without JAX, so parameter init and
latent sampling are seeded numpy Generators: same distributions, different
draws (parity for sampling is statistical)."""

from __future__ import annotations

import numpy as np


def PRNGKey(seed: int) -> np.ndarray:
    """Same shape/dtype as ``jax.random.PRNGKey(seed)`` (uint32[2])."""
    s = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.array([s >> 32, s & 0xFFFFFFFF], dtype=np.uint32)


def as_generator(key) -> np.random.Generator:
    if isinstance(key, np.random.Generator):
        return key
    if key is None:
        return np.random.default_rng(0)
    if isinstance(key, (int, np.integer)):
        return np.random.default_rng(int(key))
    arr = np.asarray(key, dtype=np.uint64).ravel()
    return np.random.default_rng([int(v) for v in arr])
