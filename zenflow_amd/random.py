"""Seeds for init / sample (stand-in for ``jax.random.PRNGKey``).

JAX's threefry stream cannot be reproduced without JAX: parameter init uses
seeded numpy Generators, latent sampling the device's counter-based Philox
generator keyed by ``key_to_seed(key)`` — same distributions, different draws
(parity for sampling is statistical; DESIGN.md §2 sampling)."""

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


def key_to_seed(key) -> int:
    """64-bit device seed of a key (``PRNGKey`` array, int, or None)."""
    if key is None:
        return 0
    if isinstance(key, (int, np.integer)):
        return int(key) & 0xFFFFFFFFFFFFFFFF
    arr = np.asarray(key).astype(np.uint64).ravel()
    if arr.size == 2:
        return (int(arr[0]) << 32) | int(arr[1])
    h = 0
    for v in arr:
        h = (h * 0x9E3779B97F4A7C15 + int(v)) & 0xFFFFFFFFFFFFFFFF
    return h
