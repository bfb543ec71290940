"""Variables I/O: FLAX variable trees <-> ``.npz``.

The reference keeps variables as an in-memory pytree only (train.py:32, 138
return ``variables``; examples/deep_set.ipynb:466-485 shows the tree). A model
trained with the JAX reference is saved with its leaves converted to numpy
(``jax.tree_util.tree_map(np.asarray, variables)``) and written here as one
``.npz`` whose keys are the '/'-joined FLAX paths, e.g.
``params/bijector/bijectors_1/Dense_0/kernel`` or
``batch_stats/bijector/bijectors_0/xmin_0``. Loading rebuilds the nested
dict that ``Flow.apply`` / ``Flow.bind`` take unchanged. Only plain numeric
arrays are stored; loading never unpickles (``allow_pickle=False``)."""

from __future__ import annotations

from typing import Any, Dict

import numpy as np

SEP = "/"


def flatten_variables(variables: Dict[str, Any], prefix: str = "") -> Dict[str, np.ndarray]:
    """Nested dict of arrays -> {"a/b/c": array}."""
    out: Dict[str, np.ndarray] = {}
    for k, v in variables.items():
        if SEP in str(k):
            raise ValueError(f"key {k!r} contains the path separator {SEP!r}")
        path = f"{prefix}{SEP}{k}" if prefix else str(k)
        if isinstance(v, dict):
            if not v:
                out[path + SEP] = np.zeros((0,), np.float32)  # keep empty collections
            else:
                out.update(flatten_variables(v, path))
        else:
            a = np.asarray(v)
            if a.dtype == object:
                raise TypeError(f"{path}: not a numeric array")
            out[path] = a
    return out


def unflatten_variables(flat: Dict[str, np.ndarray]) -> Dict[str, Any]:
    """Inverse of flatten_variables."""
    tree: Dict[str, Any] = {}
    for path, a in flat.items():
        empty = path.endswith(SEP)
        parts = path.rstrip(SEP).split(SEP)
        node = tree
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        if empty:
            node.setdefault(parts[-1], {})
        else:
            node[parts[-1]] = np.asarray(a)
    return tree


def save_variables(path, variables: Dict[str, Any]) -> None:
    """Write a FLAX-layout variable tree to ``path`` (.npz)."""
    np.savez(path, **flatten_variables(variables))


def load_variables(path) -> Dict[str, Any]:
    """Read a tree written by save_variables (or any .npz with '/'-joined FLAX
    paths); arrays only, nothing executed."""
    with np.load(path, allow_pickle=False) as f:
        return unflatten_variables({k: f[k] for k in f.files})
