"""A minimal FLAX-style module protocol (``init`` / ``apply`` / variables).

zenflow's bijectors are FLAX ``nn.Module``s (bijectors.py:28); users drive them
with ``module.init(key, x, c)`` and ``module.apply(variables, x, c, train=...,
mutable=["batch_stats"], method=...)``.  This module reproduces exactly that
calling convention and the FLAX variable-tree layout (``params`` /
``batch_stats``, submodule names ``bijector``, ``bijectors_<i>``,
``BatchNorm_0``, ``Dense_<l>``) so reference-style code and variables work
unchanged.  The arithmetic itself always runs in the HIP kernels.
"""

from __future__ import annotations

import copy
import threading
from typing import Any, Dict, Optional

import numpy as np

_tls = threading.local()


class Scope:
    """Variables bound for one ``apply`` call, plus the collections it may mutate."""

    def __init__(self, variables: Dict[str, Any], mutable):
        self.variables = variables or {}
        if mutable is True:
            mutable = ["params", "batch_stats"]
        elif isinstance(mutable, str):
            mutable = [mutable]
        self.mutable = list(mutable or [])
        self.updates: Dict[str, Any] = {}
        self.initializing = False

    def collection(self, name: str) -> Dict[str, Any]:
        return self.variables.get(name, {}) or {}


def current_scope() -> Scope:
    s = getattr(_tls, "scope", None)
    if s is None:
        raise RuntimeError(
            "Can't call a zenflow_amd module outside of init/apply; use "
            "module.apply(variables, ...) (same rule as flax.linen)."
        )
    return s


def _resolve_method(module, method):
    if method is None:
        return type(module).__call__
    if isinstance(method, str):
        return getattr(type(module), method)
    return method


class Module:
    """Base class: FLAX-like ``init`` and ``apply``."""

    def init(self, rng, *args, method=None, **kwargs) -> Dict[str, Any]:
        """Create the variables (``params`` + ``batch_stats``) for the input shapes.

        Mirrors ``flax.linen.Module.init``: parameters are drawn with FLAX's
        default initialisers (lecun_normal kernels, zero biases, BatchNorm
        scale 1 / bias 0 / mean 0 / var 1); ShiftBounds stats start at +-inf.
        ``rng`` may be ``zenflow_amd.random.PRNGKey(seed)``, an int or a
        ``numpy.random.Generator``."""
        from .random import as_generator

        gen = as_generator(rng)
        x = args[0] if args else kwargs.get("x")
        c = args[1] if len(args) > 1 else kwargs.get("c")
        shape = np.shape(x)
        D = int(shape[1]) if len(shape) > 1 else 1
        cshape = None if c is None else np.shape(c)
        C = 0 if cshape is None else (1 if len(cshape) == 1 else int(cshape[1]))
        params: Dict[str, Any] = {}
        stats: Dict[str, Any] = {}
        self._init_variables(gen, D, C, params, stats)
        self._on_init(D, C)
        out: Dict[str, Any] = {}
        if params:
            out["params"] = params
        if stats:
            out["batch_stats"] = stats
        return out

    def apply(self, variables, *args, method=None, mutable=False, **kwargs):
        """Run ``method`` (default ``__call__``) with ``variables`` bound.

        With ``mutable`` (e.g. ``["batch_stats"]``) returns ``(out, updates)``
        as FLAX does."""
        fn = _resolve_method(self, method)
        scope = Scope(variables, mutable)
        prev = getattr(_tls, "scope", None)
        _tls.scope = scope
        try:
            out = fn(self, *args, **kwargs)
        finally:
            _tls.scope = prev
        if scope.mutable:
            upd = {}
            for col in scope.mutable:
                if col in scope.updates:
                    upd[col] = scope.updates[col]
                elif col in (variables or {}):
                    upd[col] = copy.deepcopy(variables[col])
            return out, upd
        return out

    # subclasses --------------------------------------------------------------
    def _init_variables(self, gen, D, C, params, stats) -> None:
        pass

    def _on_init(self, D, C) -> None:
        pass


def lecun_normal(gen: np.random.Generator, fan_in: int, fan_out: int) -> np.ndarray:
    """flax default kernel init: variance_scaling(1, 'fan_in', 'truncated_normal')."""
    std = np.sqrt(1.0 / max(1, fan_in)) / 0.87962566103423978
    z = gen.standard_normal((fan_in, fan_out))
    bad = np.abs(z) > 2.0
    while bad.any():
        z[bad] = gen.standard_normal(int(bad.sum()))
        bad = np.abs(z) > 2.0
    return (z * std).astype(np.float32)


def get_path(tree: Dict[str, Any], path) -> Any:
    node = tree
    for k in path:
        if not isinstance(node, dict) or k not in node:
            return None
        node = node[k]
    return node


def set_path(tree: Dict[str, Any], path, value) -> None:
    node = tree
    for k in path[:-1]:
        node = node.setdefault(k, {})
    node[path[-1]] = value
