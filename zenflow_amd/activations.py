"""Activations for ``NeuralSplineCoupling(act=...)`` (bijectors.py:319: any
callable, default ``flax.linen.swish``).

The kernels evaluate the activation themselves, so ``act`` must be one they
implement: these functions (numpy forms of the flax.linen / jax.nn
functions of the same names, usable on host arrays), a name string, or any
callable that computes one of them.  A callable is never trusted by its
``__name__`` alone: it is evaluated on probe points (both signs, the kinks,
the saturating tails out to |x| = 1e3 and seeded random points) and must
match the implemented form it names, or — without a known name — one of
them (a warning says which); anything else raises NotImplementedError.

Kernels (zf_flow_create picks them): the split-MFMA kernel
runs all eight on its f16x2 scheme — swish on its tuned form, relu /
leaky_relu / tanh / gelu / elu through the ``OACT`` instantiation, sigmoid
and softplus there too, centred on 1/2 and log 2.  The trainer takes all
eight."""

from __future__ import annotations

import warnings
from typing import Callable, Union

import numpy as np

from . import _lib as L

__all__ = ["swish", "silu", "relu", "tanh", "sigmoid", "gelu", "softplus", "elu", "leaky_relu", "act_code"]


def _tag(code: int):
    def deco(fn):
        fn.zf_act = code
        return fn
    return deco


@_tag(L.ZF_ACT_SWISH)
def swish(x):
    """jax.nn.silu / flax.linen.swish: x * sigmoid(x)."""
    x = np.asarray(x)
    return x / (1 + np.exp(-x))


silu = swish


@_tag(L.ZF_ACT_RELU)
def relu(x):
    return np.maximum(np.asarray(x), 0)


@_tag(L.ZF_ACT_TANH)
def tanh(x):
    return np.tanh(x)


@_tag(L.ZF_ACT_SIGMOID)
def sigmoid(x):
    return 1 / (1 + np.exp(-np.asarray(x)))


@_tag(L.ZF_ACT_GELU)
def gelu(x):
    """jax.nn.gelu(approximate=True) (flax.linen.gelu's default)."""
    x = np.asarray(x)
    return 0.5 * x * (1 + np.tanh(np.sqrt(2 / np.pi) * (x + 0.044715 * x**3)))


@_tag(L.ZF_ACT_SOFTPLUS)
def softplus(x):
    """jax.nn.softplus = logaddexp(x, 0)."""
    return np.logaddexp(np.asarray(x), 0)


@_tag(L.ZF_ACT_ELU)
def elu(x):
    """jax.nn.elu, alpha = 1."""
    x = np.asarray(x)
    return np.where(x > 0, x, np.expm1(np.minimum(x, 0)))


@_tag(L.ZF_ACT_LEAKY_RELU)
def leaky_relu(x):
    """jax.nn.leaky_relu, negative slope 0.01."""
    x = np.asarray(x)
    return np.where(x >= 0, x, 0.01 * x)


_BY_NAME = {f.__name__: f.zf_act for f in (swish, relu, tanh, sigmoid, gelu, softplus, elu, leaky_relu)}
_BY_NAME["silu"] = L.ZF_ACT_SWISH
_NAMES = {v: k for k, v in _BY_NAME.items() if k != "silu"}


# probe points: both signs, the kinks of relu / leaky_relu / elu at 0, values
# around 1, the saturating tails out to |x| = 1e3, and seeded random points
# (so a piecewise function that agrees on a fixed grid is still caught)
_PROBE = np.concatenate([
    np.linspace(-12.0, 12.0, 97),
    [-1e-3, -1e-6, 0.0, 1e-6, 1e-3, 0.3, 0.7, 1.3],
    [-1e3, -300.0, -100.0, -40.0, -20.0, 20.0, 40.0, 100.0, 300.0, 1e3],
    np.random.default_rng(20250204).standard_normal(96) * 6.0,
    np.random.default_rng(20250205).uniform(-3.0, 3.0, 32) ** 5.0,
])


def _probe(act: Callable) -> int:
    """The implemented activation a callable computes, found by evaluating it
    (NeuralSplineCoupling.act is any callable, bijectors.py:319): a match
    within 1e-6 of max(1, |f(x)|) at every probe point; -1 if none, -2 if the
    callable cannot be evaluated on a float32 array."""
    try:
        with np.errstate(all="ignore"):
            y = np.asarray(act(_PROBE.astype(np.float32)), np.float64)
    except Exception:  # noqa: BLE001 — a callable that cannot take an array
        return -2
    if y.shape != _PROBE.shape or not np.all(np.isfinite(y)):
        return -1
    for fn in (swish, relu, tanh, sigmoid, gelu, softplus, elu, leaky_relu):
        with np.errstate(all="ignore"):
            ref = np.asarray(fn(_PROBE), np.float64)
        if np.all(np.abs(y - ref) <= 1e-6 * np.maximum(1.0, np.abs(ref))):
            return fn.zf_act
    return -1


def act_code(act: Union[str, Callable]) -> int:
    """ZF_ACT_* of an activation: a function of this module, a name string,
    or a callable that computes an implemented activation.  A callable whose
    ``__name__`` is an implemented name must also compute that activation on
    the probe points (a user's own ``def swish(x)`` with another slope is not
    jax's swish); a callable of any other name is matched by value, with a
    warning.  NotImplementedError otherwise."""
    code = getattr(act, "zf_act", None)
    if code is not None:
        return int(code)
    if isinstance(act, str):
        if act in _BY_NAME:
            return _BY_NAME[act]
        raise NotImplementedError(f"activation {act!r} has no HIP implementation ({', '.join(sorted(_BY_NAME))})")
    if not callable(act):
        raise NotImplementedError(f"activation {act!r} is neither a name nor a callable")
    name = getattr(act, "__name__", None)
    found = _probe(act)
    if name in _BY_NAME:
        want = _BY_NAME[name]
        if found == want:
            return want
        if found == -2:  # cannot be called on a host array: the name is all there is
            warnings.warn(f"activation {name!r} could not be evaluated on a host array; "
                          f"running the kernels' {name} by its name alone", RuntimeWarning, stacklevel=3)
            return want
        raise NotImplementedError(
            f"activation {act!r} is named {name!r} but does not compute the implemented {name} "
            f"(jax.nn form) on the probe points; pass zenflow_amd.activations.{_NAMES[want]} or a matching callable")
    if found >= 0:
        warnings.warn(f"activation {act!r} recognised by value as {_NAMES[found]}: the kernels run "
                      f"their {_NAMES[found]}", RuntimeWarning, stacklevel=3)
        return found
    raise NotImplementedError(
        f"activation {act!r} has no HIP implementation and computes none of the implemented ones "
        f"({', '.join(sorted(_BY_NAME))})")


def act_name(code: int) -> str:
    return _NAMES[int(code)]
