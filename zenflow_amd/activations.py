"""Activations for ``NeuralSplineCoupling(act=...)`` (bijectors.py:319: any
callable, default ``flax.linen.swish``).

The kernels evaluate the activation themselves, so ``act`` must be one they
implement: these functions (numpy forms of the flax.linen / jax.nn
functions of the same names, usable on host arrays), a name string, any
callable with one of these ``__name__``s (e.g. ``flax.linen.relu``), or any
callable that computes one of them (``lambda x: x / (1 + np.exp(-x))`` is
swish: recognised by evaluating it on probe points).  The
split-MFMA kernel fuses swish (the reference default); the others run on the
fp32-MFMA kernel and in the trainer."""

from __future__ import annotations

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


# probe points for callables of unknown name: both signs, the kinks of relu /
# leaky_relu / elu at 0, the saturating tails, values around 1
_PROBE = np.concatenate([np.linspace(-12.0, 12.0, 97), [-1e-3, -1e-6, 0.0, 1e-6, 1e-3, 0.3, 0.7, 1.3]])


def _probe(act: Callable) -> int:
    """The implemented activation a callable computes, found by evaluating it
    (NeuralSplineCoupling.act is any callable, bijectors.py:319: a lambda or
    a wrapped jax.nn function of a supported form runs on the kernels).  A
    match within 1e-6 relative over the probe points; -1 if none."""
    try:
        with np.errstate(all="ignore"):
            y = np.asarray(act(_PROBE.astype(np.float32)), np.float64)
    except Exception:  # noqa: BLE001 — a callable that cannot take an array
        return -1
    if y.shape != _PROBE.shape or not np.all(np.isfinite(y)):
        return -1
    for fn in (swish, relu, tanh, sigmoid, gelu, softplus, elu, leaky_relu):
        ref = np.asarray(fn(_PROBE), np.float64)
        if np.all(np.abs(y - ref) <= 1e-6 * np.maximum(1.0, np.abs(ref))):
            return fn.zf_act
    return -1


def act_code(act: Union[str, Callable]) -> int:
    """ZF_ACT_* of an activation: a function of this module, a name, a
    callable with one of the implemented names, or any callable that
    computes one of them (found by evaluating it, ``_probe``);
    NotImplementedError otherwise."""
    code = getattr(act, "zf_act", None)
    if code is not None:
        return int(code)
    name = act if isinstance(act, str) else getattr(act, "__name__", None)
    if name in _BY_NAME:
        return _BY_NAME[name]
    if callable(act):
        code = _probe(act)
        if code >= 0:
            return code
    raise NotImplementedError(
        f"activation {act!r} has no HIP implementation and computes none of the implemented ones "
        f"({', '.join(sorted(_BY_NAME))})")


def act_name(code: int) -> str:
    return _NAMES[int(code)]
