"""Activations for ``NeuralSplineCoupling(act=...)`` (bijectors.py:319: any
callable, default ``flax.linen.swish``).

The kernels evaluate the activation themselves, so ``act`` must be one they
implement: these functions (numpy forms of the flax.linen / jax.nn
functions of the same names, usable on host arrays), a name string, or any
callable with one of these ``__name__``s (e.g. ``flax.linen.relu``).  The
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


def act_code(act: Union[str, Callable]) -> int:
    """ZF_ACT_* of an activation (function of this module, name, or a callable
    with one of the implemented names); NotImplementedError otherwise."""
    code = getattr(act, "zf_act", None)
    if code is not None:
        return int(code)
    name = act if isinstance(act, str) else getattr(act, "__name__", None)
    if name in _BY_NAME:
        return _BY_NAME[name]
    raise NotImplementedError(
        f"activation {act!r} has no HIP implementation (implemented: {', '.join(sorted(_BY_NAME))})")


def act_name(code: int) -> str:
    return _NAMES[int(code)]
