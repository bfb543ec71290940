"""Bijectors of conditional normalizing flows — MI355X-native drop-in for
``zenflow.bijectors`` (reference: src/zenflow/bijectors.py).

Same classes, fields, defaults, errors and FLAX-style ``init``/``apply``
protocol as the reference; the transforms run as one fused HIP kernel over the
whole chain (see ``engine.Program`` and zenflow_amd/csrc/zf_flow.hip)."""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Callable, Dict, Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib as L
from .engine import Program, cached_program
from .module import Module, lecun_normal, scope_for

__all__ = [
    "Bijector",
    "ShiftBounds",
    "Roll",
    "NeuralSplineCoupling",
    "Chain",
    "chain",
    "rolling_spline_coupling",
]


from .activations import act_code, act_name, swish  # noqa: E402  (flax.linen.swish, the reference default)


def _c_dims(c) -> int:
    if c is None:
        return 0
    shape = np.shape(c) if not isinstance(c, L.DeviceArray) else c.shape
    return 1 if len(shape) == 1 else int(shape[1])


def _prep_c(c):
    """flow._normalize_c (flow.py:98-101) + upload."""
    if c is None:
        return None, False
    if isinstance(c, L.DeviceArray):
        if c.ndim == 1:
            raise ValueError("pass a 2-D (N, C) DeviceArray for c")
        return c, True
    a = np.asarray(c, dtype=np.float32)
    if a.ndim == 1:
        a = a.reshape(-1, 1)
    return L.DeviceArray.from_numpy(a), False


def _run_forward(module, x, c, train):
    """Shared __call__ of every bijector: one program over this module's chain."""
    scope = scope_for(module)
    if scope.initializing:  # inside an outer module's init: create variables only
        shape = np.shape(x) if not isinstance(x, L.DeviceArray) else x.shape
        scope.init_module(module, int(shape[1]), _c_dims(c))
        return np.array(x, np.float32, copy=True), np.zeros(shape[0], np.float32)
    xd, x_dev = L.as_device(x)
    if xd.ndim != 2:
        raise ValueError(f"x must be 2-D (N, D), got shape {xd.shape}")
    cd, _ = _prep_c(c)
    D = xd.shape[1]
    Cd = 0 if cd is None else cd.shape[1]
    prog = cached_program(module, module, scope.variables, D, Cd, cached=not train)
    if train:
        update = "batch_stats" in scope.mutable
        if not update and _has_stats(module):
            raise RuntimeError(
                "train=True updates batch_stats; pass mutable=['batch_stats'] (flax raises "
                "ModifyScopeVariableError here too)")
        y, ld, new_stats = prog.train_forward(xd, cd, scope.collection("batch_stats"), update)
        if update:
            scope.updates["batch_stats"] = new_stats
    else:
        y, ld = prog.forward(xd, cd)
    if x_dev:
        return y, ld
    return y.numpy(), ld.numpy()


def _run_inverse(module, x, c):
    scope = scope_for(module)
    if scope.initializing:
        return np.array(x, np.float32, copy=True)
    xd, x_dev = L.as_device(x)
    if xd.ndim != 2:
        raise ValueError(f"x must be 2-D (N, D), got shape {xd.shape}")
    cd, _ = _prep_c(c)
    prog = cached_program(module, module, scope.variables, xd.shape[1], 0 if cd is None else cd.shape[1])
    out = prog.inverse(xd, cd)
    return out if x_dev else out.numpy()


def _has_stats(module) -> bool:
    from .engine import flatten

    return any(op.kind in (L.ZF_OP_SHIFT_BOUNDS, L.ZF_OP_NSC) for op in flatten(module))


class Bijector(Module, ABC):
    """Bijector base class (bijectors.py:28-87).

    ``__call__(x, c=None, train=False) -> (y, log_det)`` transforms target
    samples towards the base distribution; ``inverse(x, c=None) -> x`` maps
    base samples back."""

    @abstractmethod
    def __call__(self, x, c=None, train: bool = False):
        raise NotImplementedError

    @abstractmethod
    def inverse(self, x, c=None):
        raise NotImplementedError


class Chain(Bijector, Sequence):
    """Chain of bijectors (bijectors.py:90-124): forward in order accumulating
    log-dets, inverse in reverse order."""

    def __init__(self, bijectors: Sequence[Bijector]):
        self.bijectors = tuple(bijectors)

    def __call__(self, x, c=None, train: bool = False):
        return _run_forward(self, x, c, train)

    def inverse(self, x, c=None):
        return _run_inverse(self, x, c)

    def __getitem__(self, idx: Union[int, slice]):
        return self.bijectors[idx]

    def __len__(self):
        return len(self.bijectors)

    def _init_variables(self, gen, D, C, params, stats):
        for i, b in enumerate(self.bijectors):
            p: Dict = {}
            s: Dict = {}
            b._init_variables(gen, D, C, p, s)
            if p:
                params[f"bijectors_{i}"] = p
            if s:
                stats[f"bijectors_{i}"] = s

    def __repr__(self):
        return f"Chain({list(self.bijectors)!r})"


def chain(*bijectors):
    """bijectors.py:127-129."""
    return Chain(bijectors)


class ShiftBounds(Bijector):
    """Shift values into the unit hypercube (bijectors.py:132-273).

    Eval mode uses the stored per-dim min/max (``batch_stats/xmin_i, xmax_i``);
    ``train=True`` widens them to the batch range plus ``margin``.  ``bounds``
    entries ``(i, a, b)`` fix both ends (affine) or one end (log transform)."""

    def __init__(self, margin: float = 0.1,
                 bounds: Sequence[Tuple[int, Optional[float], Optional[float]]] = ()):
        # bijectors.py:155-161 (flax runs setup lazily; the check is the same)
        if margin < 0:
            raise ValueError(f"margin must be positive (margin={margin})")
        if margin >= 1.0:
            raise ValueError(f"margin must be less than 1 (margin={margin})")
        self.margin = margin
        self.bounds = tuple(bounds)

    def __call__(self, x, c=None, train: bool = False):
        return _run_forward(self, x, c, train)

    def inverse(self, z, c=None):
        return _run_inverse(self, z, c)

    def _validate(self, D):
        from .engine import _is_set

        for i, a, b in self.bounds:  # bijectors.py:167-174
            if i >= D:
                raise ValueError(f"index {i} is out of bounds")
            if _is_set(a) and _is_set(b) and b < a:
                raise ValueError("upper bound must be larger than lower bound")

    def _init_variables(self, gen, D, C, params, stats):
        self._validate(D)
        from .engine import _is_set

        bounds = {int(i): (a, b) for (i, a, b) in self.bounds}
        for i in range(D):
            a, b = bounds.get(i, (None, None))
            if _is_set(a) and _is_set(b):
                continue
            stats[f"xmin_{i}"] = np.full(1, np.inf, np.float32)   # :243-245
            stats[f"xmax_{i}"] = np.full(1, -np.inf, np.float32)  # :246-248

    def __repr__(self):
        return f"ShiftBounds(margin={self.margin}, bounds={self.bounds})"


class Roll(Bijector):
    """Roll inputs along the last axis (bijectors.py:276-297); in the fused
    kernel this is an index rotation, no data moves."""

    def __init__(self, shift: int = 1):
        self.shift = int(shift)

    def __call__(self, x, c=None, train: bool = False):
        return _run_forward(self, x, c, train)

    def inverse(self, x, c=None):
        return _run_inverse(self, x, c)

    def __repr__(self):
        return f"Roll(shift={self.shift})"


class NeuralSplineCoupling(Bijector):
    """Rational-quadratic spline coupling (bijectors.py:300-371).

    The upper half ``xc = x[:, D//2:]`` (plus conditions ``c``) drives a
    conditioner MLP ``BatchNorm -> [Dense(w), act]* -> Dense(dt*(3K-1))``
    whose outputs parametrise a monotone RQ spline on ``xt = x[:, :D//2]``.
    The MLP runs on MFMA with activations resident in registers; the
    spline + log-det run in the same kernel's epilogue.  ``act``: swish (the
    reference default) or another activation of ``zenflow_amd.activations``
    (by function, name, or a callable of that name such as ``nn.relu``)."""

    def __init__(self, knots: int = 16, layers: Sequence[int] = (128, 128),
                 act: Callable = swish):
        self.act_code = act_code(act)  # NotImplementedError for an activation the kernels lack
        self.knots = int(knots)
        self.layers = tuple(int(w) for w in layers)
        self.act = act

    @staticmethod
    def _split(x):
        """bijectors.py:321-327."""
        x_dim = x.shape[1]
        x_split = x_dim // 2
        assert x_split > 0 and x_split < x_dim
        return x[:, :x_split], x[:, x_split:]

    def __call__(self, x, c=None, train: bool = False):
        return _run_forward(self, x, c, train)

    def inverse(self, y, c=None):
        return _run_inverse(self, y, c)

    def _init_variables(self, gen, D, C, params, stats):
        dt = D // 2
        if not (0 < dt < D):
            raise AssertionError("NeuralSplineCoupling needs D >= 2")  # :326
        DC = D - dt + C
        params["BatchNorm_0"] = {"bias": np.zeros(DC, np.float32), "scale": np.ones(DC, np.float32)}
        stats["BatchNorm_0"] = {"mean": np.zeros(DC, np.float32), "var": np.ones(DC, np.float32)}
        fan_in = DC
        widths = list(self.layers) + [dt * (3 * self.knots - 1)]
        for l, w in enumerate(widths):
            params[f"Dense_{l}"] = {
                "kernel": lecun_normal(gen, fan_in, w),
                "bias": np.zeros(w, np.float32),
            }
            fan_in = w

    def __repr__(self):
        a = "" if self.act_code == L.ZF_ACT_SWISH else f", act={act_name(self.act_code)}"
        return f"NeuralSplineCoupling(knots={self.knots}, layers={self.layers}{a})"


def rolling_spline_coupling(
    dim: int,
    knots: int = 16,
    layers: Sequence[int] = (128, 128),
    margin: Optional[float] = None,
    bounds: Sequence[Tuple[int, Optional[float], Optional[float]]] = (),
    preprocessing: Optional[Sequence[Bijector]] = None,
) -> Chain:
    """bijectors.py:374-423: ShiftBounds, then (NSC, Roll) x (dim-1), then NSC."""
    if dim < 2:
        raise ValueError("dim must be at least 2")
    if preprocessing is not None:
        bijectors = list(preprocessing)
    else:
        kwargs: Dict = {}
        if margin is not None:
            kwargs["margin"] = margin
        if bounds is not None:
            kwargs["bounds"] = bounds
        bijectors = [ShiftBounds(**kwargs)]
    for _ in range(dim - 1):
        bijectors.append(NeuralSplineCoupling(knots=knots, layers=layers))
        bijectors.append(Roll())
    bijectors.append(NeuralSplineCoupling(knots=knots, layers=layers))
    return Chain(bijectors)
