"""The Flow class — drop-in for ``zenflow.Flow`` (reference: src/zenflow/flow.py)."""

from __future__ import annotations

from typing import Any, Dict, Optional, Union

import numpy as np

from . import _lib as L
from .bijectors import Bijector, Chain, _has_stats, _prep_c
from .distributions import Beta, Distribution
from .engine import Program, cached_program
from .module import Module, scope_for
from .random import PRNGKey, key_to_seed

__all__ = ["Flow", "BoundFlow"]


class Flow(Module):
    """A conditional normalizing flow (flow.py:16-20): ``bijector`` maps data to
    the latent space, ``latent`` (default ``Beta()``) scores it."""

    def __init__(self, bijector: Bijector, latent: Optional[Distribution] = None):
        self.bijector = bijector
        self.latent = latent if latent is not None else Beta()

    # -- FLAX-style methods ----------------------------------------------------
    def __call__(self, x, c=None, *, train: bool = False):
        """log_prob of the samples (flow.py:22-48); NaN -> -inf."""
        scope = scope_for(self)
        if scope.initializing:  # inside an outer module's init: create variables only
            shape = np.shape(x) if not isinstance(x, L.DeviceArray) else x.shape
            if len(shape) != 2:
                raise ValueError(f"x must be 2-D (N, D), got {shape}")
            from .bijectors import _c_dims

            scope.init_module(self, int(shape[1]), _c_dims(c))
            return np.zeros(shape[0], np.float32)
        xd, x_dev = L.as_device(x)
        if xd.ndim != 2:
            raise ValueError(f"x must be 2-D (N, D), got {xd.shape}")
        cd, _ = _prep_c(c)
        if self.latent._dim is None:
            self.latent._dim = xd.shape[1]
        prog = self._program(scope.variables, xd.shape[1], 0 if cd is None else cd.shape[1], cached=not train)
        if train:
            update = "batch_stats" in scope.mutable
            if not update and _has_stats(self.bijector):
                raise RuntimeError("train=True updates batch_stats; pass mutable=['batch_stats']")
            stats = scope.collection("batch_stats").get("bijector", {})
            z, ld, new = prog.train_forward(xd, cd, stats, update)
            n = len(prog.ops)
            lp = prog.log_prob(z, cd, op_begin=n, op_end=n, ld_in=ld)
            if update:
                scope.updates["batch_stats"] = {"bijector": new} if new else {}
        else:
            lp = prog.log_prob(xd, cd)
        return lp if x_dev else lp.numpy()

    def sample(self, conditions_or_size: Union[Any, int], *, seed: int = 0):
        """Samples from the learned distribution (flow.py:50-78): latent draw,
        then the bijector inverse on the GPU."""
        scope = scope_for(self)
        if isinstance(conditions_or_size, (int, np.integer)):
            size, c = int(conditions_or_size), None
        else:
            c = conditions_or_size
            size = c.shape[0]
        if self.latent.dim is None:
            raise ValueError("latent dim unknown: call log_prob (or init) first")
        if scope.initializing:
            return np.zeros((size, self.latent.dim), np.float32)
        cd, c_dev = _prep_c(c)
        if cd is not None and cd.shape[0] != size:
            raise ValueError("conditions must have one row per sample")
        prog = self._program(scope.variables, self.latent.dim, 0 if cd is None else cd.shape[1])
        x = prog.sample(size, key_to_seed(PRNGKey(seed)), cd)
        return x if c_dev else x.numpy()

    def _steps(self, x, c=None, *, inverse: bool = False):
        """Per-bijector intermediates (flow.py:80-95), one segment launch each."""
        if not isinstance(self.bijector, Chain):
            raise ValueError("only for Chain bijector")
        scope = scope_for(self)
        xd, _ = L.as_device(x)
        cd, _ = _prep_c(c)
        prog = self._program(scope.variables, xd.shape[1], 0 if cd is None else cd.shape[1])
        from .engine import flatten

        bounds, k = [], 0
        for b in self.bijector:
            n = len(flatten(b))
            bounds.append((k, k + n))
            k += n
        results = []
        if inverse:
            for (b0, b1) in reversed(bounds):
                xd = prog.inverse(xd, cd, b0, b1)
                results.append(xd.numpy())
        else:
            for (b0, b1) in bounds:
                xd, _ = prog.forward(xd, cd, b0, b1)
                results.append(xd.numpy())
        return results

    # -- helpers ----------------------------------------------------------------
    def _program(self, variables, D, C, cached: bool = True) -> Program:
        """The device program for these variables.  Eval-mode programs are
        cached per (content digest of the variables, D, C, latent), so repeated
        ``apply(variables, x)`` calls pack and upload the weights once; a
        digest (xxh3 over every leaf's bytes, ~0.1 ms/MB) rather than object
        identity, because numpy leaves can be changed in place.  Train-mode
        calls write batch statistics into their program and never share it."""
        sub = {k: (v or {}).get("bijector", {}) for k, v in (variables or {}).items()}
        return cached_program(self, self.bijector, sub, D, C, self.latent, cached)

    def _init_variables(self, gen, D, C, params, stats):
        p: Dict = {}
        s: Dict = {}
        self.bijector._init_variables(gen, D, C, p, s)
        if p:
            params["bijector"] = p
        if s:
            stats["bijector"] = s

    def _on_init(self, D, C):
        if self.latent._dim is None:  # Distribution.log_prob latches dim (distributions.py:31-33)
            self.latent._dim = D

    def bind(self, variables: Dict[str, Any], dim: int, cond_dim: int = 0) -> "BoundFlow":
        """Device-resident flow for repeated calls (weights packed once)."""
        if self.latent._dim is None:
            self.latent._dim = dim
        return BoundFlow(self._program(variables, dim, cond_dim))


class BoundFlow:
    """A Flow bound to variables, weights resident in HBM; device-in/device-out."""

    def __init__(self, program: Program):
        self.program = program

    def log_prob(self, x: L.DeviceArray, c: Optional[L.DeviceArray] = None, out=None, nll_sum=None):
        return self.program.log_prob(x, c, out=out, nll_sum=nll_sum)

    def inverse(self, z: L.DeviceArray, c: Optional[L.DeviceArray] = None, out=None):
        return self.program.inverse(z, c, out=out)

    def forward(self, x: L.DeviceArray, c: Optional[L.DeviceArray] = None):
        return self.program.forward(x, c)
