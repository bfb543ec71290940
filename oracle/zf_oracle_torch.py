"""GRADIENT ORACLE for zenflow training — TEST INFRASTRUCTURE ONLY.

``jax.grad`` of the reference's ``loss_fn`` (src/zenflow/train.py:64-72:
``-mean(Flow.__call__(x, c, train=True))``) is not available offline (no
JAX).  This module restates that train-mode loss function by function after
``oracle/zf_oracle.py`` (the NumPy oracle pinned by the reference's KATs) in
PyTorch ops, so that reverse-mode autograd in float64 yields the exact
gradient of the same arithmetic — the yardstick for the GPU trainer's
hand-written reverse kernels (``zf_train.hip``), compared per parameter in
``tests/test_gpu_train.py``.  ``tests/test_oracle_torch.py`` checks that this
restatement's forward equals the NumPy oracle's (fp64, 1e-12).

Only the tests import this module; the product (``zenflow_amd``) never does.
Scope: the chains the trainer supports (ShiftBounds as the first bijector,
NeuralSplineCoupling, Roll; Normal / Beta / TruncatedNormal / Uniform
latents)."""

from __future__ import annotations

import math
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

EPS = 1e-5  # utils.py:15


def _squareplus(x, b=4.0):
    """utils.py:18-20."""
    return 0.5 * (x + torch.sqrt(x * x + b))


def _softmax_with_threshold(x, threshold):
    """utils.py:23-34 (sum in sequential order, as the NumPy oracle)."""
    x = _squareplus(x)
    n = x.shape[-1]
    c = float(threshold) / (1 - n * float(threshold))
    s = x[..., 0]
    for j in range(1, n):
        s = s + x[..., j]
    return (x / s[..., None] + c) / (1 + c * n)


def _knots(d):
    """utils.py:235-241."""
    return torch.cat([torch.zeros_like(d[..., :1]), torch.cumsum(d, dim=-1)], dim=-1)


def _take(arr, idx):
    """jnp.take_along_axis(..., mode='fill'): NaN past the end (utils.py:225-232)."""
    k = arr.shape[-1]
    ok = idx < k
    out = torch.gather(arr, -1, torch.where(ok, idx, torch.zeros_like(idx)))[..., 0]
    return torch.where(ok[..., 0], out, torch.full_like(out, float("nan")))


def rqs_forward(x, dx, dy, sl):
    """utils.py:65-141 (forward spline + per-row log-det summed in dim order)."""
    xk, yk = _knots(dx), _knots(dy)
    one = torch.ones_like(sl[..., :1])
    dk = torch.cat([one, sl, one], dim=-1)
    sk = dy / dx
    oob = (x < 0) | (x >= 1)
    idx = torch.sum((xk <= x[..., None]).to(torch.int64), dim=-1, keepdim=True) - 1
    idx = torch.clamp(idx, 0, xk.shape[-1] - 1)
    xk_i, yk_i, dx_i, dy_i = _take(xk, idx), _take(yk, idx), _take(dx, idx), _take(dy, idx)
    d_i, d_i1, s_i = _take(dk, idx), _take(dk, idx + 1), _take(sk, idx)
    z = (x - xk_i) / dx_i
    z = torch.clamp(z, EPS, 1 - EPS)
    az = 1 - z
    num = dy_i * z * (s_i * z + d_i * az)
    den = s_i + (d_i1 + d_i - 2 * s_i) * z * az
    y = torch.where(oob, x, yk_i + num / (den + EPS))
    num2 = z * (d_i1 * z + 2 * s_i * az) + d_i * az * az
    ld = 2 * torch.log(s_i + EPS) + torch.log(num2 + EPS) - 2 * torch.log(den + EPS)
    ld = torch.where(oob, torch.zeros_like(ld), ld)
    s = ld[..., 0]
    for j in range(1, ld.shape[-1]):
        s = s + ld[..., j]
    return y, s


def _unit_interval(x, st, i, margin):
    """bijectors.py:242-273, train mode (batch min/max, merged with the stored)."""
    dt = x.dtype
    ra_min = float(np.asarray(st.get(f"xmin_{i}", [np.inf]), np.float64).reshape(-1)[0])
    ra_max = float(np.asarray(st.get(f"xmax_{i}", [-np.inf]), np.float64).reshape(-1)[0])
    xmin, xmax = x.min(), x.max()
    delta = 0.5 * (xmax - xmin) * margin
    xmin = torch.minimum(torch.tensor(ra_min, dtype=dt), xmin - delta)
    xmax = torch.maximum(torch.tensor(ra_max, dtype=dt), xmax + delta)
    mul = 1 / (xmax - xmin)
    return torch.clamp((x - xmin) * mul, 0, 1), torch.log(mul)


def _safe_log(x):
    """bijectors.py:430-431."""
    return torch.log(x + torch.finfo(x.dtype).tiny)


def shift_bounds(spec, st, x):
    """bijectors.py:163-208, train mode."""
    bounds = {int(i): (a, b) for (i, a, b) in spec.get("bounds", ())}
    margin = spec.get("margin", 0.1)
    cols, ld = [], torch.zeros(x.shape[0], dtype=x.dtype)
    isset = lambda v: v is not None and np.isfinite(v)  # noqa: E731  bijectors.py:426-427
    for i in range(x.shape[1]):
        xi = x[:, i]
        a, b = bounds.get(i, (None, None))
        if isset(a) and isset(b):
            mul = 1.0 / (float(b) - float(a))
            zi, li = (xi - float(a)) * mul, torch.full_like(xi, math.log(mul))
        elif isset(a) or isset(b):
            ti = _safe_log(xi - float(a)) if isset(a) else _safe_log(float(b) - xi)
            zi, li = _unit_interval(ti, st, i, margin)
            li = li - ti
        else:
            zi, li = _unit_interval(xi, st, i, margin)
        cols.append(zi)
        ld = ld + li
    return torch.stack(cols, dim=1), ld


def _act(name, x):
    """bijectors.py:319 ``act`` (jax.nn definitions; as zf_oracle.activation)."""
    if name in ("swish", "silu"):
        return x * torch.sigmoid(x)
    if name == "relu":
        return torch.clamp(x, min=0)
    if name == "tanh":
        return torch.tanh(x)
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name == "gelu":
        return 0.5 * x * (1 + torch.tanh(math.sqrt(2 / math.pi) * (x + 0.044715 * x * x * x)))
    if name == "softplus":
        return torch.logaddexp(x, torch.zeros_like(x))
    if name == "elu":
        return torch.where(x > 0, x, torch.expm1(torch.clamp(x, max=0)))
    if name == "leaky_relu":
        return torch.where(x >= 0, x, 0.01 * x)
    raise ValueError(name)


def nsc(spec, p, x, c):
    """bijectors.py:329-365, train mode: BatchNorm on batch statistics
    (flax.linen.BatchNorm: var = max(0, mean(u^2) - mean(u)^2), eps 1e-5)."""
    K = spec.get("knots", 16)
    D = x.shape[1]
    dt_ = D // 2
    xt, xc = x[:, :dt_], x[:, dt_:]
    u = torch.cat([xc, c], dim=1) if c is not None else xc
    mean = u.mean(dim=0)
    var = torch.clamp((u * u).mean(dim=0) - mean * mean, min=0)
    u = (u - mean) / torch.sqrt(var + 1e-5) * p["BatchNorm_0"]["scale"] + p["BatchNorm_0"]["bias"]
    nl = len(spec.get("layers", (128, 128)))
    for li in range(nl):
        d = p[f"Dense_{li}"]
        u = _act(spec.get("act", "swish"), u @ d["kernel"] + d["bias"])
    d = p[f"Dense_{nl}"]
    q = (u @ d["kernel"] + d["bias"]).reshape(x.shape[0], dt_, 3 * K - 1)
    dx = _softmax_with_threshold(q[..., :K], EPS)
    dy = _softmax_with_threshold(q[..., K : 2 * K], EPS)
    sl = _squareplus(q[..., 2 * K :])
    yt, ld = rqs_forward(xt, dx, dy, sl)
    return torch.cat([yt, xc], dim=1), ld


def latent_log_prob(latent, z):
    """distributions.py (jax.scipy.stats forms, as zf_oracle.latent_log_prob)."""
    t = latent["type"]
    if t in ("normal", "truncated_normal"):
        lp = (math.log(2 * math.pi * 0.01) + (z - 0.5) ** 2 / 0.01) / -2
        if t == "truncated_normal":
            nd = 0.5 * math.erfc(5.0 / math.sqrt(2.0))
            lp = lp - math.log1p(-nd - nd)
            xs = (z - 0.5) / 0.1
            lp = torch.where((xs < -5) | (xs > 5), torch.full_like(lp, -math.inf), lp)
    elif t == "beta":
        a = float(latent.get("peakness", 12.0))
        const = -(math.lgamma(a) * 2 - math.lgamma(2 * a))
        lp = const + (a - 1) * torch.log(z) + (a - 1) * torch.log1p(-z)
        lp = torch.where((z > 1) | (z < 0), torch.full_like(lp, -math.inf), lp)
    elif t == "uniform":
        lp = torch.where((z > 1) | (z < 0), torch.full_like(z, -math.inf), torch.zeros_like(z))
    else:
        raise ValueError(t)
    s = lp[:, 0]
    for j in range(1, lp.shape[1]):
        s = s + lp[:, j]
    return s


def _tree(tree, dtype, grad):
    if isinstance(tree, dict):
        return {k: _tree(v, dtype, grad) for k, v in tree.items()}
    return torch.tensor(np.asarray(tree, np.float64), dtype=dtype, requires_grad=grad)


def _grads(tree):
    if isinstance(tree, dict):
        return {k: _grads(v) for k, v in tree.items()}
    return np.zeros(tuple(tree.shape)) if tree.grad is None else tree.grad.detach().numpy().astype(np.float64)


def train_loss_and_grad(model: Dict[str, Any], variables: Dict[str, Any], x, c=None,
                        dtype=torch.float64) -> Tuple[float, Dict[str, Any]]:
    """(loss_fn value, d loss / d params in the FLAX ``params`` layout) of
    train.py:64-72 on one batch: -mean of the train-mode log_prob
    (flow.py:22-48; flow.py:47's nan_to_num is the identity on the finite
    rows a training batch has)."""
    params = _tree(variables["params"]["bijector"], dtype, True)
    stats = variables.get("batch_stats", {}).get("bijector", {})
    xt = torch.tensor(np.asarray(x, np.float64), dtype=dtype)
    ct = None
    if c is not None:
        c = np.asarray(c, np.float64)
        ct = torch.tensor(c.reshape(-1, 1) if c.ndim == 1 else c, dtype=dtype)
    ld = torch.zeros(xt.shape[0], dtype=dtype)
    h = xt
    for i, b in enumerate(model["bijector"]["bijectors"]):
        key = f"bijectors_{i}"
        if b["type"] == "shift_bounds":
            h, l = shift_bounds(b, stats.get(key, {}), h)
        elif b["type"] == "roll":
            h, l = torch.roll(h, b.get("shift", 1), dims=-1), None
        elif b["type"] == "nsc":
            h, l = nsc(b, params[key], h, ct)
        else:
            raise ValueError(b["type"])
        if l is not None:
            ld = ld + l
    lp = latent_log_prob(model["latent"], h) + ld
    loss = -lp.mean()
    loss.backward()
    return float(loss.detach()), {"bijector": _grads(params)}
