"""CPU ORACLE for the zenflow neural-spline-flow hot path — TEST INFRASTRUCTURE ONLY.

This module is a plain-NumPy restatement of the reference algorithm
(HDembinski/zenflow @ 2025-02-04, a JAX/FLAX library).  It exists so that the
tests, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``
can CHECK the MI355X product path (``zenflow_amd``, HIP kernels behind a C ABI).
The product never imports, links or calls anything under ``oracle/``.

Parity status:

* The reference cannot be imported here: ``jax``/``jaxlib``/``flax``/``optax``
  are absent (ordinary ``ModuleNotFoundError``, no network).  So this oracle
  is a restatement, pinned by every known-answer test (KAT) the reference's own
  test suite holds that is reproducible without JAX (``tests/test_oracle_kats.py``
  restates them verbatim: ``tests/test_utils.py``, ``tests/test_bijectors.py``
  ShiftBounds/Roll/Chain KATs, ``tests/test_distributions.py`` Normal/Beta vs
  scipy).
* The conditioner MLP (FLAX ``BatchNorm``/``Dense``/``swish``) and the
  ``jnp.take_along_axis`` out-of-range behaviour are third-party arithmetic no
  reference test pins numerically: **parity unpinned** there beyond the
  invertibility / Jacobian properties the reference tests check.

Every function runs in the dtype of its inputs: ``np.float32`` reproduces the
reference's fp32 semantics (JAX x64 is off by default), ``np.float64`` is the
error yardstick.  Reductions over knots/dims are written as explicit sequential
loops so the summation order is defined (the reference's XLA order is not).
"""

from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

# utils.py:15
EPS = 1e-5

# Optional rounding-noise injection (fp64 runs only): a Generator and a relative
# amplitude.  Used by `row_sensitivity` to estimate how much each sample's
# log_prob moves under fp32-sized rounding perturbations (its conditioning).
_NOISE = {"rng": None, "eps": 0.0}


def _perturb(a):
    rng, eps = _NOISE["rng"], _NOISE["eps"]
    if rng is None or eps == 0.0:
        return a
    a = np.asarray(a)
    with np.errstate(all="ignore"):
        return a * (1 + eps * rng.standard_normal(a.shape))


def _c(dtype, v):
    return np.asarray(v, dtype=dtype)


# ---------------------------------------------------------------------------
# L1 spline numerics — src/zenflow/utils.py
# ---------------------------------------------------------------------------


def squareplus(x, b=4.0):
    """utils.py:18-20 — 0.5 * (x + sqrt(x^2 + b))."""
    x = np.asarray(x)
    dt = x.dtype
    return _c(dt, 0.5) * (x + np.sqrt(np.square(x) + _c(dt, b)))


def _seqsum_last(x):
    """Sum over the last axis in sequential order (defined order)."""
    acc = np.zeros(x.shape[:-1], dtype=x.dtype)
    for j in range(x.shape[-1]):
        acc = acc + x[..., j]
    return acc


def softmax_with_threshold(x, threshold=0.0):
    """utils.py:23-34 — squareplus 'softmax' whose smallest value is threshold."""
    x = np.asarray(x)
    dt = x.dtype
    x = squareplus(x)
    n = x.shape[-1]
    # threshold and n are Python scalars: c and 1 + c*n are float64, rounded on use
    c = float(threshold) / (1 - n * float(threshold))
    xs = _seqsum_last(x)[..., None]
    return (x / xs + _c(dt, c)) / _c(dt, 1 + c * n)


def normalize_spline_params(dx, dy, sl):
    """utils.py:37-62."""
    dx = softmax_with_threshold(dx, EPS)
    dy = softmax_with_threshold(dy, EPS)
    sl = squareplus(sl)
    return dx, dy, sl


def knots(dx):
    """utils.py:235-241 — [0, cumsum(dx)] (np.cumsum is sequential)."""
    dx = np.asarray(dx)
    cs = np.cumsum(dx, axis=-1, dtype=dx.dtype)
    pad = np.zeros(dx.shape[:-1] + (1,), dtype=dx.dtype)
    return np.concatenate([pad, cs], axis=-1)


def index(x, xk):
    """utils.py:244-250 — compare-count bin index, clipped to [0, len(xk)-1]."""
    x = np.asarray(x)
    oob = (x < 0) | (x >= 1)
    idx = np.sum(xk <= x[..., None], axis=-1)[..., None] - 1
    idx = np.clip(idx, 0, xk.shape[-1] - 1)
    return idx, oob


def _take_fill(arr, idx):
    """``jnp.take_along_axis(arr, idx, -1)[..., 0]`` with JAX's default
    ``mode="fill"``: an out-of-range index yields NaN."""
    k = arr.shape[-1]
    ok = idx < k
    safe = np.where(ok, idx, 0)
    out = np.take_along_axis(arr, safe, -1)[..., 0]
    return np.where(ok[..., 0], out, np.asarray(np.nan, dtype=arr.dtype))


# Rows whose spline input lies in the last-knot sliver band [1 - SLIVER, 1):
# there the fp32 knot sum (which can end slightly below 1) decides whether
# idx == K (fill-mode NaN, Appendix A.4), so two fp32 evaluations with
# different summation orders may legitimately disagree on finiteness.
SLIVER = 1e-5
_SLIVER_LOG: Dict[str, Any] = {"rows": None}


def sliver_rows(fn, *args, **kwargs):
    """Run ``fn`` and return (its result, bool mask of rows that touched the
    sliver band in any coupling).  Rows are axis 0 of every spline input."""
    _SLIVER_LOG["rows"] = None
    _SLIVER_LOG["on"] = True
    try:
        out = fn(*args, **kwargs)
    finally:
        _SLIVER_LOG["on"] = False
    rows = _SLIVER_LOG["rows"]
    return out, rows


def compute_rqs_input(x, dx, dy, slope, forward):
    """utils.py:205-232."""
    dt = dx.dtype
    xk = knots(dx)
    yk = knots(dy)
    one = np.ones(slope.shape[:-1] + (1,), dtype=dt)
    dk = np.concatenate([one, slope, one], axis=-1)  # :211-216
    sk = dy / dx  # :218
    idx, oob = index(x, xk if forward else yk)
    if _SLIVER_LOG.get("on"):
        band = (x >= 1 - SLIVER) & (x < 1)
        band = band.reshape(band.shape[0], -1).any(axis=1)
        prev = _SLIVER_LOG["rows"]
        _SLIVER_LOG["rows"] = band if prev is None else (prev | band)
    return (
        _take_fill(xk, idx),
        _take_fill(yk, idx),
        _take_fill(dx, idx),
        _take_fill(dy, idx),
        _take_fill(dk, idx),
        _take_fill(dk, idx + 1),
        _take_fill(sk, idx),
        oob,
    )


def rqs_forward(x, dx, dy, slope):
    """utils.py:65-141 — RQ spline forward; returns (y (M,N), log_det (M,))."""
    x = np.asarray(x)
    dt = x.dtype
    dx, dy, slope = (np.asarray(a, dtype=dt) for a in (dx, dy, slope))
    xk, yk, dxk, dyk, dk, dkp1, sk, oob = compute_rqs_input(x, dx, dy, slope, True)
    eps = _c(dt, EPS)
    one, two = _c(dt, 1), _c(dt, 2)
    with np.errstate(all="ignore"):
        z = (x - xk) / dxk  # :122
        z = np.clip(z, eps, _c(dt, 1 - EPS))  # :123 (1 - EPS is a Python float)
        az = one - z
        num = dyk * z * (sk * z + dk * az)  # :125
        den = sk + (dkp1 + dk - two * sk) * z * az  # :126
        y = yk + num / (den + eps)  # :127
        y = np.where(oob, x, y)  # :130
        num = z * (dkp1 * z + two * sk * az) + dk * az**2  # :133
        den = sk + (dkp1 + dk - two * sk) * z * az  # :134
        ld = two * np.log(sk + eps) + np.log(num + eps) - two * np.log(den + eps)
        ld = np.where(oob, _c(dt, 0), ld)  # :138
    return y, _seqsum_last(ld)  # :139


def rqs_inverse(y, dx, dy, slope):
    """utils.py:144-202 — quadratic-root inverse; returns x (M,N)."""
    y = np.asarray(y)
    dt = y.dtype
    dx, dy, slope = (np.asarray(a, dtype=dt) for a in (dx, dy, slope))
    xk, yk, dxk, dyk, dk, dkp1, sk, oob = compute_rqs_input(y, dx, dy, slope, False)
    two, four = _c(dt, 2), _c(dt, 4)
    with np.errstate(all="ignore"):
        a = dyk * (sk - dk) + (y - yk) * (dkp1 + dk - two * sk)  # :193
        b = dyk * dk - (y - yk) * (dkp1 + dk - two * sk)  # :194
        c = -sk * (y - yk)  # :195
        z = two * c / (-b - np.sqrt(b**2 - four * a * c))  # :197
        x = z * dxk + xk  # :198
        x = np.where(oob, y, x)  # :201
    return x


# ---------------------------------------------------------------------------
# Latent distributions — src/zenflow/distributions.py (jax.scipy.stats forms)
# ---------------------------------------------------------------------------


def normal_log_prob(x):
    """distributions.py:58-59, jax.scipy.stats.norm.logpdf(x, 0.5, 0.1):
    (log(2*pi*scale^2) + (x-loc)^2/scale^2) / -2, summed over the last axis."""
    x = np.asarray(x)
    dt = x.dtype
    s2 = np.square(_c(dt, 0.1))
    lognorm = np.log(_c(dt, 2 * np.pi) * s2)
    q = np.square(x - _c(dt, 0.5)) / s2
    return _seqsum_last((lognorm + q) / _c(dt, -2))


def beta_const(peakness, dtype):
    """-betaln(a, b) in ``dtype`` (computed in fp64, then rounded)."""
    a = float(peakness)
    v = math.lgamma(a) + math.lgamma(a) - math.lgamma(2 * a)
    return _c(dtype, -v)


def beta_log_prob(x, peakness=12.0):
    """distributions.py:100-104, jax.scipy.stats.beta.logpdf(x, a, a):
    -betaln(a,b) + xlogy(a-1, x) + xlog1py(b-1, -x), -inf outside [0, 1]."""
    x = np.asarray(x)
    dt = x.dtype
    am1 = _c(dt, peakness) - _c(dt, 1)
    with np.errstate(all="ignore"):
        lp = beta_const(peakness, dt) + (am1 * np.log(x) + am1 * np.log1p(-x))
        lp = np.where((x > 1) | (x < 0), _c(dt, -np.inf), lp)
    return _seqsum_last(lp)


def truncnorm_log_prob(x):
    """distributions.py:72-73, truncnorm.logpdf(x, -5, 5, loc=0.5, scale=0.1)."""
    # jax: norm.logpdf(x, loc, scale) - _log_gauss_mass(a, b), -inf where the
    # standardised x is outside [a, b]; central-case mass log1p(-ndtr(a) - ndtr(-b)).
    x = np.asarray(x)
    dt = x.dtype
    lo, hi = -5.0, 5.0
    nd = _c(dt, 0.5 * math.erfc(5.0 / math.sqrt(2.0)))
    logmass = np.log1p(-nd - nd)
    s2 = np.square(_c(dt, 0.1))
    lognorm = np.log(_c(dt, 2 * np.pi) * s2)
    q = np.square(x - _c(dt, 0.5)) / s2
    lp = (lognorm + q) / _c(dt, -2) - logmass
    xs = (x - _c(dt, 0.5)) / _c(dt, 0.1)
    lp = np.where((xs < lo) | (xs > hi), _c(dt, -np.inf), lp)
    return _seqsum_last(lp)


def uniform_log_prob(x):
    """distributions.py:122-123, uniform.logpdf(x): 0 on [0,1], -inf outside."""
    x = np.asarray(x)
    dt = x.dtype
    lp = np.where((x > 1) | (x < 0), _c(dt, -np.inf), _c(dt, 0))
    return _seqsum_last(lp)


def latent_log_prob(latent: Dict[str, Any], x):
    t = latent["type"]
    if t == "normal":
        return normal_log_prob(x)
    if t == "beta":
        return beta_log_prob(x, latent.get("peakness", 12.0))
    if t == "truncated_normal":
        return truncnorm_log_prob(x)
    if t == "uniform":
        return uniform_log_prob(x)
    raise ValueError(t)


# ---------------------------------------------------------------------------
# Bijectors — src/zenflow/bijectors.py
# ---------------------------------------------------------------------------


def _is_set(v):
    """bijectors.py:426-427."""
    return v is not None and np.isfinite(v)


def safe_log(x):
    """bijectors.py:430-431."""
    return np.log(x + np.finfo(x.dtype).smallest_normal)


def _unit_interval(x, stats, i, margin, train, dt):
    """bijectors.py:242-273 — returns (z, ld, xmin, xmax)."""
    ra_min = np.asarray(stats.get(f"xmin_{i}", np.full(1, np.inf)), dtype=dt)
    ra_max = np.asarray(stats.get(f"xmax_{i}", np.full(1, -np.inf)), dtype=dt)
    if train:
        xmin = x.min()
        xmax = x.max()
        xdelta = _c(dt, 0.5) * (xmax - xmin) * _c(dt, margin)
        xmin = xmin - xdelta
        xmax = xmax + xdelta
        xmin = np.minimum(ra_min, xmin)
        xmax = np.maximum(ra_max, xmax)
    else:
        xmin, xmax = ra_min, ra_max
    with np.errstate(all="ignore"):
        mul = _c(dt, 1) / (xmax - xmin)
        z = (x - xmin) * mul
        ld = np.log(mul)
    z = np.clip(z, _c(dt, 0), _c(dt, 1))
    return z, ld, xmin, xmax


def shift_bounds_forward(spec, stats, x, train=False, dtype=np.float32):
    """bijectors.py:163-208. Returns (z, log_det, new_stats)."""
    x = np.asarray(x)
    if x.dtype.kind in "iu":  # :178-179
        x = x.astype(np.float32)
    x = x.astype(dtype)
    dt = x.dtype
    bounds = {int(i): (a, b) for (i, a, b) in spec.get("bounds", ())}
    margin = spec.get("margin", 0.1)
    z = np.empty_like(x)
    log_det = np.zeros(x.shape[0], dt)
    new_stats = dict(stats)
    with np.errstate(all="ignore"):
        for i in range(x.shape[1]):
            xi = x[:, i]
            a, b = bounds.get(i, (None, None))
            if _is_set(a):
                if _is_set(b):
                    mul = _c(dt, 1) / (_c(dt, b) - _c(dt, a))
                    zi = (xi - _c(dt, a)) * mul
                    ld = np.log(mul)
                else:
                    ti = safe_log(xi - _c(dt, a))
                    zi, ld, lo, hi = _unit_interval(ti, stats, i, margin, train, dt)
                    new_stats[f"xmin_{i}"], new_stats[f"xmax_{i}"] = lo, hi
                    ld = ld - ti
            elif _is_set(b):
                ti = safe_log(_c(dt, b) - xi)
                zi, ld, lo, hi = _unit_interval(ti, stats, i, margin, train, dt)
                new_stats[f"xmin_{i}"], new_stats[f"xmax_{i}"] = lo, hi
                ld = ld - ti
            else:
                zi, ld, lo, hi = _unit_interval(xi, stats, i, margin, train, dt)
                new_stats[f"xmin_{i}"], new_stats[f"xmax_{i}"] = lo, hi
            z[:, i] = zi
            log_det = log_det + ld
    return z, log_det, new_stats


def shift_bounds_inverse(spec, stats, z, dtype=np.float32):
    """bijectors.py:210-240."""
    z = np.asarray(z, dtype=dtype)
    dt = z.dtype
    bounds = {int(i): (a, b) for (i, a, b) in spec.get("bounds", ())}
    x = np.empty_like(z)
    one = _c(dt, 1)
    with np.errstate(all="ignore"):
        for i in range(z.shape[1]):
            zi = z[:, i]
            a, b = bounds.get(i, (None, None))
            if _is_set(a) and _is_set(b):
                xi = zi * _c(dt, b) + (one - zi) * _c(dt, a)
            else:
                xmin = np.asarray(stats[f"xmin_{i}"], dtype=dt)
                xmax = np.asarray(stats[f"xmax_{i}"], dtype=dt)
                ti = zi * xmax + (one - zi) * xmin
                if _is_set(a):
                    xi = np.exp(ti) + _c(dt, a)
                elif _is_set(b):
                    xi = _c(dt, b) - np.exp(ti)
                else:
                    xi = ti
            x[:, i] = xi
    return x


def roll(x, shift):
    """bijectors.py:288-297 — jnp.roll along the last axis."""
    return np.roll(x, shift, axis=-1)


def swish(x):
    """flax.linen.swish = jax.nn.silu: x * sigmoid(x)."""
    with np.errstate(all="ignore"):
        return x * (np.asarray(1, x.dtype) / (np.asarray(1, x.dtype) + np.exp(-x)))


def activation(name, x):
    """The conditioner activation (bijectors.py:319 ``act``, default
    flax.linen.swish) in the dtype of ``x``: the jax.nn definitions."""
    dt = x.dtype
    with np.errstate(all="ignore"):
        if name in ("swish", "silu"):
            return swish(x)
        if name == "relu":
            return np.maximum(x, _c(dt, 0))
        if name == "tanh":
            return np.tanh(x)
        if name == "sigmoid":
            return _c(dt, 1) / (_c(dt, 1) + np.exp(-x))
        if name == "gelu":  # approximate=True (flax.linen.gelu default)
            c = _c(dt, np.sqrt(2 / np.pi))
            return _c(dt, 0.5) * x * (_c(dt, 1) + np.tanh(c * (x + _c(dt, 0.044715) * x * x * x)))
        if name == "softplus":
            return np.logaddexp(x, _c(dt, 0))
        if name == "elu":
            return np.where(x > 0, x, np.expm1(np.minimum(x, _c(dt, 0))))
        if name == "leaky_relu":
            return np.where(x >= 0, x, _c(dt, 0.01) * x)
    raise ValueError(name)


def _batchnorm(u, p, s, train, dt, momentum=0.99, eps=1e-5):
    """flax.linen.BatchNorm (bijectors.py:342): y = (u-mean)*rsqrt(var+eps)*scale+bias."""
    if train:
        mean = u.mean(axis=0, dtype=np.float64).astype(dt)
        mean2 = np.square(u).mean(axis=0, dtype=np.float64).astype(dt)
        var = np.maximum(_c(dt, 0), mean2 - np.square(mean))
        new_mean = _c(dt, momentum) * np.asarray(s["mean"], dt) + _c(dt, 1 - momentum) * mean
        new_var = _c(dt, momentum) * np.asarray(s["var"], dt) + _c(dt, 1 - momentum) * var
        new_s = {"mean": new_mean, "var": new_var}
    else:
        mean = np.asarray(s["mean"], dt)
        var = np.asarray(s["var"], dt)
        new_s = s
    mul = _c(dt, 1) / np.sqrt(var + _c(dt, eps))
    mul = mul * np.asarray(p["scale"], dt)
    y = (u - mean) * mul + np.asarray(p["bias"], dt)
    return y, new_s


def nsc_params(spec, params, stats, x, c, train, dt):
    """bijectors.py:329-357 — conditioner MLP + normalize_spline_params.

    Returns (xt, xc, dx, dy, slope, new_stats)."""
    K = spec.get("knots", 16)
    D = x.shape[1]
    split = D // 2  # :321-327
    assert 0 < split < D
    xt, xc = x[:, :split], x[:, split:]
    S = 3 * K - 1
    u = np.hstack((xc, np.asarray(c, dt))) if c is not None else xc  # :341
    u, new_bn = _batchnorm(u, params["BatchNorm_0"], stats["BatchNorm_0"], train, dt)
    nl = len(spec.get("layers", (128, 128)))
    for li in range(nl):  # :343-345
        d = params[f"Dense_{li}"]
        u = _perturb(activation(spec.get("act", "swish"), u @ np.asarray(d["kernel"], dt) + np.asarray(d["bias"], dt)))
    d = params[f"Dense_{nl}"]
    p = _perturb(u @ np.asarray(d["kernel"], dt) + np.asarray(d["bias"], dt))  # :346
    p = p.reshape((x.shape[0], split, S))  # :347
    dx, dy, sl = normalize_spline_params(p[..., :K], p[..., K : 2 * K], p[..., 2 * K :])
    return xt, xc, dx, dy, sl, {"BatchNorm_0": new_bn}


def nsc_forward(spec, params, stats, x, c, train, dt):
    """bijectors.py:359-365."""
    xt, xc, dx, dy, sl, new_stats = nsc_params(spec, params, stats, x, c, train, dt)
    yt, ld = rqs_forward(xt, dx, dy, sl)
    return np.hstack((yt, xc)), ld, new_stats


def nsc_inverse(spec, params, stats, y, c, dt):
    """bijectors.py:367-371."""
    yt, yc, dx, dy, sl, _ = nsc_params(spec, params, stats, y, c, False, dt)
    return np.hstack((rqs_inverse(yt, dx, dy, sl), yc))


def bijector_forward(spec, params, stats, x, c, train, dt):
    """Dispatch one bijector forward; returns (y, ld, new_stats)."""
    t = spec["type"]
    if t == "shift_bounds":
        return shift_bounds_forward(spec, stats or {}, x, train, dt)
    if t == "roll":
        return roll(x, spec.get("shift", 1)), np.zeros(x.shape[0], dt), stats
    if t == "nsc":
        return nsc_forward(spec, params, stats, x, c, train, dt)
    if t == "chain":
        return chain_forward(spec, params or {}, stats or {}, x, c, train, dt)
    raise ValueError(t)


def bijector_inverse(spec, params, stats, x, c, dt):
    t = spec["type"]
    if t == "shift_bounds":
        return shift_bounds_inverse(spec, stats, x, dt)
    if t == "roll":
        return roll(x, -spec.get("shift", 1))
    if t == "nsc":
        return nsc_inverse(spec, params, stats, x, c, dt)
    if t == "chain":
        return chain_inverse(spec, params or {}, stats or {}, x, c, dt)
    raise ValueError(t)


def chain_forward(spec, params, stats, x, c, train, dt):
    """bijectors.py:103-111 — sequential composition, log_det accumulated."""
    x = np.asarray(x)
    if x.dtype.kind in "iu":
        x = x.astype(np.float32)
    x = x.astype(dt)
    log_det = np.zeros(x.shape[0], dt)
    new_stats = dict(stats)
    for i, b in enumerate(spec["bijectors"]):
        key = f"bijectors_{i}"
        x, ld, ns = bijector_forward(b, params.get(key), stats.get(key), x, c, train, dt)
        x = _perturb(x)
        if ns:
            new_stats[key] = ns
        log_det = log_det + _perturb(ld)
    return x, log_det, new_stats


def chain_inverse(spec, params, stats, x, c, dt):
    """bijectors.py:113-116 — reverse order."""
    x = np.asarray(x, dtype=dt)
    for i in reversed(range(len(spec["bijectors"]))):
        key = f"bijectors_{i}"
        x = bijector_inverse(spec["bijectors"][i], params.get(key), stats.get(key), x, c, dt)
    return x


def _normalize_c(c):
    """flow.py:98-101."""
    if c is not None:
        c = np.asarray(c)
        if c.ndim == 1:
            c = c.reshape(-1, 1)
    return c


def flow_log_prob(model, variables, x, c=None, train=False, dtype=np.float32):
    """flow.py:22-48. ``model = {"bijector": spec, "latent": {...}}``.

    Returns (log_prob, new_batch_stats)."""
    params = variables.get("params", {}).get("bijector", {})
    stats = variables.get("batch_stats", {}).get("bijector", {})
    c = _normalize_c(c)
    if c is not None:
        c = c.astype(dtype)
    z, ld, ns = bijector_forward(model["bijector"], params, stats, x, c, train, dtype)
    lp = latent_log_prob(model["latent"], z) + ld  # :46
    lp = jnp_nan_to_num(lp, nan=-np.inf)  # :47
    return lp, ns


def jnp_nan_to_num(x, nan=0.0):
    """``jax.numpy.nan_to_num(x, nan=nan)`` for a real floating array (flow.py:47).

    JAX's published implementation (jax/_src/numpy: ``nan_to_num``) is a
    sequential ``where`` chain on the RUNNING result, with posinf/neginf
    defaulting to ``finfo(dtype).max/.min``::

        out = where(isnan(x), nan, x)
        out = where(isposinf(out), posinf, out)
        out = where(isneginf(out), neginf, out)

    so with ``nan=-inf`` a NaN row first becomes -inf and then
    ``finfo.min`` (-3.4028235e38 in fp32).  NumPy's ``np.nan_to_num`` takes
    all three masks from the INPUT instead (NaN would stay -inf), which is
    why this is spelled out rather than delegated."""
    x = np.asarray(x)
    fi = np.finfo(x.dtype)
    out = np.where(np.isnan(x), np.asarray(nan, x.dtype), x)
    out = np.where(np.isposinf(out), fi.max, out)
    out = np.where(np.isneginf(out), fi.min, out)
    return out.astype(x.dtype)


def flow_inverse(model, variables, z, c=None, dtype=np.float32):
    """flow.py:70-78 after the latent draw: bijector.inverse(z, c)."""
    params = variables.get("params", {}).get("bijector", {})
    stats = variables.get("batch_stats", {}).get("bijector", {})
    c = _normalize_c(c)
    if c is not None:
        c = c.astype(dtype)
    return bijector_inverse(model["bijector"], params, stats, np.asarray(z, dtype), c, dtype)


def row_sensitivity(model, variables, x, c=None, reps=4, eps=2.0**-22, seed=0):
    """Per-sample conditioning: max |lp_noisy - lp64| over `reps` fp64
    evaluations with relative noise `eps` (~4 fp32 ulp) injected after every
    hidden activation, conditioner output, bijector output and log-det term.
    A row whose log_prob moves by s under such perturbations cannot be
    reproduced closer than ~s by ANY fp32 evaluation (the reference's
    included); the parity tests widen the 1e-5 bound by it."""
    base, _ = flow_log_prob(model, variables, x, c, dtype=np.float64)
    rng = np.random.default_rng(seed)
    out = np.zeros_like(base)
    try:
        _NOISE.update(rng=rng, eps=eps)
        for _ in range(reps):
            lp, _ = flow_log_prob(model, variables, x, c, dtype=np.float64)
            with np.errstate(invalid="ignore"):
                dd = np.abs(lp - base)
            out = np.fmax(out, np.where(np.isfinite(dd), dd, 0.0))
    finally:
        _NOISE.update(rng=None, eps=0.0)
    return out


def nll(log_prob):
    """train.py:75-78 — -jnp.mean(log_prob) of an fp32 array.

    Accumulated in fp64 (a defined order), with the reference's fp32 overflow
    kept: ``jnp.mean`` sums in fp32, so a batch whose sum leaves the fp32
    range — e.g. two rows at finfo.min after flow.py:47 — has an infinite
    NLL there (and train.py:124-127 aborts)."""
    lp = np.asarray(log_prob, dtype=np.float64)
    return nll_from_sum(float(lp.sum()), lp.shape[0])


def nll_from_sum(total, n):
    """-total/n, infinite where the fp32 sum would overflow (see ``nll``)."""
    if total != total:
        return float("nan")
    with np.errstate(over="ignore"):
        if not np.isfinite(np.float32(total)):
            return float("inf") if total < 0 else float("-inf")
    return float(-total / max(1, n))
