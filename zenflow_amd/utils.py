"""Spline numerics — drop-in for ``zenflow.utils`` (reference: src/zenflow/utils.py).

Each function runs a HIP kernel (zenflow_amd/csrc/zf_rqs.hip).  Host arrays
in -> host arrays out; ``DeviceArray`` in -> ``DeviceArray`` out."""

from __future__ import annotations

from typing import Tuple

import numpy as np

from . import _lib as L
from ._lib import DeviceArray, check

__all__ = [
    "squareplus",
    "normalize_spline_params",
    "rational_quadratic_spline_forward",
    "rational_quadratic_spline_inverse",
]

EPS = 1e-5  # utils.py:15


def _dev(a):
    return L.as_device(a, np.float32)


def squareplus(x, b: float = 4):
    """utils.py:18-20 — 0.5 * (x + sqrt(x^2 + b))."""
    xd, was = _dev(x)
    out = DeviceArray(xd.shape)
    check(L.load_library().zf_squareplus(xd.ptr, out.ptr, int(np.prod(xd.shape)), float(b), L.stream()),
          "zf_squareplus")
    return out if was else out.numpy()


def softmax_with_threshold(x, threshold: float = 0):
    """utils.py:23-34 — squareplus-based softmax whose minimum is ``threshold``."""
    xd, was = _dev(x)
    K = xd.shape[-1]
    M = int(np.prod(xd.shape[:-1], dtype=np.int64))
    out = DeviceArray(xd.shape)
    check(L.load_library().zf_softmax_with_threshold(xd.ptr, out.ptr, M, K, float(threshold), L.stream()),
          "zf_softmax_with_threshold")
    return out if was else out.numpy()


def normalize_spline_params(dx, dy, sl) -> Tuple:
    """utils.py:37-62 — widths/heights via thresholded softmax (EPS), slopes via
    squareplus.  One launch of ``zf_normalize_spline_params`` over fresh copies
    (the kernel works in place; host inputs are copied by the upload anyway)."""
    K = np.shape(dx)[-1]
    if np.shape(dy) != np.shape(dx) or tuple(np.shape(sl)) != tuple(np.shape(dx)[:-1]) + (K - 1,):
        raise ValueError(f"dx/dy (..., K) and slope (..., K-1) shapes differ: {np.shape(dx)}, {np.shape(dy)}, {np.shape(sl)}")
    outs, wases = [], []
    for a in (dx, dy, sl):
        ad, was = _dev(a)
        wases.append(was)
        if was:  # never write into the caller's device buffer
            c = DeviceArray(ad.shape)
            c.copy_from(ad)
            ad = c
        outs.append(ad)
    M = int(np.prod(outs[0].shape[:-1], dtype=np.int64))
    check(L.load_library().zf_normalize_spline_params(outs[0].ptr, outs[1].ptr, outs[2].ptr, M, K, L.stream()),
          "zf_normalize_spline_params")
    return tuple(o if was else o.numpy() for o, was in zip(outs, wases))


def _shapes(x, dx, dy, slope):
    if x.ndim != 2:
        raise ValueError(f"x must have shape (M, N), got {x.shape}")
    M, N = x.shape
    K = dx.shape[-1]
    if dx.shape != (M, N, K) or dy.shape != (M, N, K):
        raise ValueError(f"dx/dy must have shape ({M}, {N}, K), got {dx.shape}, {dy.shape}")
    if slope.shape != (M, N, K - 1):
        raise ValueError(f"slope must have shape ({M}, {N}, {K - 1}), got {slope.shape}")
    return M, N, K


def rational_quadratic_spline_forward(x, dx, dy, slope):
    """utils.py:65-141 — RQ spline (Durkan et al. 2019) on [0, 1], identity
    outside.  x (M, N), dx/dy (M, N, K), slope (M, N, K-1) ->
    (y (M, N), log_det (M,))."""
    xd, was = _dev(x)
    dxd, _ = _dev(dx)
    dyd, _ = _dev(dy)
    sld, _ = _dev(slope)
    M, N, K = _shapes(xd, dxd, dyd, sld)
    y = DeviceArray((M, N))
    ld = DeviceArray((M,))
    check(L.load_library().zf_rqs_forward(xd.ptr, dxd.ptr, dyd.ptr, sld.ptr, y.ptr, ld.ptr, M, N, K,
                                          L.stream()), "zf_rqs_forward")
    return (y, ld) if was else (y.numpy(), ld.numpy())


def rational_quadratic_spline_inverse(y, dx, dy, slope):
    """utils.py:144-202 — inverse RQ spline via the quadratic root; returns x (M, N)."""
    yd, was = _dev(y)
    dxd, _ = _dev(dx)
    dyd, _ = _dev(dy)
    sld, _ = _dev(slope)
    M, N, K = _shapes(yd, dxd, dyd, sld)
    x = DeviceArray((M, N))
    check(L.load_library().zf_rqs_inverse(yd.ptr, dxd.ptr, dyd.ptr, sld.ptr, x.ptr, M, N, K,
                                          L.stream()), "zf_rqs_inverse")
    return x if was else x.numpy()
