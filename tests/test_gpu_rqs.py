"""K1 parity: zenflow_amd.utils (HIP kernels via the C ABI) vs the oracle and
the reference's own utils tests (tests/test_utils.py).  Needs the GPU."""

import numpy as np
import pytest
from numpy.testing import assert_allclose

from oracle import zf_oracle as O

pytestmark = pytest.mark.gpu
F32 = np.float32


def _zu():
    from zenflow_amd import utils

    return utils


def random_params(rng, M, N, K, scale=1.0):
    dx = (scale * rng.standard_normal((M, N, K))).astype(F32)
    dy = (scale * rng.standard_normal((M, N, K))).astype(F32)
    sl = (scale * rng.standard_normal((M, N, K - 1))).astype(F32)
    return O.normalize_spline_params(dx, dy, sl)


def test_rational_quadratic_spline_1():
    """test_utils.py:7-13 through the HIP kernel."""
    u = _zu()
    x = np.linspace(-1, 2, 10).reshape(-1, 1)
    W = np.tile([0.25] * 4, len(x)).reshape(*x.shape, -1)
    D = np.tile([1.0] * 3, len(x)).reshape(*x.shape, -1)
    y, log_det = u.rational_quadratic_spline_forward(x, W, W, D)
    assert_allclose(y, x, atol=1e-5)


def test_rational_quadratic_spline_2():
    """test_utils.py:16-50 through the HIP kernel (jacobi -> fp64 central differences)."""
    u = _zu()
    rng = np.random.default_rng(1)
    x = np.linspace(-0.1, 1.1, 1000).reshape(1000, 1)
    dx, dy, slope = u.normalize_spline_params(
        0.1 * rng.normal(size=3), 0.1 * rng.normal(size=3), 0.1 * rng.normal(size=2)
    )
    nx = x.size
    dx = np.tile(dx, nx).reshape(*x.shape, -1)
    dy = np.tile(dy, nx).reshape(*x.shape, -1)
    slope = np.tile(slope, nx).reshape(*x.shape, -1)
    y, log_det = u.rational_quadratic_spline_forward(x, dx, dy, slope)
    h = 1e-7
    d64 = [v.astype(np.float64) for v in (dx, dy, slope)]
    j = ((O.rqs_forward(x + h, *d64)[0] - O.rqs_forward(x - h, *d64)[0]) / (2 * h)).ravel()
    assert_allclose(y, x, atol=0.1)
    assert_allclose(log_det, np.log(j), atol=0.01)
    x2 = u.rational_quadratic_spline_inverse(y, dx, dy, slope)
    assert_allclose(x2, x, atol=1e-4)


@pytest.mark.parametrize("threshold", (0, 0.1))
def test_softmax_with_threshold(threshold):
    """test_utils.py:77-94."""
    u = _zu()
    y = u.softmax_with_threshold(np.array([(-5.0, 1.0, 2.0), (-4.0, 2.0, 3.0)]), threshold)
    assert_allclose(y.sum(-1), 1, rtol=1e-6)
    assert np.all(y >= threshold * (1 - 1e-6))
    assert_allclose(y, O.softmax_with_threshold(np.array([(-5.0, 1.0, 2.0), (-4.0, 2.0, 3.0)], F32), threshold), rtol=1e-6)


def test_normalize_and_squareplus_vs_oracle():
    u = _zu()
    rng = np.random.default_rng(5)
    a = (3 * rng.standard_normal((257, 16))).astype(F32)
    b = (3 * rng.standard_normal((257, 16))).astype(F32)
    c = (3 * rng.standard_normal((257, 15))).astype(F32)
    got = u.normalize_spline_params(a, b, c)
    ref = O.normalize_spline_params(a, b, c)
    for g, r in zip(got, ref):
        assert_allclose(g, r, rtol=2e-6, atol=1e-7)
    # x*x+b may contract to an fma on the GPU; cancellation at large negative x
    assert_allclose(u.squareplus(a), O.squareplus(a), rtol=1e-5)


@pytest.mark.parametrize("K", [2, 4, 5, 8, 16, 32])
@pytest.mark.parametrize("M", [1, 3, 1023, 4099])
def test_normalize_spline_params_shapes(K, M):
    """The float4 stream kernel (K in {4, 8, 16, 32}: ragged tails, rows on
    K/4 lanes, slope tails) and the LDS row kernel (other K) vs the oracle."""
    u = _zu()
    rng = np.random.default_rng(K * 7 + M)
    a = (3 * rng.standard_normal((M, 2, K))).astype(F32)
    b = (3 * rng.standard_normal((M, 2, K))).astype(F32)
    c = (3 * rng.standard_normal((M, 2, K - 1))).astype(F32)
    got = u.normalize_spline_params(a, b, c)
    ref = O.normalize_spline_params(a, b, c)
    # rtol = the north star's 1e-5: x*x + 4 contracts to an fma on the GPU, and
    # squareplus cancels at large negative logits (a 2-knot row divides two
    # such values directly: up to ~3e-6 here)
    for g, r in zip(got, ref):
        assert g.shape == r.shape
        assert_allclose(g, r, rtol=1e-5, atol=1e-7)
    assert_allclose(got[0].sum(-1), 1, rtol=2e-6)


@pytest.mark.parametrize("K", [1, 2, 3, 4, 5, 8, 16, 32, 64])
@pytest.mark.parametrize("N", [1, 2, 3, 8])
def test_rqs_parity(K, N):
    """Random normalised params incl. out-of-bounds x; y, log_det and inverse."""
    u = _zu()
    rng = np.random.default_rng(K * 100 + N)
    M = 3001  # ragged: not a multiple of the block's rows
    dx, dy, sl = random_params(rng, M, N, K, scale=1.5)
    x = rng.uniform(-0.2, 1.2, size=(M, N)).astype(F32)
    y, ld = u.rational_quadratic_spline_forward(x, dx, dy, sl)
    yr, ldr = O.rqs_forward(x, dx, dy, sl)
    fin = np.isfinite(yr)
    assert np.array_equal(fin, np.isfinite(y))
    assert_allclose(y[fin], yr[fin], rtol=2e-6, atol=2e-6)
    finl = np.isfinite(ldr)
    assert np.array_equal(finl, np.isfinite(ld))
    assert_allclose(ld[finl], ldr[finl], rtol=1e-5, atol=1e-5)
    xi = u.rational_quadratic_spline_inverse(yr, dx, dy, sl)
    xr = O.rqs_inverse(yr, dx, dy, sl)
    fin = np.isfinite(xr)
    assert np.array_equal(fin, np.isfinite(xi))
    assert_allclose(xi[fin], xr[fin], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("K", [16, 32])
def test_rqs_parity_bench_shape(K):
    """K1 at the bench's timed shape — one cfg2 coupling over 2^20 rows x 2
    transformed dims (bench.py spline_kernel) — against the oracle on every
    row: y, log_det, and the inverse of the reference's y."""
    u = _zu()
    rng = np.random.default_rng(K)
    M = 1 << 20
    dx, dy, sl = random_params(rng, M, 2, K, scale=1.5)
    x = rng.uniform(-0.05, 1.05, size=(M, 2)).astype(F32)
    y, ld = u.rational_quadratic_spline_forward(x, dx, dy, sl)
    yr, ldr = O.rqs_forward(x, dx, dy, sl)
    fin = np.isfinite(yr)
    assert np.array_equal(fin, np.isfinite(y))
    assert_allclose(y[fin], yr[fin], rtol=2e-6, atol=2e-6)
    finl = np.isfinite(ldr)
    assert np.array_equal(finl, np.isfinite(ld))
    assert_allclose(ld[finl], ldr[finl], rtol=1e-5, atol=1e-5)
    xi = u.rational_quadratic_spline_inverse(yr, dx, dy, sl)
    xr = O.rqs_inverse(yr, dx, dy, sl)
    fin = np.isfinite(xr)
    assert np.array_equal(fin, np.isfinite(xi))
    assert_allclose(xi[fin], xr[fin], rtol=1e-5, atol=1e-5)


def test_rqs_edge_cases():
    """Sliver idx == K (fill-mode gather -> NaN), x == 1 (OOB identity), NaN x,
    empty batch."""
    u = _zu()
    K = 4
    dx = np.full((1, 5, K), 0.2499999, F32)  # sums to < 1
    dy = np.full((1, 5, K), 0.25, F32)
    sl = np.ones((1, 5, K - 1), F32)
    x = np.array([[0.99999994, 1.0, np.nan, 0.5, -0.0]], F32)
    y, ld = u.rational_quadratic_spline_forward(x, dx, dy, sl)
    yr, ldr = O.rqs_forward(x, dx, dy, sl)
    assert np.isnan(y[0, 0]) and np.isnan(yr[0, 0])
    assert y[0, 1] == 1.0 and yr[0, 1] == 1.0
    assert np.isnan(y[0, 2]) and np.isnan(yr[0, 2])
    assert_allclose(y[0, 3:], yr[0, 3:], atol=1e-6)
    assert np.isnan(ld[0]) and np.isnan(ldr[0])
    y0, ld0 = u.rational_quadratic_spline_forward(
        np.zeros((0, 2), F32), np.zeros((0, 2, K), F32), np.zeros((0, 2, K), F32), np.zeros((0, 2, K - 1), F32)
    )
    assert y0.shape == (0, 2) and ld0.shape == (0,)


def test_rqs_golden():
    """Committed golden vectors (tests/golden/make_golden.py)."""
    from pathlib import Path

    u = _zu()
    g = Path(__file__).parent / "golden"
    for f in sorted(g.glob("rqs_K*.npz")):
        d = np.load(f)
        y, ld = u.rational_quadratic_spline_forward(d["x"], d["dx"], d["dy"], d["slope"])
        fin = np.isfinite(d["y"])
        assert_allclose(y[fin], d["y"][fin], rtol=2e-6, atol=2e-6, err_msg=f.name)
        assert_allclose(ld, d["log_det"], rtol=1e-5, atol=1e-5, err_msg=f.name)
        xi = u.rational_quadratic_spline_inverse(d["y"], d["dx"], d["dy"], d["slope"])
        fin = np.isfinite(d["x_inv"])
        assert_allclose(xi[fin], d["x_inv"][fin], rtol=1e-5, atol=1e-5, err_msg=f.name)


@pytest.mark.parametrize("N", [1, 2, 3, 8, 40])
@pytest.mark.parametrize("monotone", [True, False])
def test_rqs_k32_two_lane_matches_one_lane(N, monotone, monkeypatch):
    """K = 32 runs two lanes per item (rqs_kernel_pair: lane 1 continues lane
    0's in-order knot sums, so bins and knots carry the one-lane kernel's
    bits): the same results as the one-lane kernel (ZF_K1_ONE_LANE=1) up to
    the compiler's fma contraction of the evaluation (a few ulp), forward,
    log_det (lane-shuffle rows, N <= 32, and the LDS rows, N = 40) and
    inverse, on normalised and on raw (non-monotone knots: the generic-search
    fallback) parameters; identical finiteness (same bins)."""
    u = _zu()
    K = 32
    rng = np.random.default_rng(900 + N)
    M = 2051
    if monotone:
        dx, dy, sl = random_params(rng, M, N, K, scale=1.5)
    else:
        dx = (0.06 * rng.standard_normal((M, N, K)) + 0.03).astype(F32)
        dy = (0.06 * rng.standard_normal((M, N, K)) + 0.03).astype(F32)
        sl = np.abs(rng.standard_normal((M, N, K - 1))).astype(F32) + 0.1
    x = rng.uniform(-0.1, 1.1, size=(M, N)).astype(F32)
    y2, ld2 = u.rational_quadratic_spline_forward(x, dx, dy, sl)
    xi2 = u.rational_quadratic_spline_inverse(x, dx, dy, sl)
    monkeypatch.setenv("ZF_K1_ONE_LANE", "1")
    y1, ld1 = u.rational_quadratic_spline_forward(x, dx, dy, sl)
    xi1 = u.rational_quadratic_spline_inverse(x, dx, dy, sl)
    for a, b in ((y1, y2), (ld1, ld2), (xi1, xi2)):
        assert np.array_equal(np.isfinite(a), np.isfinite(b))
        f = np.isfinite(a)
        assert_allclose(b[f], a[f], rtol=1e-6, atol=1e-6)
