"""Pin the CPU oracle against every known answer the reference's own tests hold
that is reproducible without JAX.  CPU only.

Each test cites the reference test it restates.  Inputs the reference draws
from jax.random are re-drawn from numpy with the same distributions (the
property checked is the same); `jacobi` numerical Jacobians are restated as
fp64 central differences."""

import numpy as np
import pytest
from numpy.testing import assert_allclose
from scipy.stats import beta as sp_beta
from scipy.stats import multivariate_normal

from oracle import zf_oracle as O

F32 = np.float32


# --- tests/test_utils.py ----------------------------------------------------


def test_rational_quadratic_spline_1():
    """test_utils.py:7-13: uniform bins + unit slopes => identity (OOB included)."""
    x = np.linspace(-1, 2, 10).reshape(-1, 1).astype(F32)
    W = np.tile([0.25] * 4, len(x)).reshape(*x.shape, -1).astype(F32)
    H = W.copy()
    D = np.tile([1.0] * 3, len(x)).reshape(*x.shape, -1).astype(F32)
    y, log_det = O.rqs_forward(x, W, H, D)
    assert_allclose(y, x, atol=1e-5)


def _rqs2_params():
    rng = np.random.default_rng(1)
    scale, knots = 0.1, 3
    a = scale * rng.normal(size=knots)
    b = scale * rng.normal(size=knots)
    c = scale * rng.normal(size=knots - 1)
    return a, b, c


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_rational_quadratic_spline_2(dtype):
    """test_utils.py:16-50: log_det == log dy/dx (atol 0.01), inverse (atol 1e-4)."""
    x = np.linspace(-0.1, 1.1, 1000).reshape(1000, 1).astype(dtype)
    a, b, c = (v.astype(dtype) for v in _rqs2_params())
    dx, dy, slope = O.normalize_spline_params(a, b, c)
    nx = x.size
    dx = np.tile(dx, nx).reshape(*x.shape, -1)
    dy = np.tile(dy, nx).reshape(*x.shape, -1)
    slope = np.tile(slope, nx).reshape(*x.shape, -1)
    y, log_det = O.rqs_forward(x, dx, dy, slope)
    # jacobi -> fp64 central differences of the fp64 oracle
    h = 1e-7
    x64 = x.astype(np.float64)
    d64 = [v.astype(np.float64) for v in (dx, dy, slope)]
    yp, _ = O.rqs_forward(x64 + h, *d64)
    ym, _ = O.rqs_forward(x64 - h, *d64)
    j = ((yp - ym) / (2 * h)).ravel()
    assert_allclose(y, x, atol=0.1)
    assert_allclose(log_det, np.log(j), atol=0.01)
    x2 = O.rqs_inverse(y, dx, dy, slope)
    assert_allclose(x2, x, atol=1e-4)


def test_index():
    """test_utils.py:53-68."""
    x = np.array([-2, -1, -0.5, -0.1, 0.0, 0.1, 0.5, 1.0, 1.5]).reshape(1, -1)
    xk = np.array([-1, 0, 1]).reshape(1, 3)
    expected = []
    for xi in x[0]:
        if xi < xk[0][0]:
            expected.append(0)
        elif xk[0][-1] <= xi:
            expected.append(2)
        else:
            for j in range(len(xk[0]) - 1):
                if xk[0][j] <= xi < xk[0][j + 1]:
                    expected.append(j)
                    break
    ind, oob = O.index(x, xk)
    assert_allclose(ind[0, :, 0], expected)


def test_knots():
    """test_utils.py:71-74."""
    assert_allclose(O.knots(np.array((0.25, 0.25, 0.25))), [0, 0.25, 0.5, 0.75])


@pytest.mark.parametrize("threshold", (0, 0.1))
def test_softmax_with_threshold_1(threshold):
    """test_utils.py:77-83."""
    y = O.softmax_with_threshold(np.array((-5.0, 1.0, 2.0)), threshold)
    assert_allclose(np.sum(y), 1)
    assert np.all(y >= threshold)


def test_softmax_with_threshold_2():
    """test_utils.py:86-94."""
    y = O.softmax_with_threshold(np.array([(-5.0, 1.0, 2.0), (-4.0, 2.0, 3.0)]), 0.1)
    assert_allclose(np.sum(y[0]), 1)
    assert_allclose(np.sum(y[1]), 1)
    assert_allclose(np.sum(y), 2)
    assert np.all(y[0] >= 0.1)
    assert np.all(y[1] >= 0.1)


# --- tests/test_bijectors.py -------------------------------------------------

SB = lambda margin=0.1, bounds=(): {"type": "shift_bounds", "margin": margin, "bounds": bounds}
ROLL = {"type": "roll", "shift": 1}


def test_shift_bounds_1():
    """test_bijectors.py:35-58 (KAT)."""
    x = np.array([[1, 5], [3, 4], [6, 2]])
    y, log_det, bs = O.shift_bounds_forward(SB(0.01), {}, x, train=True)
    assert_allclose(bs["xmin_0"], 0.975)
    assert_allclose(bs["xmax_0"], 6.025)
    assert_allclose(bs["xmin_1"], 1.985)
    assert_allclose(bs["xmax_1"], 5.015)
    y_ref = np.column_stack(
        [
            (x[:, 0] - bs["xmin_0"]) / (bs["xmax_0"] - bs["xmin_0"]),
            (x[:, 1] - bs["xmin_1"]) / (bs["xmax_1"] - bs["xmin_1"]),
        ]
    )
    assert_allclose(y, y_ref, atol=5e-6)
    x2 = O.shift_bounds_inverse(SB(0.01), bs, y)
    assert_allclose(x2, x, atol=1e-6)


def test_shift_bounds_2():
    """test_bijectors.py:61-92 (x re-drawn with numpy, same distributions)."""
    rng = np.random.default_rng(0)
    x = np.column_stack(
        [
            2 * rng.uniform(size=10) - 1,
            rng.exponential(size=10) * 10 + 10,
            1 - rng.exponential(size=10),
        ]
    ).astype(F32)
    spec = SB(0.0, [(0, -1, 1), (1, 10, None), (2, None, 1)])
    y, _, bs = O.shift_bounds_forward(spec, {}, x, train=True)
    x2 = O.shift_bounds_inverse(spec, bs, y)
    assert y.shape == x.shape and x2.shape == x.shape
    y0 = (x[:, 0] + 1) / 2
    t = np.log(x[:, 1] - 10)
    y1 = (t - t.min()) / (t.max() - t.min())
    t = np.log(1 - x[:, 2])
    y2 = (t - t.min()) / (t.max() - t.min())
    assert_allclose(y[:, 0], y0, atol=1e-6)
    assert_allclose(y[:, 1], y1, atol=1e-6)
    assert_allclose(y[:, 2], y2, atol=1e-6)
    assert_allclose(x2, x, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize(
    "col,bound",
    [(lambda r: 2 * r.uniform(size=10) - 1, (0, -1, 1)),
     (lambda r: r.exponential(size=10) * 10 + 10, (0, 10, None)),
     (lambda r: 1 - r.exponential(size=10), (0, None, 1))],
)
def test_shift_bounds_4(col, bound):
    """test_bijectors.py:131-165: log_det == log|dz/dx| (jacobi -> central differences)."""
    x = col(np.random.default_rng(2)).reshape(-1, 1).astype(np.float64)
    spec = SB(0.1, [bound])
    y, _, bs = O.shift_bounds_forward(spec, {}, x, train=True, dtype=np.float64)
    m = (y[:, 0] > 0.1) & (y[:, 0] < 0.9)
    x = x[m]
    _, ld, _ = O.shift_bounds_forward(spec, bs, x, dtype=np.float64)
    h = 1e-6
    yp, _, _ = O.shift_bounds_forward(spec, bs, x + h, dtype=np.float64)
    ym, _, _ = O.shift_bounds_forward(spec, bs, x - h, dtype=np.float64)
    assert_allclose(ld, np.log(np.abs((yp - ym)[:, 0] / (2 * h))), atol=1e-3)


def test_roll():
    """test_bijectors.py:168-176."""
    x = np.array([[1, 5], [3, 4], [6, 2]])
    z = O.roll(x, 1)
    assert_allclose(z, [[5, 1], [4, 3], [2, 6]])
    assert_allclose(O.roll(z, -1), x)


def test_chain_1():
    """test_bijectors.py:179-188."""
    x = np.array([[1, 2, 3], [4, 5, 6]])
    spec = {"type": "chain", "bijectors": [ROLL, ROLL]}
    z, ld, _ = O.chain_forward(spec, {}, {}, x, None, True, F32)
    assert_allclose(z, [[2, 3, 1], [5, 6, 4]])
    assert_allclose(ld, np.zeros(2))
    assert_allclose(O.chain_inverse(spec, {}, {}, z, None, F32), x)


def test_chain_2():
    """test_bijectors.py:191-206."""
    x = np.array([[2.5, 2, 3], [1, 3.5, 4.5], [4, 5, 6]])
    spec = {"type": "chain", "bijectors": [SB(0.0), ROLL]}
    y, ld, bs = O.chain_forward(spec, {}, {}, x, None, True, F32)
    assert_allclose(y, [[0.0, 0.5, 0.0], [0.5, 0.0, 0.5], [1.0, 1.0, 1.0]])
    _, ld_ref, _ = O.shift_bounds_forward(SB(0.0), bs["bijectors_0"], x)
    assert_allclose(ld, ld_ref, atol=5e-6)
    assert_allclose(O.chain_inverse(spec, {}, bs, y, None, F32), x, rtol=1e-6)


# --- tests/test_distributions.py -----------------------------------------------


def test_normal():
    """test_distributions.py:28-37 (log_prob vs multivariate_normal, atol 1e-5)."""
    x = np.random.default_rng(1).uniform(size=(10, 3))
    lp = O.normal_log_prob(x.astype(F32))
    ref = multivariate_normal.logpdf(x, 0.5 * np.ones(3), np.identity(3) * 0.1**2)
    assert_allclose(lp, ref, atol=1e-5)


def test_truncated_normal():
    """test_distributions.py:46-55 (vs multivariate_normal, atol 5e-6)."""
    x = np.random.default_rng(1).uniform(size=(10, 3))
    lp = O.truncnorm_log_prob(x.astype(F32))
    ref = multivariate_normal.logpdf(x, 0.5 * np.ones(3), np.identity(3) * 0.1**2)
    assert_allclose(lp, ref, atol=5e-6)


def test_beta():
    """test_distributions.py:64-75 (vs scipy beta.logpdf(x, 12, 12); the reference
    asserts rtol 1e-7 on fp32 values — here 2e-6, i.e. a few fp32 ulp of the sum)."""
    x = np.random.default_rng(1).uniform(size=(10, 3))
    lp = O.beta_log_prob(x.astype(F32))
    assert_allclose(lp, sp_beta.logpdf(x, 12, 12).sum(-1), rtol=2e-6)
    lp64 = O.beta_log_prob(x)
    assert_allclose(lp64, sp_beta.logpdf(x, 12, 12).sum(-1), rtol=1e-12)


def test_uniform():
    """test_distributions.py:11-25."""
    lp = O.uniform_log_prob(np.zeros((10, 3), F32))
    assert lp.shape == (10,)
    assert_allclose(lp, 0)


# --- fp32 oracle vs fp64 oracle on a whole flow (error yardstick) ----------------


def test_flow_fp32_vs_fp64():
    from tests.flowcases import make_case

    case = make_case("cfg2", N=512, seed=3)
    lp32, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float32)
    lp64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
    fin = np.isfinite(lp64)
    assert fin.mean() > 0.99
    err = np.abs(lp32[fin] - lp64[fin]) / np.maximum(1, np.abs(lp64[fin]))
    assert err.max() < 1e-5
