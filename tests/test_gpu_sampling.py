"""On-device latent sampling: Distribution.sample and
Flow.sample with the counter-based Philox generator (zf_latent_sample,
zf_flow_sample).

jax.random's threefry draws cannot be reproduced without JAX, so parity is
(1) statistical — Kolmogorov-Smirnov against scipy's distributions and the
moment checks of the reference's tests/test_distributions.py — and (2)
structural: Flow.sample(seed) is bit-identical to Chain.inverse applied to
Distribution.sample(seed), and Chain.inverse is parity-tested against the
oracle (tests/test_gpu_flow.py)."""

import numpy as np
import pytest
from scipy import stats

import zenflow_amd.distributions as dist
from zenflow_amd import _lib as L
from zenflow_amd.random import PRNGKey, key_to_seed
from tests.flowcases import build_flow, make_case

pytestmark = pytest.mark.gpu

N = 1 << 16


def _draw(d, n=N, dim=3, seed=7):
    d._dim = dim
    return d.sample(n, PRNGKey(seed))


@pytest.mark.parametrize(
    "d,ref",
    [
        (dist.Normal(), stats.norm(0.5, 0.1)),
        (dist.TruncatedNormal(), stats.truncnorm(-5, 5, loc=0.5, scale=0.1)),
        (dist.Beta(), stats.beta(12, 12)),
        (dist.Beta(3.0), stats.beta(3, 3)),
        (dist.Uniform(), stats.uniform(0, 1)),
    ],
)
def test_latent_distribution_ks(d, ref):
    z = _draw(d)
    assert z.shape == (N, 3) and z.dtype == np.float32 and np.isfinite(z).all()
    for j in range(3):
        p = stats.kstest(z[:, j].astype(np.float64), ref.cdf).pvalue
        assert p > 1e-4, f"dim {j}: KS p={p:.2e}"
    # dims independent (sample correlation ~ N(0, 1/N))
    r = np.corrcoef(z.T)
    assert np.abs(r[np.triu_indices(3, 1)]).max() < 6 / np.sqrt(N)


def test_latent_support_and_moments():
    """tests/test_distributions.py moment / support checks at the same n."""
    n = 20000
    zn = _draw(dist.Normal(), n)
    np.testing.assert_allclose(zn.mean(0), 0.5, atol=5e-2)
    np.testing.assert_allclose(np.cov(zn.T), 0.1**2 * np.identity(3), atol=5e-2)
    zt = _draw(dist.TruncatedNormal(), n)
    assert np.all(np.abs(zt - 0.5) <= 0.5 + 1e-6)
    zb = _draw(dist.Beta(), n)
    assert np.all(zb > 0) and np.all(zb < 1)
    zu = _draw(dist.Uniform(), n)
    assert zu.min() >= 0 and zu.max() < 1


def test_latent_determinism_and_row_independence():
    d = dist.Beta()
    a = _draw(d, 5000, seed=11)
    b = _draw(d, 5000, seed=11)
    c = _draw(d, 1000, seed=11)
    e = _draw(d, 1000, seed=12)
    assert np.array_equal(a, b)
    assert np.array_equal(a[:1000], c)  # counter-based: row r depends only on (seed, r)
    assert not np.array_equal(c, e)


def test_latent_sample_errors():
    lib = L.load_library()
    z = L.DeviceArray((4, 2))
    assert lib.zf_latent_sample(L.ZF_LATENT_BETA, 0.5, 1, z.ptr, 4, 2, None) == -1
    assert lib.zf_latent_sample(99, 0.0, 1, z.ptr, 4, 2, None) == -1
    assert lib.zf_latent_sample(L.ZF_LATENT_NORMAL, 0.0, 1, z.ptr, 0, 2, None) == 0


@pytest.mark.parametrize("name", ["cfg2", "cfg1", "cfg4", "small", "cfg5", "h512", "h384c2"])
def test_flow_sample_equals_inverse_of_latent(name):
    """zf_flow_sample (latent drawn in the inverse kernel's prologue) ==
    Chain.inverse(Distribution.sample) bit for bit, on both fused kernels."""
    case = make_case(name, N=8, seed=43)
    cfg = case["cfg"]
    flow = build_flow(cfg)
    bf = flow.bind(case["variables"], cfg["D"], cfg["C"])
    prog = bf.program
    n = 3000
    c = None
    if cfg["C"]:
        c = L.DeviceArray.from_numpy(np.random.default_rng(5).standard_normal((n, cfg["C"])).astype(np.float32))
    seed = key_to_seed(PRNGKey(9))
    xs = prog.sample(n, seed, c).numpy()
    flow.latent._dim = cfg["D"]
    z = flow.latent.sample(n, PRNGKey(9))
    xi = prog.inverse(L.DeviceArray.from_numpy(z), c).numpy()
    assert np.array_equal(xs, xi, equal_nan=True)
    assert np.isfinite(xs).mean() > 0.99


def test_flow_sample_api_statistics():
    """Flow.sample through the API: the flow maps its latent samples back to
    data, so log_prob of the samples is finite and forward(samples) has the
    latent's moments (cfg2: Normal(0.5, 0.1) latent)."""
    case = make_case("cfg2", N=4096, seed=44)
    flow = build_flow(case["cfg"])
    flow.init(PRNGKey(0), case["x"][:1])
    xs = flow.apply(case["variables"], 20000, method="sample", seed=5)
    assert xs.shape == (20000, 4) and np.isfinite(xs).all()
    sub = {k: v["bijector"] for k, v in case["variables"].items()}
    z, _ = flow.bijector.apply(sub, xs)
    inside = np.all((z > 0.02) & (z < 0.98), axis=1)  # away from ShiftBounds clipping
    assert inside.mean() > 0.99
    np.testing.assert_allclose(z[inside].mean(0), 0.5, atol=5e-3)
    np.testing.assert_allclose(z[inside].std(0), 0.1, atol=5e-3)
