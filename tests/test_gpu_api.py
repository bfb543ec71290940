"""The reference's own bijector / distribution / flow tests, restated through the
zenflow_amd API (tests/test_bijectors.py, test_distributions.py, test_flow.py).
Reads like the reference: same calls, same assertions.  Needs the GPU."""

import numpy as np
import pytest
from numpy.testing import assert_allclose
from scipy.stats import beta as sp_beta
from scipy.stats import multivariate_normal

import zenflow_amd.bijectors as bi
import zenflow_amd.distributions as dist
from zenflow_amd import Flow
from zenflow_amd.random import PRNGKey
from oracle import zf_oracle as O

pytestmark = pytest.mark.gpu
KEY = PRNGKey(0)


def test_ShiftBounds_1():
    x = np.array([[1, 5], [3, 4], [6, 2]])
    sb = bi.ShiftBounds(margin=0.01)
    variables = sb.init(KEY, x, None)
    (y, log_det), updates = sb.apply(variables, x, None, train=True, mutable=["batch_stats"])
    bs = updates["batch_stats"]
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
    x2 = sb.apply(updates, y, None, method="inverse")
    assert_allclose(x2, x, atol=1e-6)


def test_ShiftBounds_2():
    rng = np.random.default_rng(0)
    x = np.column_stack(
        [2 * rng.uniform(size=10) - 1, rng.exponential(size=10) * 10 + 10, 1 - rng.exponential(size=10)]
    ).astype(np.float32)
    bounds = [(0, -1, 1), (1, 10, None), (2, None, 1)]
    tr = bi.ShiftBounds(margin=0.0, bounds=bounds)
    vars = tr.init(KEY, x, None)
    (y, ld), vars = tr.apply(vars, x, None, train=True, mutable=["batch_stats"])
    x2 = tr.apply(vars, y, None, method="inverse")
    assert y.shape == x.shape and x2.shape == x.shape
    t1 = np.log(x[:, 1] - 10)
    t2 = np.log(1 - x[:, 2])
    assert_allclose(y[:, 0], (x[:, 0] + 1) / 2, atol=1e-6)
    assert_allclose(y[:, 1], (t1 - t1.min()) / (t1.max() - t1.min()), atol=1e-6)
    assert_allclose(y[:, 2], (t2 - t2.min()) / (t2.max() - t2.min()), atol=1e-6)
    # log_det vs the oracle (same train-mode statistics)
    _, ldr, _ = O.shift_bounds_forward({"margin": 0.0, "bounds": bounds}, {}, x, train=True)
    assert_allclose(ld, ldr, rtol=1e-5, atol=1e-5)


def test_ShiftBounds_bad_args():
    with pytest.raises(ValueError):
        bi.ShiftBounds(margin=-0.1)
    with pytest.raises(ValueError):
        bi.ShiftBounds(margin=1.0)
    with pytest.raises(ValueError):
        bi.ShiftBounds(bounds=[(5, 0, 1)]).init(KEY, np.zeros((3, 2)), None)
    with pytest.raises(ValueError):
        bi.ShiftBounds(bounds=[(0, 1, 0)]).init(KEY, np.zeros((3, 2)), None)


def test_Roll():
    x = np.array([[1, 5], [3, 4], [6, 2]])
    roll = bi.Roll()
    variables = roll.init(KEY, x, None)
    (z, log_det) = roll.apply(variables, x, None, train=True)
    assert_allclose(z, np.array([[5, 1], [4, 3], [2, 6]]))
    assert_allclose(log_det, np.zeros(3))
    x2 = roll.apply(variables, z, None, method="inverse")
    assert_allclose(x2, x)


def test_Chain_1():
    x = np.array([[1, 2, 3], [4, 5, 6]])
    chain = bi.Chain([bi.Roll(), bi.Roll()])
    assert len(chain) == 2
    variables = chain.init(KEY, x, None)
    (z, log_det) = chain.apply(variables, x, None, train=True)
    assert_allclose(z, [[2, 3, 1], [5, 6, 4]])
    assert_allclose(log_det, np.zeros(2))
    x2 = chain.apply(variables, z, None, method="inverse")
    assert_allclose(x2, x)


def test_Chain_2():
    x = np.array([[2.5, 2, 3], [1, 3.5, 4.5], [4, 5, 6]])
    chain = bi.Chain([bi.ShiftBounds(margin=0.0), bi.Roll()])
    variables = chain.init(KEY, x, None)
    (y, log_det), updates = chain.apply(variables, x, None, train=True, mutable=["batch_stats"])
    assert_allclose(y, [[0.0, 0.5, 0.0], [0.5, 0.0, 0.5], [1.0, 1.0, 1.0]])
    log_det_ref = chain[0].apply({"batch_stats": updates["batch_stats"]["bijectors_0"]}, x, None)[1]
    assert_allclose(log_det, log_det_ref, atol=5e-6)
    x2 = chain.apply(updates, y, None, method="inverse")
    assert_allclose(x2, x, rtol=1e-6)


def test_Chain_3():
    x = np.array([[1.5, 2], [1, 3.5], [3.5, 4]])
    c = np.array([[1.0], [2.0], [3.0]])
    chain = bi.chain(bi.ShiftBounds(), bi.NeuralSplineCoupling(), bi.Roll(), bi.NeuralSplineCoupling())
    variables = chain.init(KEY, x, c)
    (y, log_det), updates = chain.apply(variables, x, c, train=True, mutable=["batch_stats"])
    variables = {"params": variables["params"], "batch_stats": updates["batch_stats"]}
    (y, log_det) = chain.apply(variables, x, c, train=False)
    x2 = chain.apply(variables, y, c, method="inverse")
    assert_allclose(x2, x, rtol=1e-5)


def test_NeuralSplineCoupling_1():
    x = np.array([[1.5, 2], [1, 3.5], [3.5, 4]])
    c = np.array([[1.0], [2.0], [3.0]])
    nsc = bi.NeuralSplineCoupling()
    variables = nsc.init(KEY, x, c)
    (y, log_det) = nsc.apply(variables, x, c, train=False)
    x2 = nsc.apply(variables, y, c, method="inverse")
    assert_allclose(x2, x, atol=1e-5)


def test_NeuralSplineCoupling_2():
    x = np.array([[1.5, 2, 3.3], [1, 3.5, 4.5], [3.5, 4, 5.5]])
    xt, xc = bi.NeuralSplineCoupling._split(x)
    assert xt.shape[1] == 1
    assert xc.shape[1] == 2


def test_rolling_spline_coupling():
    x = np.array([[1.5, 2], [1, 3.5], [3.5, 4]])
    c = np.array([[1.0], [2.0], [3.0]])
    rsc = bi.rolling_spline_coupling(x.shape[1], layers=(64, 64))
    variables = rsc.init(KEY, x, c)
    (y, log_det), updates = rsc.apply(variables, x, c, train=True, mutable=["batch_stats"])
    variables = {"params": variables["params"], "batch_stats": updates["batch_stats"]}
    (y, log_det) = rsc.apply(variables, x, c, train=False)
    x2 = rsc.apply(variables, y, c, method="inverse")
    assert_allclose(x2, x, atol=1e-4)


@pytest.mark.parametrize("name", ["cfg4", "h384c2"])  # h384c2: a hidden width on the layered path
def test_train_mode_matches_oracle(name):
    """Train-mode forward (batch statistics for ShiftBounds + BatchNorm) vs the
    oracle, and the running-average updates."""
    from tests.flowcases import build_flow, make_case

    case = make_case(name, N=3000, seed=31)
    flow = build_flow(case["cfg"])
    lp, upd = flow.apply(case["variables"], case["x"], case["c"], train=True, mutable=["batch_stats"])
    ref, ref_stats = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], train=True)
    fin = np.isfinite(ref) & np.isfinite(lp)
    assert np.mean(np.isfinite(ref) != np.isfinite(lp)) <= 1e-3
    assert_allclose(lp[fin], ref[fin], rtol=2e-5, atol=2e-5)
    got = upd["batch_stats"]["bijector"]
    D = case["cfg"]["D"]
    for j in range(D):
        for k in (f"xmin_{j}", f"xmax_{j}"):
            assert_allclose(got["bijectors_0"][k], ref_stats["bijectors_0"][k], rtol=1e-6)
    for b in [k for k in ref_stats if k != "bijectors_0" and "BatchNorm_0" in ref_stats[k]]:
        for k in ("mean", "var"):
            assert_allclose(got[b]["BatchNorm_0"][k], ref_stats[b]["BatchNorm_0"][k], rtol=1e-5, atol=1e-6)


def test_rolling_spline_coupling_bad_input():
    with pytest.raises(ValueError):
        bi.rolling_spline_coupling(0)
    with pytest.raises(ValueError):
        bi.rolling_spline_coupling(1)


# --- tests/test_distributions.py ---------------------------------------------


def test_Normal():
    d = dist.Normal()
    x = np.random.default_rng(1).uniform(size=(10, 3))
    lp = d.log_prob(x)
    assert_allclose(lp, multivariate_normal.logpdf(x, 0.5 * np.ones(3), np.identity(3) * 0.1**2), atol=1e-5)
    s = d.sample(20000, PRNGKey(0))
    assert s.shape == (20000, 3)
    assert_allclose(s.mean(0), 0.5, atol=5e-2)
    assert_allclose(np.cov(s.T), 0.1**2 * np.identity(3), atol=5e-2)


def test_TruncatedNormal():
    d = dist.TruncatedNormal()
    x = np.random.default_rng(1).uniform(size=(10, 3))
    lp = d.log_prob(x)
    assert_allclose(lp, multivariate_normal.logpdf(x, 0.5 * np.ones(3), np.identity(3) * 0.1**2), atol=5e-6)
    s = d.sample(20000, PRNGKey(0))
    assert s.shape == (20000, 3)
    assert_allclose(s.mean(0), 0.5, atol=5e-2)


def test_Beta():
    d = dist.Beta()
    x = np.random.default_rng(1).uniform(size=(10, 3))
    lp = d.log_prob(x)
    assert_allclose(lp, sp_beta.logpdf(x, 12, 12).sum(-1), rtol=2e-6)
    s = d.sample(20000, PRNGKey(0))
    assert s.shape == (20000, 3)
    assert_allclose(s.mean(0), 0.5, atol=5e-2)
    assert np.all(s > 0) and np.all(s < 1)
    assert repr(d) == "Beta(peakness=12.0)"
    with pytest.raises(ValueError):
        dist.Beta(-1)


def test_Uniform():
    uni = dist.Uniform()
    lp = uni.log_prob(np.zeros((10, 3)))
    assert lp.shape == (10,)
    assert_allclose(lp, 0)
    x = uni.sample(2, PRNGKey(0))
    assert x.shape == (2, 3)
    assert np.min(x) >= 0 and np.max(x) < 1
    assert repr(uni) == "Uniform()"


# --- tests/test_flow.py ---------------------------------------------------------


def test_Flow_1():
    flow = Flow(bi.ShiftBounds())
    x = np.array([[3.0, 2.0], [1.0, 4.0], [5.0, 6.0]])
    variables = flow.init(PRNGKey(0), x)
    log_prob, variables = flow.apply(variables, x, train=True, mutable=["batch_stats"])
    x2 = flow.apply(variables, 1000, method="sample")
    assert x2.shape == (1000, 2)
    assert x2[:, 0].min() >= 1 - 0.2 and x2[:, 0].max() <= 5 + 0.2


def test_Flow_2():
    flow = Flow(bi.ShiftBounds())
    x = np.array([[3.0, 2.0], [1.0, 4.0], [5.0, 6.0]])
    c = np.array([1.0, 2.0, 3.0])
    variables = flow.init(PRNGKey(0), x)
    log_prob, variables = flow.apply(variables, x, c, train=True, mutable=["batch_stats"])
    x2 = flow.apply(variables, c, method="sample")
    assert x2.shape == (3, 2)


def test_Flow_two_moons_sample_roundtrip():
    """Flow.sample = latent draw -> bijector inverse; log_prob of the samples is
    finite and forward(sample) recovers the latent draw."""
    from tests.flowcases import build_flow, make_case

    case = make_case("cfg1", N=256, seed=41)
    flow = build_flow(case["cfg"])
    flow.init(PRNGKey(0), case["x"])  # latches latent dim
    xs = flow.apply(case["variables"], 512, method="sample", seed=3)
    assert xs.shape == (512, 2) and np.isfinite(xs).all()
    lp = flow.apply(case["variables"], xs)
    assert np.isfinite(lp).mean() > 0.95


def test_apply_caches_program_by_content():
    """flow.apply(variables, x) packs and uploads the weights once per
    distinct variables content: same tree -> same program;
    an in-place change of a leaf -> a new program with the new weights;
    train-mode calls never reuse (or dirty) the cached eval program."""
    from tests.flowcases import build_flow, make_case

    case = make_case("cfg1", N=512, seed=43)
    flow = build_flow(case["cfg"])
    v = case["variables"]
    lp1 = flow.apply(v, case["x"])
    progs = list(flow._programs.values())
    lp2 = flow.apply(v, case["x"])
    assert list(flow._programs.values()) == progs and len(progs) == 1
    assert np.array_equal(lp1, lp2, equal_nan=True)
    flow.apply(v, case["x"], train=True, mutable=["batch_stats"])
    assert list(flow._programs.values()) == progs
    assert np.array_equal(flow.apply(v, case["x"]), lp1, equal_nan=True)
    # in-place edit of one bias: the digest changes, the output follows the oracle
    bias = v["params"]["bijector"]["bijectors_1"]["Dense_0"]["bias"]
    bias += np.float32(0.25)
    lp3 = flow.apply(v, case["x"])
    assert len(flow._programs) == 2
    ref, _ = O.flow_log_prob(case["model"], v, case["x"], None)
    f = np.isfinite(ref)
    assert_allclose(lp3[f], ref[f], rtol=2e-5, atol=2e-5)
    assert not np.allclose(lp3[f], lp1[f])


def test_nested_flow_deep_set():
    """DeepSetFlow (examples/deep_set.ipynb:318-328): the outer module calls
    self.flow(y, c, train=train) and self.flow.sample(c, seed=seed); the
    results equal a top-level Flow applied to the flow sub-tree bit for bit,
    and train-mode batch-stats updates land at batch_stats/flow."""
    from tests.flowcases import make_deep_set_module

    DeepSetFlow = make_deep_set_module()
    m = DeepSetFlow(bi.rolling_spline_coupling(2, layers=(64,) * 3))
    rng = np.random.default_rng(5)
    x = rng.standard_normal((1000, 3)).astype(np.float32)
    y = (0.5 + 0.1 * rng.standard_normal((1000, 2))).astype(np.float32)
    v = m.init(KEY, x, y)
    _, upd = m.apply(v, x, y, train=True, mutable=["batch_stats"])
    assert sorted(upd["batch_stats"]) == ["flow"]
    v = {"params": v["params"], "batch_stats": upd["batch_stats"]}
    lp = m.apply(v, x, y)
    c = m.apply(v, x, method=lambda mod, x: mod.phi(x))
    sub = {"params": v["params"]["flow"], "batch_stats": v["batch_stats"]["flow"]}
    top = Flow(m.bijectors)
    assert np.array_equal(lp, top.apply(sub, y, c), equal_nan=True)
    # train-mode update of the nested flow == the top-level one
    _, u_top = top.apply(sub, y, c, train=True, mutable=["batch_stats"])
    _, u_nest = m.apply(v, x, y, train=True, mutable=["batch_stats"])
    for path in [("bijectors_0", "xmin_0"), ("bijectors_1", "BatchNorm_0", "mean")]:
        a, b = u_top["batch_stats"]["bijector"], u_nest["batch_stats"]["flow"]["bijector"]
        for k in path:
            a, b = a[k], b[k]
        assert np.array_equal(a, b)
    s_nest = m.apply(v, x, seed=3, method="sample")
    s_top = top.apply(sub, c, seed=3, method="sample")
    assert s_nest.shape == (1000, 2) and np.array_equal(s_nest, s_top, equal_nan=True)


def test_bijector_apply_caches_program():
    """Bijector-level apply (Chain / NSC) packs the weights once per distinct
    variables content, as Flow does."""
    ch = bi.rolling_spline_coupling(2, layers=(32, 32))
    x = (0.5 + 0.1 * np.random.default_rng(1).standard_normal((256, 2))).astype(np.float32)
    v = ch.init(KEY, x, None)
    _, upd = ch.apply(v, x, None, train=True, mutable=["batch_stats"])
    v = {"params": v["params"], "batch_stats": upd["batch_stats"]}
    y1, ld1 = ch.apply(v, x, None)
    assert len(ch._programs) == 1
    y2, ld2 = ch.apply(v, x, None)
    assert len(ch._programs) == 1 and np.array_equal(y1, y2) and np.array_equal(ld1, ld2)
    xi = ch.apply(v, y1, None, method="inverse")
    assert len(ch._programs) == 1
    assert_allclose(xi, x, atol=2e-5)
