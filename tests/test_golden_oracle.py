"""The committed golden fixtures (tests/golden/make_golden.py) are reproduced
by the CPU oracle: inputs regenerate bit-identically from their seeds and the
oracle's outputs match the stored ones (BLAS summation order may differ
between hosts, hence a 1e-6 relative tolerance on the MLP-dependent values)."""

import json
from pathlib import Path

import numpy as np
import pytest
from numpy.testing import assert_allclose

from oracle import zf_oracle as O
from tests.flowcases import make_case

G = Path(__file__).parent / "golden"


@pytest.mark.parametrize("K", [8, 16, 32])
def test_rqs_fixture(K):
    d = np.load(G / f"rqs_K{K}.npz")
    y, ld = O.rqs_forward(d["x"], d["dx"], d["dy"], d["slope"])
    assert np.array_equal(y, d["y"], equal_nan=True)
    assert np.array_equal(ld, d["log_det"], equal_nan=True)
    xi = O.rqs_inverse(d["y"], d["dx"], d["dy"], d["slope"])
    assert np.array_equal(xi, d["x_inv"], equal_nan=True)


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4", "cfg5"])
def test_flow_fixture(name):
    d = np.load(G / f"flow_{name}.npz")
    meta = json.loads(str(d["meta"]))
    case = make_case(meta["name"], N=int(meta["N"]), seed=int(meta["seed"]))
    assert np.array_equal(case["x"], d["x"])
    lp, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"])
    fin = np.isfinite(d["log_prob"])
    assert np.array_equal(np.isfinite(lp), fin)
    assert_allclose(lp[fin], d["log_prob"][fin], rtol=1e-6, atol=1e-6)


def test_inverse_fixture():
    d = np.load(G / "flow_cfg3_inverse.npz")
    meta = json.loads(str(d["meta"]))
    case = make_case(meta["name"], N=int(meta["N"]), seed=int(meta["seed"]))
    z = (0.5 + 0.1 * np.random.default_rng(int(meta["z_seed"])).standard_normal((int(meta["N"]), 4)))
    assert np.array_equal(z.astype(np.float32), d["z"])
    x = O.flow_inverse(case["model"], case["variables"], d["z"], None)
    assert_allclose(x, d["x"], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg4"])
def test_edge_fixture(name):
    """NaN / clipped-edge rows: the oracle reproduces finfo.min for them and
    the infinite NLL of the batch (flow.py:47, train.py:78)."""
    d = np.load(G / f"flow_edges_{name}.npz")
    meta = json.loads(str(d["meta"]))
    case = make_case(meta["name"], N=int(meta["N"]), seed=int(meta["seed"]))
    c = d["c"] if "c" in d.files else None
    lp, _ = O.flow_log_prob(case["model"], case["variables"], d["x"], c)
    edge = np.abs(d["log_prob"]) >= 1e38
    assert np.isnan(d["x"][:2]).any(axis=1).all() and edge[:2].all()
    assert np.array_equal(lp[edge], d["log_prob"][edge])
    assert (lp[edge] == np.finfo(np.float32).min).all()
    assert_allclose(lp[~edge], d["log_prob"][~edge], rtol=1e-6, atol=1e-6)
    assert O.nll(lp) == float(d["nll"]) == np.inf


def test_jnp_nan_to_num_semantics():
    """JAX's where chain: masks from the running result, so NaN -> -inf ->
    finfo.min (NumPy's np.nan_to_num would leave -inf)."""
    f = np.finfo(np.float32)
    x = np.array([np.nan, np.inf, -np.inf, 1.5, -2.0], np.float32)
    out = O.jnp_nan_to_num(x, nan=-np.inf)
    assert out.dtype == np.float32
    assert out.tolist() == [f.min, f.max, f.min, 1.5, -2.0]
    assert np.nan_to_num(x, nan=-np.inf)[0] == -np.inf  # the semantics we do NOT follow
    assert O.jnp_nan_to_num(x, nan=0.0).tolist() == [0.0, f.max, f.min, 1.5, -2.0]


def test_nll_fp32_overflow():
    """-jnp.mean sums in fp32: one finfo.min row stays finite, two overflow."""
    from zenflow_amd.dist import nll_from_sum

    f = float(np.finfo(np.float32).min)
    for fn in (O.nll_from_sum, nll_from_sum):
        assert np.isfinite(fn(f - 10.0, 4))
        assert fn(2 * f, 4) == np.inf
        assert fn(-2 * f, 4) == -np.inf
        assert np.isnan(fn(np.nan, 4))
        assert fn(-8.0, 4) == 2.0
