"""Pins the gradient oracle (oracle/zf_oracle_torch.py, torch float64
autograd of the train-mode loss) to the NumPy oracle: the same loss value
(fp64, 1e-12) and per-parameter derivatives equal to central differences of
the NumPy oracle's fp64 loss.  CPU only."""

import numpy as np
import pytest

from oracle import zf_oracle as O
from oracle import zf_oracle_torch as OT
from tests.flowcases import make_case


def _np_loss(case, variables):
    x = case["x"].astype(np.float64)
    c = None if case["c"] is None else case["c"].astype(np.float64)
    lp, _ = O.flow_log_prob(case["model"], variables, x, c, train=True, dtype=np.float64)
    return -lp.mean()


@pytest.mark.parametrize("name", ["small", "cfg2", "cfg4", "odd", "relu", "gelu", "tanh", "softplus", "sigmoid", "elu",
                                  "leaky_relu"])
def test_torch_loss_equals_numpy_oracle(name):
    case = make_case(name, N=256, seed=71)
    loss, _ = OT.train_loss_and_grad(case["model"], case["variables"], case["x"], case["c"])
    assert loss == pytest.approx(_np_loss(case, case["variables"]), rel=1e-12, abs=1e-12)


@pytest.mark.parametrize("name", ["small", "cfg4", "gelu", "elu"])
def test_torch_grad_matches_central_differences(name):
    case = make_case(name, N=64, seed=72)
    _, g = OT.train_loss_and_grad(case["model"], case["variables"], case["x"], case["c"])
    rng = np.random.default_rng(0)
    params = case["variables"]["params"]["bijector"]
    checked = 0
    for key in sorted(params):
        for mod in sorted(params[key]):
            for leaf in sorted(params[key][mod]):
                arr = params[key][mod][leaf]
                for flat in rng.choice(arr.size, size=min(3, arr.size), replace=False):
                    i = np.unravel_index(flat, arr.shape)
                    old = arr[i]
                    h = 1e-5 * max(1e-2, abs(float(old)))  # small: elu and relu are only C1 / C0
                    vals = []
                    for s in (+1, -1):
                        arr[i] = np.float32(old + s * h)
                        hh = float(arr[i]) - float(old)
                        vals.append((_np_loss(case, case["variables"]), hh))
                    arr[i] = old
                    fd = (vals[0][0] - vals[1][0]) / (vals[0][1] - vals[1][1])
                    an = g["bijector"][key][mod][leaf][i]
                    assert abs(an - fd) <= 1e-4 * abs(fd) + 1e-7, f"{key}/{mod}/{leaf}{i}: {an} vs {fd}"
                    checked += 1
    assert checked > 20
