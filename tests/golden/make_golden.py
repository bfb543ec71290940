"""Generate the committed golden fixtures under tests/golden/ from the fp32 CPU
oracle (itself pinned by tests/test_oracle_kats.py against the reference's
known-answer tests).  Run: ``python tests/golden/make_golden.py``.

* rqs_K{8,16,32}.npz — utils.rational_quadratic_spline_{forward,inverse}
  inputs/outputs (M=2048, N=2, logits with sigma in {0.1, 1, 3}, x incl. OOB);
* flow_<cfg>.npz — Flow.log_prob for BASELINE configs at small N, with the
  case metadata (inputs are regenerated from the seed and checked equal);
* flow_cfg3_inverse.npz — config 3 (the cfg2 flow run backwards, Chain.inverse
  as in Flow.sample): z = 0.5 + 0.1 N(0, 1) -> x, fp32 and fp64 oracle.
"""

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle import zf_oracle as O  # noqa: E402
from tests.flowcases import make_case  # noqa: E402

OUT = Path(__file__).resolve().parent


def rqs_fixtures():
    for K in (8, 16, 32):
        rng = np.random.default_rng(K)
        M, N = 512, 2
        sig = rng.choice([0.1, 1.0, 3.0], size=(M, 1, 1)).astype(np.float32)
        dx = (sig * rng.standard_normal((M, N, K))).astype(np.float32)
        dy = (sig * rng.standard_normal((M, N, K))).astype(np.float32)
        sl = (sig * rng.standard_normal((M, N, K - 1))).astype(np.float32)
        dx, dy, sl = O.normalize_spline_params(dx, dy, sl)
        x = rng.uniform(-0.1, 1.1, size=(M, N)).astype(np.float32)
        y, ld = O.rqs_forward(x, dx, dy, sl)
        xi = O.rqs_inverse(y, dx, dy, sl)
        np.savez_compressed(OUT / f"rqs_K{K}.npz", x=x, dx=dx, dy=dy, slope=sl, y=y, log_det=ld, x_inv=xi)


def flow_fixtures():
    for name, N, seed in [("cfg1", 1024, 101), ("cfg2", 1024, 102), ("cfg4", 1024, 104), ("cfg5", 256, 105)]:
        case = make_case(name, N=N, seed=seed)
        lp, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"])
        lp64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
        meta = json.dumps({"name": name, "N": N, "seed": seed})
        sens = O.row_sensitivity(case["model"], case["variables"], case["x"], case["c"])
        np.savez_compressed(OUT / f"flow_{name}.npz", x=case["x"], log_prob=lp, log_prob64=lp64,
                            sensitivity=sens, meta=np.array(meta))


def inverse_fixture():
    name, N, seed = "cfg2", 1024, 103
    case = make_case(name, N=N, seed=seed)
    z = (0.5 + 0.1 * np.random.default_rng(4).standard_normal((N, 4))).astype(np.float32)
    x = O.flow_inverse(case["model"], case["variables"], z, None)
    x64 = O.flow_inverse(case["model"], case["variables"], z.astype(np.float64), None, dtype=np.float64)
    meta = json.dumps({"name": name, "N": N, "seed": seed, "z_seed": 4})
    np.savez_compressed(OUT / "flow_cfg3_inverse.npz", z=z, x=x, x64=x64, meta=np.array(meta))


def edge_fixtures():
    """flow_edges_<cfg>.npz: flow.py:47 on NaN rows and on rows clipped to the
    ShiftBounds edges.  jnp.nan_to_num(nan=-inf) maps NaN -> -inf -> finfo.min
    and a Beta latent at its support edge (z == 1 after the clip) gives -inf ->
    finfo.min; with two or more such rows the fp32 NLL sum overflows (inf)."""
    for name, seed in [("cfg1", 201), ("cfg2", 202), ("cfg4", 204)]:
        N = 64
        case = make_case(name, N=N, seed=seed)
        x = case["x"].copy()
        sb = case["variables"]["batch_stats"]["bijector"]["bijectors_0"]
        D = x.shape[1]
        xmin = np.array([sb[f"xmin_{i}"][0] for i in range(D)], np.float32)
        xmax = np.array([sb[f"xmax_{i}"][0] for i in range(D)], np.float32)
        x[0, 0] = np.nan
        x[1, :] = np.nan
        x[2, :] = 1e30  # clips to z = 1 in every dim
        x[3, :] = -1e30  # clips to z = 0
        x[4, :] = xmax
        x[5, :] = xmin
        x[6, :] = np.inf
        x[7, :] = -np.inf
        x[8, -1] = np.nan  # NaN in a conditioning column only
        lp, _ = O.flow_log_prob(case["model"], case["variables"], x, case["c"])
        fin = np.abs(lp) < 1e38
        meta = json.dumps({"name": name, "N": N, "seed": seed})
        extra = {} if case["c"] is None else {"c": case["c"]}
        np.savez_compressed(OUT / f"flow_edges_{name}.npz", x=x, log_prob=lp, nll=np.float64(O.nll(lp)),
                            nll_finite=np.float64(O.nll(lp[fin])), meta=np.array(meta), **extra)


if __name__ == "__main__":
    rqs_fixtures()
    flow_fixtures()
    inverse_fixture()
    edge_fixtures()
    for f in sorted(OUT.glob("*.npz")):
        print(f.name, f.stat().st_size)
