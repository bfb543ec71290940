"""Train the BASELINE flows with ``zenflow_amd.train`` and write TRAINED
variables as fixtures, so the kernel parity tests also run on weights that
training produced (not only on lecun-initialised ones).  Needs the GPU:

    python tests/golden/make_trained.py [OUTDIR]     (default gpurun_out/trained)

then copy ``trained_<cfg>.npz`` (FLAX-path variables, zenflow_amd.io format)
and ``trained_<cfg>_data.npz`` (held-out inputs x[, c] and the training
curve) into tests/golden/.

* cfg1  two_moons (examples/two_moons.ipynb): make_moons(10_000, noise=0.1,
  random_state=1), D=2, K=8, Beta latent.
* cfg4  two_moons_conditional with a 2-D condition (one-hot class label;
  examples/two_moons_conditional.ipynb uses the 1-D label), K=16, Beta latent.
* cfg2  4-D, K=16, Normal latent, on a skewed correlated synthetic sample.
"""

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from tests.flowcases import CONFIGS, build_flow  # noqa: E402


def data(name):
    if name in ("cfg1", "cfg4"):
        from sklearn.datasets import make_moons

        X, lab = make_moons(10_000, noise=0.1, random_state=1)
        X = X.astype(np.float32)
        C = np.eye(2, dtype=np.float32)[lab] if name == "cfg4" else None
    else:
        rng = np.random.default_rng(5)
        A = rng.standard_normal((4, 4)).astype(np.float32)
        z = rng.standard_normal((20_000, 4)).astype(np.float32)
        X = (z @ A).astype(np.float32)
        X[:, 0] = np.exp(0.5 * X[:, 0])  # skewed marginal
        X[:, 2] = np.tanh(X[:, 2]) + 0.1 * X[:, 3]
        C = None
    n = X.shape[0] * 4 // 5
    return X[:n], X[n:], (None if C is None else C[:n]), (None if C is None else C[n:])


def main(out):
    import zenflow_amd as zf

    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    for name, epochs in [("cfg1", 60), ("cfg4", 60), ("cfg2", 40)]:
        cfg = CONFIGS[name]
        flow = build_flow(cfg)
        Xtr, Xte, Ctr, Cte = data(name)
        var, best, ltr, lte = zf.train(flow, Xtr, Xte, Ctr, Cte, epochs=epochs, batch_size=512,
                                       progress=False, seed=0)
        steps = epochs * -(-Xtr.shape[0] // 512)
        print(f"{name}: {steps} steps, best epoch {best}, test NLL {lte[0]:.4f} -> {lte[best]:.4f}", flush=True)
        zf.save_variables(out / f"trained_{name}.npz", var)
        meta = json.dumps({"name": name, "epochs": epochs, "batch_size": 512, "best_epoch": int(best),
                           "steps": int(steps)})
        extra = {} if Cte is None else {"c": Cte[:4096]}
        np.savez_compressed(out / f"trained_{name}_data.npz", x=Xte[:4096], loss_train=np.asarray(ltr),
                            loss_test=np.asarray(lte), meta=np.array(meta), **extra)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out" / "trained")
