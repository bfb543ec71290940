"""Gradient-oracle worker for tests/test_gpu_train.py: float64 autograd of
the train-mode loss (oracle/zf_oracle_torch.py), float32 autograd over
three row orders, and float64 autograd at inputs and parameters jittered by
~4 fp32 ulp (the gradient's conditioning), for one tests/flowcases case,
into an .npz.  Runs in its
own CPU-only process: importing torch (which bundles its own HIP runtime and
RCCL) into the GPU test process would shadow the system librccl there.

    python -m tests.grad_oracle NAME N SEED OUT.npz"""

import os
import sys

os.environ["HIP_VISIBLE_DEVICES"] = ""  # this process never touches the GPU

import numpy as np  # noqa: E402


def _flat(tree, path=()):
    if isinstance(tree, dict):
        for k in sorted(tree):
            yield from _flat(tree[k], path + (k,))
    else:
        yield "/".join(path), np.asarray(tree, np.float64)


def main(name, N, seed, out):
    import torch

    from oracle import zf_oracle_torch as OT
    from tests.flowcases import make_case

    case = make_case(name, N=N, seed=seed)
    x, c = case["x"], case["c"]
    res = {}
    _, g64 = OT.train_loss_and_grad(case["model"], case["variables"], x, c, torch.float64)
    for k, v in _flat(g64):
        res["g64:" + k] = v
    for r in range(3):
        p = np.random.default_rng(r).permutation(N) if r else np.arange(N)
        _, g32 = OT.train_loss_and_grad(case["model"], case["variables"], x[p], None if c is None else c[p],
                                        torch.float32)
        for k, v in _flat(g32):
            res[f"g32_{r}:" + k] = v
    # conditioning: float64 autograd with ~4 fp32 ulp of relative noise on
    # every input and parameter (as oracle.row_sensitivity does for log_prob)
    import copy

    for r in range(2):
        rng = np.random.default_rng(100 + r)
        v = copy.deepcopy(case["variables"])

        def jitter(tree):
            for k in tree:
                if isinstance(tree[k], dict):
                    jitter(tree[k])
                else:
                    a = np.asarray(tree[k], np.float64)
                    tree[k] = a * (1 + 2.0**-22 * rng.standard_normal(a.shape))

        jitter(v["params"])
        xp = x.astype(np.float64) * (1 + 2.0**-22 * rng.standard_normal(x.shape))
        _, gp = OT.train_loss_and_grad(case["model"], v, xp, c, torch.float64)
        for k, val in _flat(gp):
            res[f"g64p_{r}:" + k] = val
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
