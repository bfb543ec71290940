"""Diagnose 2-rank vs 1-device trainer differences: python scripts/diag_dp.py NAME N SEED"""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from tests.test_gpu_train import _setup, _leaves, _get  # noqa: E402
from zenflow_amd.launch import spawn  # noqa: E402

name, N, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
d = tempfile.mkdtemp()
env = dict(os.environ, ZF_TEST_CASE=f"{name}:{N}:{seed}", ZF_TEST_STEPS="0")
assert spawn(2, [str(ROOT / "tests/dist_worker.py"), "train_dp", d], env=env, timeout=240) == 0
r = np.load(Path(d) / "rank0.npz")
case, flow, tr = _setup(name, N, seed)
loss, g = tr.loss_grad(case["x"], case["c"])
os.environ["ZF_TRAIN_BN_SMALL"] = "0"
_, _, trb = _setup(name, N, seed)
_, gb = trb.loss_grad(case["x"], case["c"])
print("1dev small vs 1dev big: differing entries", int(np.sum(g != gb)), "big vs dp", int(np.sum(gb != r["grad"])))
print("loss 1dev", repr(loss), "dp", repr(float(r["loss"])))
t1 = tr.grad_tree(g)
t2 = tr.grad_tree(r["grad"])
for path, a in _leaves(t1):
    b = _get(t2, path)
    nd = int(np.sum(a != b))
    if nd:
        print("/".join(path), nd, "of", a.size, "max rel", float(np.max(np.abs(a - b)) / max(1e-30, np.abs(a).max())))
