"""Gradient diagnostics: analytic (GPU trainer) vs central finite differences
of the fp64 oracle loss, per parameter group and step size."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tests.test_gpu_train import _direction, _oracle_loss, _setup  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
case, flow, tr = _setup(name, 512, 62)
prog = tr.program
_, g = tr.loss_grad(case["x"], case["c"])
rng = np.random.default_rng(0)
nsc = [i for i, op in enumerate(prog.ops) if op.kind == 3]
groups = {}
for ci, i in enumerate(nsc):
    d = prog.desc.ops[i]
    DC = prog.D - prog.D // 2 + prog.C
    nh = d.n_hidden
    S = 3 * d.knots - 1
    spans = {"bn": (d.off_bn + 2 * DC, d.off_bn + 4 * DC)}
    for l in range(nh + 1):
        out = d.hidden[l] if l < nh else (prog.D // 2) * S
        spans[f"W{l}"] = (d.off_w[l], d.off_b[l])
        spans[f"b{l}"] = (d.off_b[l], d.off_b[l] + out)
    for k, (a, b) in spans.items():
        sel = np.zeros(prog.blob.shape)
        sel[a:b] = 1
        groups[f"c{ci}.{k}"] = sel
for label, sel in groups.items():
    v = _direction(prog, rng, sel)
    an = float(np.dot(g.astype(np.float64), v))
    fds = []
    for eps in (1e-2, 1e-3, 1e-4):
        lp_, _ = _oracle_loss(case, prog, prog.blob + eps * v)
        lm_, _ = _oracle_loss(case, prog, prog.blob - eps * v)
        fds.append((lp_ - lm_) / (2 * eps))
    rel = abs(an - fds[2]) / max(1e-12, abs(fds[2]))
    print(f"{label:12s} analytic {an:+.6e}  fd(1e-2,1e-3,1e-4) {fds[0]:+.6e} {fds[1]:+.6e} {fds[2]:+.6e}  rel {rel:.2e}")
