"""Training on the GPU (zenflow.train, train.py:18-138).

* loss_fn (train.py:64-72) value and batch-statistics update vs the fp64
  oracle in train mode;
* its gradient (jax.grad) vs central finite differences of the fp64 oracle
  loss along random parameter directions — all parameters, and per group
  (BatchNorm, first / hidden / last Dense of one coupling) to localise errors;
* one optimiser step vs optax's nadamw / adamw update formula;
* train() end to end: same return structure as the reference, loss falls.
optax itself is not installable here: its update is restated from the
published algorithm (parity unpinned beyond that)."""

import numpy as np
import pytest

from oracle import zf_oracle as O
from tests.flowcases import build_flow, make_case

pytestmark = pytest.mark.gpu


def _setup(name, N, seed, **kw):
    from zenflow_amd.train import Trainer

    case = make_case(name, N=N, seed=seed)
    cfg = case["cfg"]
    flow = build_flow(cfg)
    flow.latent._dim = cfg["D"]
    tr = Trainer(flow, case["variables"], cfg["D"], cfg["C"], N, **kw)
    return case, flow, tr


def _oracle_loss(case, prog, blob):
    v = prog.blob_to_variables(blob)
    variables = {"params": {"bijector": v["params"]}, "batch_stats": {"bijector": v["batch_stats"]}}
    x = case["x"].astype(np.float64)
    c = None if case["c"] is None else case["c"].astype(np.float64)
    lp, ns = O.flow_log_prob(case["model"], variables, x, c, train=True, dtype=np.float64)
    return -lp.mean(), ns


CASES = [("small", 128, 61), ("cfg2", 128, 62), ("cfg4", 128, 63)]


@pytest.mark.parametrize("name,N,seed", CASES)
def test_train_loss_and_stats(name, N, seed):
    case, flow, tr = _setup(name, N, seed)
    prog = tr.program
    loss, _ = tr.loss_grad(case["x"], case["c"], update_stats=True)
    ref, ns = _oracle_loss(case, prog, prog.blob)
    assert loss == pytest.approx(ref, rel=2e-5, abs=2e-5)
    # running statistics after one train-mode pass == the oracle's new batch_stats
    got = tr.variables()["batch_stats"]["bijector"]
    for k, sub in ns.items():
        for name2, leaf in sub.items():
            if isinstance(leaf, dict):
                for kk, vv in leaf.items():
                    np.testing.assert_allclose(got[k][name2][kk], vv, rtol=2e-5, atol=1e-6)
            else:
                np.testing.assert_allclose(got[k][name2], leaf, rtol=2e-5, atol=1e-6)


def _direction(prog, rng, select=None):
    v = rng.standard_normal(prog.blob.shape) * prog.param_mask
    if select is not None:
        v = v * select
    scale = np.abs(prog.blob[prog.param_mask == 1]).mean() + 1e-3
    return v * scale / max(1e-12, np.linalg.norm(v) / np.sqrt(max(1, (v != 0).sum())))


@pytest.mark.parametrize("name,N,seed", CASES)
def test_train_gradient_directional(name, N, seed):
    case, flow, tr = _setup(name, N, seed)
    prog = tr.program
    _, g = tr.loss_grad(case["x"], case["c"])
    assert np.all(g[prog.param_mask == 0] == 0)
    rng = np.random.default_rng(seed)
    # parameter groups of the first coupling (natural blob offsets)
    groups = {"all": None}
    nsc = [i for i, op in enumerate(prog.ops) if op.kind == 3]
    d = prog.desc.ops[nsc[0]]
    DC = prog.D - prog.D // 2 + prog.C
    nh = d.n_hidden
    for label, (a, n) in {
        "bn": (d.off_bn + 2 * DC, 2 * DC),
        "dense0": (d.off_w[0], d.off_b[0] + prog.desc.ops[nsc[0]].hidden[0] - d.off_w[0]),
        "dense_last": (d.off_w[nh], 0),
    }.items():
        sel = np.zeros(prog.blob.shape)
        end = a + n if n else (d.off_b[nh] + (prog.D // 2) * (3 * d.knots - 1))
        sel[a:end] = 1
        groups[label] = sel
    # The loss is only piecewise smooth in the parameters: a row whose input
    # crosses a knot switches bins, where the parameter gradient jumps.  A
    # central difference over a step that moves some rows across knots is
    # off by O(rows crossed); over three step sizes at least one is clean.
    for label, sel in groups.items():
        for rep in range(2):
            v = _direction(prog, rng, sel)
            an = float(np.dot(g.astype(np.float64), v))
            fds = []
            for eps in (1e-3, 3e-4, 1e-4):
                lp_, _ = _oracle_loss(case, prog, prog.blob + eps * v)
                lm_, _ = _oracle_loss(case, prog, prog.blob - eps * v)
                fds.append((lp_ - lm_) / (2 * eps))
            err = min(abs(an - fd) for fd in fds)
            assert err <= 2e-3 * abs(an) + 2e-6, f"{name}/{label}: analytic {an} vs fd {fds}"


def _leaves(tree, path=()):
    if isinstance(tree, dict):
        for k in sorted(tree):
            yield from _leaves(tree[k], path + (k,))
    else:
        yield path, np.asarray(tree, np.float64)


def _get(tree, path):
    for k in path:
        tree = tree[k]
    return np.asarray(tree, np.float64)


GRAD_CASES = CASES + [("cfg1", 1024, 66), ("d8", 512, 67), ("d2h256", 256, 68), ("odd", 300, 69),
                      ("relu", 256, 70), ("gelu", 256, 71), ("tanh", 256, 72), ("softplus", 256, 73),
                      ("sigmoid", 256, 74), ("elu", 256, 75), ("leaky_relu", 256, 76), ("mixed", 256, 77),
                      # a batch whose forward Dense layers run the bf16x3 split-MFMA GEMM (>= 512 128x128 tiles)
                      ("cfg2", 65536, 79), ("cfg5", 32768, 78),
                      # hidden 512 / 384 (the eval path for these widths is the layered one)
                      ("h512", 256, 83), ("h384c2", 256, 84)]


@pytest.mark.parametrize("name,N,seed", GRAD_CASES)
def test_train_gradient_per_parameter(name, N, seed):
    """jax.grad of loss_fn (train.py:64-72, 82) per parameter: the GPU
    trainer's fp32 reverse pass vs float64 autograd of the oracle's loss
    (oracle/zf_oracle_torch.py).  Every element of every parameter tensor:
    |g_gpu - g64| <= 1e-5 * max|g64| + 2 max(|g32 - g64|, |g64' - g64|)
    (maxima over that tensor), where g32 is the same autograd in float32 over
    three row orders of the batch (the rounding of the batch sums any fp32
    evaluation, the reference's included, is subject to) and g64' the
    float64 gradient at inputs and parameters jittered by ~4 fp32 ulp (its
    conditioning: how far another fp32 per-row arithmetic can land)."""
    import subprocess
    import sys
    import tempfile
    from pathlib import Path

    case, flow, tr = _setup(name, N, seed)
    _, g = tr.loss_grad(case["x"], case["c"])
    gg = tr.grad_tree(g)
    # the autograd oracle runs in a CPU-only child (tests/grad_oracle.py)
    root = Path(__file__).resolve().parents[1]
    with tempfile.TemporaryDirectory() as d:
        out = Path(d) / "g.npz"
        subprocess.run([sys.executable, "-m", "tests.grad_oracle", name, str(N), str(seed), str(out)], cwd=root,
                       check=True, timeout=600)
        ref = dict(np.load(out))
    worst, bad = {}, []
    for key in sorted(k for k in ref if k.startswith("g64:")):
        path = tuple(key[4:].split("/"))
        r64 = ref[key]
        got = _get(gg, path)
        assert got.shape == r64.shape, path
        scale = max(np.abs(r64).max(), 1e-30)
        e = np.abs(got - r64)
        e32 = max(np.abs(ref[f"g32_{k}:" + key[4:]] - r64).max() for k in range(3))
        cond = max(np.abs(ref[f"g64p_{k}:" + key[4:]] - r64).max() for k in range(2))
        ok = e <= 1e-5 * scale + 2 * max(e32, cond)
        worst["/".join(path)] = (float(e.max() / scale), float(e32 / scale), float(cond / scale))
        if not ok.all():
            bad.append(f"{'/'.join(path)}: {np.sum(~ok)} of {ok.size} over, max rel {e.max() / scale:.3g} "
                       f"(fp32 autograd {e32 / scale:.3g}, conditioning {cond / scale:.3g})")
    rel = max(v[0] for v in worst.values())
    rel32 = max(v[1] for v in worst.values())
    relc = max(v[2] for v in worst.values())
    from tests.test_gpu_flow import _append_record

    _append_record("grad_parity.jsonl", {"case": name, "rows": N, "leaves": len(worst),
                                         "gpu_max_rel_err_vs_fp64": rel, "torch32_max_rel_err_vs_fp64": rel32,
                                         "conditioning_max_rel": relc,
                                         "over": bad})
    assert not bad, bad


@pytest.mark.parametrize("nesterov", [True, False])
def test_optimizer_step_matches_optax_formula(nesterov):
    from zenflow_amd.train import Optimizer

    opt = Optimizer(learning_rate=1e-2, nesterov=nesterov)
    case, flow, tr = _setup("small", 256, 64, optimizer=opt)
    prog = tr.program
    _, g = tr.loss_grad(case["x"], case["c"])
    theta0 = prog.blob.astype(np.float64)
    tr.step(case["x"], case["c"])
    v1 = tr.variables()
    theta1 = prog.blob.copy()
    # rebuild the stepped blob from the returned variables
    from zenflow_amd.engine import Program

    p1 = Program(flow.bijector, {k: vv["bijector"] for k, vv in v1.items()}, prog.D, prog.C, latent=flow.latent)
    theta1 = p1.blob.astype(np.float64)
    m = (1 - opt.b1) * g
    vv = (1 - opt.b2) * g.astype(np.float64) ** 2
    if nesterov:
        mhat = opt.b1 * m / (1 - opt.b1**2) + (1 - opt.b1) * g / (1 - opt.b1)
    else:
        mhat = m / (1 - opt.b1)
    vhat = vv / (1 - opt.b2)
    expect = theta0 - opt.learning_rate * (mhat / (np.sqrt(vhat) + opt.eps) + opt.weight_decay * theta0)
    mask = prog.param_mask == 1
    np.testing.assert_allclose(theta1[mask], expect[mask], rtol=1e-4, atol=1e-6)


def test_train_end_to_end_two_moons():
    """zenflow.train on a two-moons sample (examples/two_moons.ipynb shape):
    returns (best_variables, best_epoch, loss_train, loss_test); the test
    loss falls well below its first-epoch value."""
    from sklearn.datasets import make_moons

    import zenflow_amd as zf
    from zenflow_amd import bijectors as bi
    from zenflow_amd import distributions as dist

    X, _ = make_moons(4000, noise=0.05, random_state=1)
    X = X.astype(np.float32)
    flow = zf.Flow(bi.rolling_spline_coupling(2, knots=8, layers=(64, 64)), latent=dist.Beta())
    # epochs=40: patience = int(0.05 * 40) = 2 (with fewer than 20 epochs the
    # reference's `epoch % patience` divides by zero, train.py:129-131)
    best, best_epoch, lt, ls = zf.train(flow, X[:3000], X[3000:], epochs=40, batch_size=256, progress=False)
    assert len(lt) == len(ls) and 8 < len(ls) <= 40 and 0 <= best_epoch < len(ls)
    assert np.all(np.isfinite(ls))
    assert min(ls) < ls[0] - 0.3
    lp = flow.apply(best, X[3000:])
    assert np.isfinite(lp).mean() > 0.99
    assert -lp.mean() == pytest.approx(ls[best_epoch], rel=1e-5)


def test_step_graph_matches_eager(monkeypatch):
    """zf_trainer_step replays one captured hipGraph per batch size; the
    graph and the eagerly launched step give bit-identical parameters (every
    reduction has a fixed order), including a ragged last batch."""
    from zenflow_amd.io import flatten_variables
    from zenflow_amd.train import Trainer

    flat = []
    losses = []
    for graph in ("1", "0"):
        monkeypatch.setenv("ZF_TRAIN_GRAPH", graph)
        case, flow, _ = _setup("cfg4", 300, 65)
        tr = Trainer(flow, case["variables"], 2, 2, 256)
        x, c = case["x"], case["c"]
        for _ in range(3):
            tr.step(x[:256], c[:256])
            tr.step(x[256:], c[256:])
        losses.append(tr.last_loss())
        flat.append(flatten_variables(tr.variables()))
    assert losses[0] == losses[1]
    assert flat[0].keys() == flat[1].keys()
    for k in flat[0]:
        np.testing.assert_array_equal(flat[0][k], flat[1][k], err_msg=k)


@pytest.mark.parametrize("name,N,seed", [("cfg2", 1024, 66), ("d2h256", 2048, 67), ("gelu", 512, 68), ("cfg4", 300, 69),
                                         ("cfg1", 65536, 70)])
def test_split_set_gemm_matches_single_kernel(name, N, seed, monkeypatch):
    """Small batches run the 64x64 GEMM tiles as four blocks, one per
    accumulator set of the interleaved kernel, plus a combine (SPLITQ in
    zf_train.hip): the same loss, gradient and trained parameters, bit for
    bit, as the single-kernel form (ZF_TRAIN_SPLITQ=0).  At 65536 rows the
    first Dense runs one thread per output under either setting (ADVICE r4:
    the switch names the small-batch forms only)."""
    from zenflow_amd import _lib as L

    out = []
    for sq in ("1", "0"):
        monkeypatch.setenv("ZF_TRAIN_SPLITQ", sq)
        case, flow, tr = _setup(name, N, seed)
        loss, g = tr.loss_grad(case["x"], case["c"])
        for _ in range(2):
            tr.step(case["x"], case["c"])
        blob = np.empty_like(tr.program.blob)
        L.check(L.load_library().zf_trainer_get_blob(tr.handle, blob.ctypes.data), "get_blob")
        out.append((loss, g, tr.last_loss(), blob))
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1]), f"{np.sum(out[0][1] != out[1][1])} gradient entries differ"
    assert out[0][2] == out[1][2]
    assert np.array_equal(out[0][3], out[1][3], equal_nan=True)


@pytest.mark.parametrize("name,N,seed", [("cfg2", 65536, 80), ("d2h256", 65536, 81)])
def test_train_x3_gemm_matches_fp32_gemm(name, N, seed, monkeypatch):
    """Large batches run the forward Dense layers on the bf16x3 split-MFMA
    GEMM (gemm_x3_kernel): loss and every gradient element within 1e-5 of
    the tensor's scale of the fp32-MFMA GEMM's (ZF_TRAIN_X3=0) — two fp32
    evaluations of the same sums in different orders.  (Deeper flows, whose
    gradients amplify a forward rounding difference further, are held to
    float64 autograd with their conditioning instead: cfg5 in GRAD_CASES.)"""
    case, flow, tr = _setup(name, N, seed)
    loss_x3, g_x3 = tr.loss_grad(case["x"], case["c"])
    monkeypatch.setenv("ZF_TRAIN_X3", "0")
    import subprocess
    import sys
    code = (
        "import numpy as np, sys; sys.path.insert(0, '.');"
        "from tests.test_gpu_train import _setup;"
        f"case, flow, tr = _setup({name!r}, {N}, {seed});"
        "l, g = tr.loss_grad(case['x'], case['c']);"
        "np.savez(sys.argv[1], l=np.float64(l), g=g)")
    from pathlib import Path
    import tempfile
    root = Path(__file__).resolve().parents[1]
    with tempfile.TemporaryDirectory() as d:
        out = Path(d) / "ref.npz"
        subprocess.run([sys.executable, "-c", code, str(out)], cwd=root, check=True, timeout=300)
        ref = np.load(out)
        loss_32, g_32 = float(ref["l"]), ref["g"]
    assert abs(loss_x3 - loss_32) <= 1e-5 * max(1.0, abs(loss_32))
    scale = np.abs(g_32).max()
    assert np.abs(g_x3 - g_32).max() <= 1e-5 * scale, np.abs(g_x3 - g_32).max() / scale
