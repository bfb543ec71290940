"""Shared test cases: flow configurations (BASELINE.json configs), FLAX-layout
variables and synthetic inputs, built without touching the product code.

``make_case`` returns the oracle model spec, the variables pytree (exactly the
tree FLAX would hold for ``Flow(rolling_spline_coupling(D, ...))``) and
seeded inputs.  The GPU tests build the matching zenflow_amd module with
``build_flow`` and feed it the same variables."""

from __future__ import annotations

import numpy as np

# BASELINE.json configs; N here is the test size.
CONFIGS = {
    "cfg1": dict(D=2, C=0, K=8, layers=(128, 128), latent="beta"),  # two_moons
    "cfg2": dict(D=4, C=0, K=16, layers=(128, 128), latent="normal"),  # 4D fwd / inv
    "cfg4": dict(D=2, C=2, K=16, layers=(128, 128), latent="beta"),  # two_moons_conditional
    "cfg4c1": dict(D=2, C=1, K=16, layers=(128, 128), latent="beta"),  # ref NB: 1-D label
    "cfg5": dict(D=16, C=0, K=32, layers=(256, 256), latent="normal", couplings=8),
    "small": dict(D=3, C=0, K=5, layers=(64, 64), latent="normal"),
    "odd": dict(D=5, C=3, K=7, layers=(48, 96, 32), latent="truncated_normal"),
    "uniform": dict(D=2, C=0, K=4, layers=(32,), latent="uniform"),
    "deep": dict(D=2, C=8, K=16, layers=(128,) * 6, latent="beta"),  # deep_set NB shape
    # one transformed dim on the split-MFMA kernel's one-dim last-layer layout:
    # hidden 128 with dc = 2 and a condition; hidden 256 (dim-pair path)
    "d3c1": dict(D=3, C=1, K=16, layers=(128, 128), latent="normal"),
    "d2h256": dict(D=2, C=0, K=32, layers=(256, 256), latent="normal"),
    # the reference defaults rolling_spline_coupling(dim, knots=16, layers=(128, 128))
    # at dim >= 6 (dim-pair loop at hidden 128), K = 32 at hidden 128, K = 8 at
    # hidden 256, hidden 64 (padded to 128 on the split-MFMA kernel)
    "d6": dict(D=6, C=0, K=16, layers=(128, 128), latent="normal"),
    "d8": dict(D=8, C=0, K=16, layers=(128, 128), latent="normal"),
    "d16": dict(D=16, C=0, K=16, layers=(128, 128), latent="normal"),
    "d7k32c2": dict(D=7, C=2, K=32, layers=(128, 128), latent="truncated_normal", couplings=4),
    "d4k32": dict(D=4, C=0, K=32, layers=(128, 128), latent="normal"),
    "d3k32": dict(D=3, C=0, K=32, layers=(128, 96), latent="beta"),
    "d4h256k8": dict(D=4, C=1, K=8, layers=(256, 256), latent="normal"),
    "d5h64": dict(D=5, C=0, K=16, layers=(64, 64), latent="normal"),
    # knot counts between the instantiated 8 / 16 / 32: the split-MFMA kernel
    # pads them with inert knots (x3_padded_knots; 15 -> 32, 7 -> 16)
    "k12": dict(D=4, C=0, K=12, layers=(128, 128), latent="normal"),
    "k5c1": dict(D=3, C=1, K=5, layers=(128, 128), latent="beta"),
    "k15": dict(D=4, C=0, K=15, layers=(128, 128), latent="normal"),
    "k24h256": dict(D=6, C=0, K=24, layers=(256, 256), latent="normal", couplings=3),
    "k3": dict(D=2, C=0, K=3, layers=(64, 64), latent="normal"),
    # round 5: one padded knot (K = 7 / 15 / 31 on the 8 / 16 /
    # 32 instantiations: the sliver starts at the padded knot), 33..64 knots on the
    # K = 64 instantiation (one wave per SIMD), knots above 64 on the layered
    # path, and a chain mixing knot counts (every coupling at the largest one's
    # instantiation, each with its own knot constants)
    "k7": dict(D=4, C=0, K=7, layers=(128, 128), latent="normal"),
    "k31": dict(D=4, C=0, K=31, layers=(128, 128), latent="normal"),
    "k40": dict(D=4, C=0, K=40, layers=(128, 128), latent="normal"),
    "k64": dict(D=4, C=0, K=64, layers=(128, 128), latent="normal"),
    "k64c1": dict(D=3, C=1, K=64, layers=(128, 128), latent="beta"),
    "k100": dict(D=4, C=0, K=100, layers=(128, 128), latent="normal"),
    "kmix": dict(D=4, C=0, K=(16, 8, 31, 12), layers=(128, 128), latent="normal"),
    # a 1-knot coupling inside a mixed chain keeps the flow on the
    # fp32 kernel (as a flow of 1-knot couplings is)
    "kmix1": dict(D=4, C=0, K=(16, 1, 8, 12), layers=(128, 128), latent="normal"),
    # the ends of the knot range: two knots (padded to 8), 63 (one padded knot
    # on the K = 64 instantiation), 200 (the layered path's cap)
    "k2": dict(D=2, C=0, K=2, layers=(64, 64), latent="normal"),
    "k63": dict(D=3, C=0, K=63, layers=(128, 128), latent="normal"),
    "k200": dict(D=2, C=1, K=200, layers=(64,), latent="beta"),
    # NeuralSplineCoupling(act=...) other than swish (bijectors.py:319): the
    # split-MFMA kernel's activation switch (sigmoid / softplus: the fp32
    # kernel) and the trainer
    "relu": dict(D=4, C=0, K=16, layers=(128, 128), latent="normal", act="relu"),
    "gelu": dict(D=3, C=1, K=8, layers=(64, 64), latent="beta", act="gelu"),
    "tanh": dict(D=2, C=0, K=16, layers=(128,), latent="normal", act="tanh"),
    "softplus": dict(D=4, C=0, K=8, layers=(32, 32), latent="normal", act="softplus"),
    "sigmoid": dict(D=2, C=2, K=16, layers=(64,), latent="beta", act="sigmoid"),
    "elu": dict(D=5, C=0, K=8, layers=(64, 64), latent="normal", act="elu"),
    "leaky_relu": dict(D=4, C=0, K=16, layers=(96,), latent="normal", act="leaky_relu"),
    # one activation per coupling (a Chain of differently configured couplings)
    "mixed": dict(D=4, C=0, K=16, layers=(128, 128), latent="normal", act=("relu", "swish", "gelu", "tanh")),
    "mixed_fp32": dict(D=3, C=0, K=8, layers=(64,), latent="normal", act=("swish", "sigmoid", "elu")),
    # hidden widths above 256 (layer_utils.rect / tri build any width): the
    # layered path (BatchNorm, the trainer's GEMMs, per-(row, dim) spline kernels)
    "h512": dict(D=4, C=0, K=16, layers=(512, 512), latent="normal"),
    "h384c2": dict(D=3, C=2, K=8, layers=(384,), latent="beta", act="gelu"),
    "h1024k5": dict(D=5, C=0, K=5, layers=(1024, 64), latent="truncated_normal", couplings=2),
    # a 260-wide input (K % 8 != 0) keeps Dense_1 on the trainer's GEMM, whose
    # output row maxima then come from the standalone row-max kernel for the
    # f16x2 last layer (zf_layered.hip)
    "h260": dict(D=3, C=0, K=8, layers=(260, 264), latent="normal"),
}
LAYERED = ["h512", "h384c2", "h1024k5", "h260"]
ACTS = ["relu", "gelu", "tanh", "softplus", "sigmoid", "elu", "leaky_relu", "mixed", "mixed_fp32"]


def chain_spec(cfg):
    D, layers = cfg["D"], list(cfg["layers"])
    L = cfg.get("couplings", D)
    acts = cfg.get("act", "swish")
    acts = [acts] if isinstance(acts, str) else list(acts)  # a list: one per coupling, cycled
    ks = cfg["K"] if isinstance(cfg["K"], (tuple, list)) else (cfg["K"],)  # likewise knots
    bij = [{"type": "shift_bounds", "margin": cfg.get("margin", 0.1), "bounds": cfg.get("bounds", ())}]
    for i in range(L - 1):
        bij.append({"type": "nsc", "knots": ks[i % len(ks)], "layers": layers, "act": acts[i % len(acts)]})
        bij.append({"type": "roll", "shift": 1})
    bij.append({"type": "nsc", "knots": ks[(L - 1) % len(ks)], "layers": layers, "act": acts[(L - 1) % len(acts)]})
    return {"type": "chain", "bijectors": bij}


def _lecun(rng, fan_in, fan_out):
    std = np.sqrt(1.0 / fan_in) / 0.87962566103423978
    z = np.clip(rng.standard_normal((fan_in, fan_out)), -2, 2)
    return (z * std).astype(np.float32)


def make_variables(cfg, rng, bias_scale=0.3):
    D, C = cfg["D"], cfg["C"]
    spec = chain_spec(cfg)
    dt = D // 2
    DC = D - dt + C
    params, stats = {}, {}
    for i, b in enumerate(spec["bijectors"]):
        key = f"bijectors_{i}"
        if b["type"] == "nsc":
            K = b["knots"]
            p = {
                "BatchNorm_0": {
                    "scale": (1 + 0.1 * rng.standard_normal(DC)).astype(np.float32),
                    "bias": (0.1 * rng.standard_normal(DC)).astype(np.float32),
                }
            }
            fan_in = DC
            for l, w in enumerate(list(b["layers"]) + [dt * (3 * K - 1)]):
                p[f"Dense_{l}"] = {
                    "kernel": _lecun(rng, fan_in, w),
                    "bias": (bias_scale * rng.standard_normal(w)).astype(np.float32),
                }
                fan_in = w
            params[key] = p
            stats[key] = {
                "BatchNorm_0": {
                    "mean": (0.2 * rng.standard_normal(DC)).astype(np.float32),
                    "var": (1 + 0.5 * rng.uniform(size=DC)).astype(np.float32),
                }
            }
    return spec, {"params": {"bijector": params}, "batch_stats": {"bijector": stats}}


def make_case(name, N=4096, seed=0, bias_scale=0.3):
    """Seeded case: x ~ N(0, I), c ~ N(0, I); ShiftBounds stats from a separate
    train-mode pass (margin 0.1) so some eval rows clip."""
    from oracle import zf_oracle as O

    cfg = dict(CONFIGS[name])
    rng = np.random.default_rng(seed)
    spec, variables = make_variables(cfg, rng, bias_scale)
    xs = rng.standard_normal((4096, cfg["D"])).astype(np.float32)
    _, _, sb = O.shift_bounds_forward(spec["bijectors"][0], {}, xs, train=True)
    variables["batch_stats"]["bijector"]["bijectors_0"] = {k: np.asarray(v, np.float32) for k, v in sb.items()}
    x = rng.standard_normal((N, cfg["D"])).astype(np.float32)
    c = rng.standard_normal((N, cfg["C"])).astype(np.float32) if cfg["C"] else None
    model = {"bijector": spec, "latent": {"type": cfg["latent"]}}
    return {"cfg": cfg, "model": model, "variables": variables, "x": x, "c": c, "name": name}


def build_flow(cfg):
    """The zenflow_amd module matching ``chain_spec(cfg)``."""
    import zenflow_amd as zf
    from zenflow_amd import bijectors as bi
    from zenflow_amd import distributions as dist

    latent = {
        "normal": dist.Normal,
        "beta": dist.Beta,
        "truncated_normal": dist.TruncatedNormal,
        "uniform": dist.Uniform,
    }[cfg["latent"]]()
    spec = chain_spec(cfg)
    mods = []
    for b in spec["bijectors"]:
        if b["type"] == "shift_bounds":
            mods.append(bi.ShiftBounds(margin=b["margin"], bounds=b["bounds"]))
        elif b["type"] == "nsc":
            mods.append(bi.NeuralSplineCoupling(knots=b["knots"], layers=tuple(b["layers"]), act=b.get("act", "swish")))
        else:
            mods.append(bi.Roll(b["shift"]))
    return zf.Flow(bi.Chain(mods), latent=latent)


# --- nested Flow (examples/deep_set.ipynb:318-328): a user module holding a Flow
def make_deep_set_module():
    """DeepSetFlow of the reference's deep-set example, restated on the
    zenflow_amd module protocol: a conditioning network ``phi`` (here one
    tanh Dense layer through ``Module.param``) and ``self.flow = Flow(...)``
    built in ``setup()``, called as ``self.flow(y, c, train=train)`` and
    ``self.flow.sample(c, seed=seed)``."""
    import zenflow_amd as zf

    class Phi(zf.Module):
        def __call__(self, x):
            w = self.param("kernel", lambda rng, shape: (0.5 * rng.standard_normal(shape)).astype(np.float32),
                           (x.shape[1], 2))
            b = self.param("bias", lambda rng, shape: np.zeros(shape, np.float32), (2,))
            return np.tanh(np.asarray(x, np.float32) @ w + b).astype(np.float32)

    class DeepSetFlow(zf.Module):
        def __init__(self, bijectors):
            self.bijectors = bijectors

        def setup(self):
            self.phi = Phi()
            self.flow = zf.Flow(self.bijectors)

        def __call__(self, x, y, train: bool = False):
            c = self.phi(x)
            return self.flow(y, c, train=train)

        def sample(self, x, seed):
            c = self.phi(x)
            return self.flow.sample(c, seed=seed)

    return DeepSetFlow
