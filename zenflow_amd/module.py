"""A minimal FLAX-style module protocol (``init`` / ``apply`` / variables).

zenflow's bijectors are FLAX ``nn.Module``s (bijectors.py:28); users drive them
with ``module.init(key, x, c)`` and ``module.apply(variables, x, c, train=...,
mutable=["batch_stats"], method=...)``.  This module reproduces exactly that
calling convention and the FLAX variable-tree layout (``params`` /
``batch_stats``, submodule names ``bijector``, ``bijectors_<i>``,
``BatchNorm_0``, ``Dense_<l>``) so reference-style code and variables work
unchanged.  The arithmetic itself always runs in the HIP kernels.
"""

from __future__ import annotations

import copy
import functools
import inspect
import itertools
import threading
from typing import Any, Callable, Dict, Optional, Tuple, Union

import numpy as np

_tls = threading.local()
_serial = itertools.count(1)


class Scope:
    """Variables bound for one ``apply`` (or ``init``) call of the OUTERMOST
    module, plus the collections it may mutate.  Child modules see a
    ``SubScope`` of it at their attribute path (``scope_for``)."""

    def __init__(self, variables: Dict[str, Any], mutable, owner=None, initializing: bool = False, rng=None):
        self.variables = variables or {}
        if mutable is True:
            mutable = ["params", "batch_stats"]
        elif isinstance(mutable, str):
            mutable = [mutable]
        self.mutable = list(mutable or [])
        self.updates: Dict[str, Any] = {}
        self.owner = owner
        self.initializing = initializing
        self.rng = rng  # numpy Generator while initializing
        self.path: Tuple[str, ...] = ()
        # modules whose methods are running (innermost last), the per-call
        # counters of inline submodules (flax compact naming: <Class>_<i> per
        # parent), and this call's id (auto-names are re-derived per call)
        self.stack: list = []
        self.counters: Dict[Tuple[int, str], int] = {}
        self.serial = next(_serial)

    def collection(self, name: str) -> Dict[str, Any]:
        return self.variables.get(name, {}) or {}

    def put(self, col: str, name: str, value) -> None:
        """Create a variable while initializing."""
        self.variables.setdefault(col, {})[name] = value

    def init_module(self, module, D: int, C: int) -> None:
        """Initializing: create ``module``'s own variables (its
        ``_init_variables`` for inputs of D dims and C conditions) here."""
        p: Dict[str, Any] = {}
        st: Dict[str, Any] = {}
        module._init_variables(self.rng, D, C, p, st)
        for k, v in p.items():
            self.put("params", k, v)
        for k, v in st.items():
            self.put("batch_stats", k, v)
        module._on_init(D, C)


class _Updates:
    """``scope.updates[col] = tree`` of a child: written into the root's
    updates at the child's path, on a copy of the whole collection (FLAX
    returns the full updated collection)."""

    def __init__(self, root: Scope, path):
        self.root, self.path = root, tuple(path)

    def __setitem__(self, col: str, value) -> None:
        if col not in self.root.updates:
            self.root.updates[col] = copy.deepcopy(self.root.variables.get(col, {}) or {})
        set_path(self.root.updates[col], self.path, value)

    def __contains__(self, col) -> bool:
        return col in self.root.updates


class SubScope:
    """A child module's view of the root scope: every collection at ``path``
    (e.g. ``variables["params"]["flow"]`` for ``self.flow`` of an outer
    module, as flax.linen names submodules by attribute)."""

    def __init__(self, root: Scope, path):
        self.root, self.path = root, tuple(path)
        self.mutable = root.mutable
        self.initializing = root.initializing
        self.rng = root.rng
        self.updates = _Updates(root, self.path)

    @property
    def variables(self) -> Dict[str, Any]:
        out = {}
        for col, tree in self.root.variables.items():
            v = get_path(tree or {}, self.path)
            if v is not None:
                out[col] = v
        return out

    def collection(self, name: str) -> Dict[str, Any]:
        return get_path(self.root.variables.get(name, {}) or {}, self.path) or {}

    def put(self, col: str, name: str, value) -> None:
        set_path(self.root.variables.setdefault(col, {}), self.path + (name,), value)

    init_module = Scope.init_module


def current_scope() -> Scope:
    s = getattr(_tls, "scope", None)
    if s is None:
        raise RuntimeError(
            "Can't call a zenflow_amd module outside of init/apply; use "
            "module.apply(variables, ...) (same rule as flax.linen)."
        )
    return s


def _chain(module, owner):
    """Attribute path from ``owner`` down to ``module``, or None when the
    chain of ``_zf_parent`` / ``_zf_name`` links does not reach it."""
    path = []
    m = module
    while m is not None and m is not owner:
        name = m.__dict__.get("_zf_name")
        if name is None:
            return None
        path.append(name)
        m = m.__dict__.get("_zf_parent")
    return None if m is None else list(reversed(path))


def scope_for(module) -> Union[Scope, SubScope]:
    """The scope ``module`` sees: the root scope when it is the module that
    ``apply``/``init`` was called on, else the sub-scope at its attribute
    path below that module — so a Flow held as ``self.flow`` by an outer
    module reads ``variables[col]["flow"]`` (examples/deep_set.ipynb:
    ``self.flow(y, c, train=train)``).  A submodule created inline in a
    method (``Phi()(x)``) or held where no attribute names it (a dict, a
    ``_private`` attribute) is named ``<Class>_<i>`` after the module that
    calls it, as flax.linen's compact methods name them; a module with no
    link to the one ``apply``/``init`` runs on raises."""
    s = current_scope()
    if s.owner is None or module is s.owner:
        return s
    path = _chain(module, s.owner)
    if path is None or (module.__dict__.get("_zf_auto") not in (None, s.serial)):
        _adopt(s, module)
        path = _chain(module, s.owner)
    if path is None:
        raise RuntimeError(
            f"{type(module).__name__} is used inside {type(s.owner).__name__}.apply/init but is not one of its "
            "submodules (assign it as an attribute, or create it inside the calling module's method)")
    return SubScope(s, path)


def _adopt(s: Scope, module) -> None:
    """Name an unlinked ``module`` after the module whose method is running
    (the caller): ``<Class>_<i>``, i counting that caller's inline children
    of the class in this call (flax compact naming)."""
    parent = next((m for m in reversed(s.stack) if m is not module), s.owner)
    if parent is None:
        return
    cls = type(module).__name__
    key = (id(parent), cls)
    i = s.counters.get(key, 0)
    s.counters[key] = i + 1
    d = module.__dict__
    d["_zf_parent"] = parent
    d["_zf_name"] = f"{cls}_{i}"
    d["_zf_auto"] = s.serial


def _wrap_method(fn):
    """A module method run under a scope: pushes the module on the scope's
    call stack (so inline submodules it calls are named after it), names the
    module itself if nothing links it to the scope's owner, and while
    initializing creates the variables its setup() declared."""

    @functools.wraps(fn)
    def wrapped(self, *args, **kwargs):
        s = getattr(_tls, "scope", None)
        if s is None or (s.stack and s.stack[-1] is self):
            return fn(self, *args, **kwargs)
        if s.owner is not None and self is not s.owner:
            if _chain(self, s.owner) is None or self.__dict__.get("_zf_auto") not in (None, s.serial):
                _adopt(s, self)
        s.stack.append(self)
        try:
            self._ensure_setup()  # once per init/apply call
            if s.initializing:
                for name in list(self.__dict__.get("_zf_refs", {})):
                    getattr(self, name)  # flax creates setup()'s variables at init
            return fn(self, *args, **kwargs)
        finally:
            s.stack.pop()

    wrapped._zf_wrapped = True
    return wrapped


_NOT_WRAPPED = {"init", "apply", "param", "variable", "setup", "bind"}


class _SetupRef:
    """What ``self.param`` / ``self.variable`` return inside ``setup()``: a
    declaration, bound to the variables of whichever init/apply call reads
    the attribute (setup() itself re-runs per init/apply call, as flax
    re-runs it per bind: ``Module._ensure_setup``)."""

    def __init__(self, kind, args):
        self.kind, self.args = kind, args

    def resolve(self, module):
        d = module.__dict__
        in_setup = d.get("_zf_in_setup")
        if in_setup:
            # setup() reading a variable it has just declared (flax allows
            # `self.w = self.param(...); n = self.w.shape[0]`): resolve it
            # against the init/apply call that triggered setup()
            if getattr(_tls, "scope", None) is None:
                raise RuntimeError(
                    f"{type(module).__name__}.setup() reads {self.kind} {self.args[0]!r} outside init/apply: "
                    "variables declared in setup() have values only inside module.init / module.apply"
                )
            d["_zf_in_setup"] = False
        try:
            if self.kind == "param":
                return Module.param(module, *self.args)
            return Module.variable(module, *self.args)
        finally:
            if in_setup:
                d["_zf_in_setup"] = True

    def __repr__(self):
        return f"<{self.kind} {self.args[0]!r} declared in setup()>"


def _same_value(a, b) -> bool:
    if a is b:
        return True
    if isinstance(a, Module) or isinstance(b, Module):
        return _same_module_config(a, b)
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return type(a) is type(b) and len(a) == len(b) and all(_same_value(x, y) for x, y in zip(a, b))
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return (isinstance(a, np.ndarray) and isinstance(b, np.ndarray) and a.dtype == b.dtype
                and a.shape == b.shape and bool(np.array_equal(a, b)))
    if (type(a) is type(b) and not callable(a) and hasattr(a, "__dict__")
            and type(a).__eq__ is object.__eq__):  # plain config objects (a latent distribution)
        va = {k: v for k, v in vars(a).items() if not k.startswith("_")}  # lazily set state (Distribution._dim)
        vb = {k: v for k, v in vars(b).items() if not k.startswith("_")}
        return va.keys() == vb.keys() and all(_same_value(va[k], vb[k]) for k in va)
    try:
        return bool(a == b)
    except Exception:
        return False


def _same_module_config(a, b) -> bool:
    """Two modules (or lists of modules) of one class with equal public
    attributes: the instance a setup() re-run may keep."""
    if isinstance(a, (list, tuple)) or isinstance(b, (list, tuple)):
        return (isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)) and len(a) == len(b)
                and all(isinstance(x, Module) for x in a) and all(_same_module_config(x, y) for x, y in zip(a, b)))
    if not (isinstance(a, Module) and isinstance(b, Module)) or type(a) is not type(b):
        return False
    # constructor configuration only: what a's own setup() derived is not
    sa, sb = a.__dict__.get("_zf_setup_attrs", ()), b.__dict__.get("_zf_setup_attrs", ())
    pa = {k: v for k, v in a.__dict__.items() if not k.startswith("_") and k not in sa}
    pb = {k: v for k, v in b.__dict__.items() if not k.startswith("_") and k not in sb}
    return pa.keys() == pb.keys() and all(_same_value(pa[k], pb[k]) for k in pa)


def _resolve_method(module, method):
    if method is None:
        return type(module).__call__
    if isinstance(method, str):
        return getattr(type(module), method)
    return method


def _name_children(parent, name: str, value) -> None:
    if isinstance(value, Module):
        value.__dict__["_zf_parent"] = parent
        value.__dict__["_zf_name"] = name
    elif isinstance(value, (list, tuple)):
        for i, v in enumerate(value):
            if isinstance(v, Module):  # flax: <attr>_<i>
                v.__dict__["_zf_parent"] = parent
                v.__dict__["_zf_name"] = f"{name}_{i}"


class Module:
    """Base class: FLAX-like ``init`` and ``apply``.

    Submodules assigned as attributes (in ``__init__`` or in a ``setup()``
    method, which runs lazily as in flax.linen) are named by their attribute
    (``self.flow`` -> ``"flow"``, a list ``self.layers`` -> ``"layers_<i>"``)
    and read their variables from that sub-tree when called inside the outer
    module's ``apply``/``init``.  ``param``/``variable`` give user modules
    their own variables."""

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        for name, fn in list(cls.__dict__.items()):
            if (name.startswith("_") and name != "__call__") or name in _NOT_WRAPPED:
                continue
            if inspect.isfunction(fn) and not getattr(fn, "_zf_wrapped", False):
                setattr(cls, name, _wrap_method(fn))

    def __setattr__(self, name, value):
        d = self.__dict__
        if d.get("_zf_in_setup") and not name.startswith("_"):
            d.setdefault("_zf_setup_attrs", set()).add(name)
        if isinstance(value, _SetupRef):  # self.w = self.param(...) in setup()
            d.setdefault("_zf_refs", {})[name] = value
            d.pop(name, None)
            return
        object.__setattr__(self, name, value)
        if not name.startswith("_"):
            _name_children(self, name, value)

    def __getattr__(self, name):
        d = self.__dict__
        refs = d.get("_zf_refs")
        if refs is not None and name in refs:  # a setup() declaration: this call's value
            return refs[name].resolve(self)
        # flax runs setup() lazily on first attribute access
        if not name.startswith("__") and not d.get("_zf_setup_done") and callable(getattr(type(self), "setup", None)):
            self._ensure_setup()
            return getattr(self, name)
        raise AttributeError(f"{type(self).__name__!s} has no attribute {name!r}")

    def _ensure_setup(self) -> None:
        """Run setup() once per init/apply call (flax re-runs it on every
        bind), so attributes it derives from param values (``self.w2 =
        self.w * 2``) follow the variables of the current call.
        Outside any call it runs once, lazily.  A submodule that a re-run
        creates again with the same configuration keeps the previous instance,
        so per-instance device-program caches survive repeated apply calls."""
        d = self.__dict__
        if not callable(getattr(type(self), "setup", None)):
            return
        s = getattr(_tls, "scope", None)
        key = None if s is None else s.serial
        if d.get("_zf_setup_done") and (key is None or d.get("_zf_setup_serial") == key):
            return
        old = {}
        if d.get("_zf_setup_done"):
            for name in d.pop("_zf_setup_attrs", ()):
                if name in d:
                    old[name] = d.pop(name)
            d.pop("_zf_refs", None)
        d["_zf_setup_done"] = True
        d["_zf_setup_serial"] = key
        d["_zf_in_setup"] = True
        try:
            self.setup()
        finally:
            d["_zf_in_setup"] = False
        for name, prev in old.items():
            if name in d and _same_module_config(prev, d[name]):
                object.__setattr__(self, name, prev)
                _name_children(self, name, prev)

    def init(self, rng, *args, method=None, **kwargs) -> Dict[str, Any]:
        """Create the variables (``params`` + ``batch_stats``) for the input shapes.

        Mirrors ``flax.linen.Module.init``: parameters are drawn with FLAX's
        default initialisers (lecun_normal kernels, zero biases, BatchNorm
        scale 1 / bias 0 / mean 0 / var 1); ShiftBounds stats start at +-inf.
        ``rng`` may be ``zenflow_amd.random.PRNGKey(seed)``, an int or a
        ``numpy.random.Generator``.  A module that does not define its own
        variables (a user module holding a Flow, say) runs ``method`` once in
        initializing mode: each submodule creates its variables from the
        inputs it is called with (outputs are placeholders, not computed)."""
        from .random import as_generator

        gen = as_generator(rng)
        if type(self)._init_variables is Module._init_variables:
            scope = Scope({}, True, owner=self, initializing=True, rng=gen)
            prev = getattr(_tls, "scope", None)
            _tls.scope = scope
            try:
                self._ensure_setup()  # inside the scope: setup() may read what it declares
                _resolve_method(self, method)(self, *args, **kwargs)
            finally:
                _tls.scope = prev
            return {k: v for k, v in scope.variables.items() if v}
        x = args[0] if args else kwargs.get("x")
        c = args[1] if len(args) > 1 else kwargs.get("c")
        shape = np.shape(x)
        D = int(shape[1]) if len(shape) > 1 else 1
        cshape = None if c is None else np.shape(c)
        C = 0 if cshape is None else (1 if len(cshape) == 1 else int(cshape[1]))
        params: Dict[str, Any] = {}
        stats: Dict[str, Any] = {}
        self._init_variables(gen, D, C, params, stats)
        self._on_init(D, C)
        out: Dict[str, Any] = {}
        if params:
            out["params"] = params
        if stats:
            out["batch_stats"] = stats
        return out

    def apply(self, variables, *args, method=None, mutable=False, **kwargs):
        """Run ``method`` (default ``__call__``) with ``variables`` bound.

        With ``mutable`` (e.g. ``["batch_stats"]``) returns ``(out, updates)``
        as FLAX does."""
        fn = _resolve_method(self, method)
        scope = Scope(variables, mutable, owner=self)
        prev = getattr(_tls, "scope", None)
        _tls.scope = scope
        try:
            self._ensure_setup()  # inside the scope: setup() may read what it declares
            out = fn(self, *args, **kwargs)
        finally:
            _tls.scope = prev
        if scope.mutable:
            upd = {}
            for col in scope.mutable:
                if col in scope.updates:
                    upd[col] = scope.updates[col]
                elif col in (variables or {}):
                    upd[col] = copy.deepcopy(variables[col])
            return out, upd
        return out

    # variables of user modules (flax.linen.Module.param / .variable) ---------
    def param(self, name: str, init_fn: Callable, *init_args):
        """``params`` variable ``name`` of this module: created by
        ``init_fn(rng, *init_args)`` while initializing, read otherwise.
        Inside ``setup()`` it declares the variable: the attribute it is
        assigned to reads the value of the current init/apply call."""
        if self.__dict__.get("_zf_in_setup"):
            return _SetupRef("param", (name, init_fn, *init_args))
        s = scope_for(self)
        cur = s.collection("params")
        if name not in cur:
            if not s.initializing:
                raise KeyError(f"params/{'/'.join(s.path + (name,))} is missing from the variables")
            s.put("params", name, init_fn(s.rng, *init_args))
            cur = s.collection("params")
        return cur[name]

    def variable(self, col: str, name: str, init_fn: Callable, *init_args) -> "Variable":
        """A mutable variable of collection ``col`` (e.g. ``batch_stats``)."""
        if self.__dict__.get("_zf_in_setup"):
            return _SetupRef("variable", (col, name, init_fn, *init_args))
        s = scope_for(self)
        if name not in s.collection(col):
            if not s.initializing:
                raise KeyError(f"{col}/{'/'.join(s.path + (name,))} is missing from the variables")
            s.put(col, name, init_fn(*init_args))
        return Variable(s, col, name)

    # subclasses --------------------------------------------------------------
    def _init_variables(self, gen, D, C, params, stats) -> None:
        pass

    def _on_init(self, D, C) -> None:
        pass


class Variable:
    """flax.core.scope.Variable: ``.value`` reads the bound variable; setting
    it requires the collection to be mutable and lands in the updates."""

    def __init__(self, scope, col: str, name: str):
        self._scope, self._col, self._name = scope, col, name

    @property
    def value(self):
        s = self._scope
        root = s.root if isinstance(s, SubScope) else s
        path = s.path if isinstance(s, SubScope) else ()
        if self._col in root.updates:  # updated earlier in this call
            tree = get_path(root.updates[self._col], path)
            if tree is not None and self._name in tree:
                return tree[self._name]
        return s.collection(self._col)[self._name]

    @value.setter
    def value(self, v):
        s = self._scope
        if s.initializing:
            s.put(self._col, self._name, v)
            return
        if self._col not in s.mutable:
            raise RuntimeError(f"collection {self._col!r} is not mutable (pass mutable=[{self._col!r}])")
        root = s.root if isinstance(s, SubScope) else s
        path = s.path if isinstance(s, SubScope) else ()
        # the latest value of the collection (an earlier update of this call included)
        base = get_path(root.updates[self._col], path) if self._col in root.updates else None
        tree = copy.deepcopy(base if base is not None else s.collection(self._col))
        tree[self._name] = v
        s.updates[self._col] = tree


def lecun_normal(gen: np.random.Generator, fan_in: int, fan_out: int) -> np.ndarray:
    """flax default kernel init: variance_scaling(1, 'fan_in', 'truncated_normal')."""
    std = np.sqrt(1.0 / max(1, fan_in)) / 0.87962566103423978
    z = gen.standard_normal((fan_in, fan_out))
    bad = np.abs(z) > 2.0
    while bad.any():
        z[bad] = gen.standard_normal(int(bad.sum()))
        bad = np.abs(z) > 2.0
    return (z * std).astype(np.float32)


def get_path(tree: Dict[str, Any], path) -> Any:
    node = tree
    for k in path:
        if not isinstance(node, dict) or k not in node:
            return None
        node = node[k]
    return node


def set_path(tree: Dict[str, Any], path, value) -> None:
    node = tree
    for k in path[:-1]:
        node = node.setdefault(k, {})
    node[path[-1]] = value
