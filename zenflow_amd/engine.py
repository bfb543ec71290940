"""Compile a zenflow module tree + FLAX variables into one device flow program.

A ``Program`` flattens (Flow ->) Chain -> {ShiftBounds, Roll,
NeuralSplineCoupling} into the C ABI's op list, writes the variables into the
natural parameter blob (``zf_flow_plan`` offsets) and hands it to
``zf_flow_create``, which packs it into MFMA fragment order on the device.
Eval-mode forward / inverse / log_prob are ONE fused kernel launch over the
whole chain.  Train mode (batch statistics, bijectors.py:250-260 and flax
BatchNorm) runs op by op: a device column-statistics reduction, a few bytes of
host bookkeeping (the running-average update), then the op itself.
"""

from __future__ import annotations

import ctypes as ct
import copy
import math
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import _lib as L
from ._lib import DeviceArray, check
from .module import get_path, set_path

try:  # fast content digest when available; stdlib otherwise
    import xxhash as _xxhash
except ImportError:  # pragma: no cover - depends on the environment
    _xxhash = None
import hashlib
from collections import OrderedDict

BN_MOMENTUM = 0.99  # flax.linen.BatchNorm default
BN_EPS = 1e-5


@dataclass
class OpRec:
    kind: int
    path: Tuple[str, ...]
    module: Any


def flatten(module, path: Tuple[str, ...] = ()) -> List[OpRec]:
    """Chain.__call__ order (bijectors.py:108-110); nested chains are inlined."""
    from .bijectors import Chain, NeuralSplineCoupling, Roll, ShiftBounds

    if isinstance(module, Chain):
        out: List[OpRec] = []
        for i, b in enumerate(module.bijectors):
            out.extend(flatten(b, path + (f"bijectors_{i}",)))
        return out
    if isinstance(module, ShiftBounds):
        return [OpRec(L.ZF_OP_SHIFT_BOUNDS, path, module)]
    if isinstance(module, Roll):
        return [OpRec(L.ZF_OP_ROLL, path, module)]
    if isinstance(module, NeuralSplineCoupling):
        return [OpRec(L.ZF_OP_NSC, path, module)]
    raise NotImplementedError(
        f"{type(module).__name__} has no HIP implementation in zenflow_amd "
        "(supported: Chain, ShiftBounds, Roll, NeuralSplineCoupling)"
    )


def _is_set(v) -> bool:
    """bijectors.py:426-427."""
    return v is not None and bool(np.isfinite(v))


def sb_modes(module, D) -> List[Tuple[int, float, float]]:
    """Per-dim (mode, a, b) of a ShiftBounds (bijectors.py:176-205)."""
    bounds = {int(i): (a, b) for (i, a, b) in module.bounds}
    out = []
    for i in range(D):
        a, b = bounds.get(i, (None, None))
        if _is_set(a) and _is_set(b):
            out.append((L.ZF_SB_BOTH, float(a), float(b)))
        elif _is_set(a):
            out.append((L.ZF_SB_LOWER, float(a), 0.0))
        elif _is_set(b):
            out.append((L.ZF_SB_UPPER, 0.0, float(b)))
        else:
            out.append((L.ZF_SB_NONE, 0.0, 0.0))
    return out


def _arr(v, shape, name) -> np.ndarray:
    a = np.asarray(v, dtype=np.float32)
    if a.shape != tuple(shape):
        raise ValueError(f"variable {name} has shape {a.shape}, expected {tuple(shape)}")
    return a


class Program:
    """Device flow program for a module tree bound to concrete variables."""

    def __init__(self, root, variables: Dict[str, Any], D: int, C: int, latent=None):
        L.ensure_device()
        self.root = root
        self.D = int(D)
        self.C = int(C)
        self.ops = flatten(root)
        self.latent = latent
        params = variables.get("params", {}) if variables else {}
        stats = variables.get("batch_stats", {}) if variables else {}
        desc = L.ZfFlowDesc()
        desc.dim = self.D
        desc.cond_dim = self.C
        desc.latent, desc.latent_param = _latent_code(latent)
        if len(self.ops) > 64:
            raise NotImplementedError("more than 64 bijectors in one chain")
        desc.n_ops = len(self.ops)
        for i, op in enumerate(self.ops):
            d = desc.ops[i]
            d.kind = op.kind
            if op.kind == L.ZF_OP_ROLL:
                d.shift = int(op.module.shift)
            elif op.kind == L.ZF_OP_NSC:
                m = op.module
                if len(m.layers) < 1:
                    raise NotImplementedError("NeuralSplineCoupling with no hidden layer")
                if len(m.layers) > 16:
                    raise NotImplementedError("more than 16 hidden layers")
                d.knots = int(m.knots)
                d.n_hidden = len(m.layers)
                for l, w in enumerate(m.layers):
                    d.hidden[l] = int(w)
                d.act = int(m.act_code)
        n = ct.c_int64()
        lib = L.load_library()
        check(lib.zf_flow_plan(ct.byref(desc), ct.byref(n)), "zf_flow_plan")
        blob = np.zeros(max(1, n.value), np.float32)
        self.param_mask = np.zeros(blob.shape, np.uint8)
        self._fill_blob(desc, blob, params, stats)
        self.blob = blob  # natural layout (host copy): what the trainer starts from
        h = ct.c_void_p()
        check(lib.zf_flow_create(ct.byref(desc), blob.ctypes.data, n.value, ct.byref(h)), "zf_flow_create")
        self.desc = desc
        self.handle = h.value
        self._ws: Optional[DeviceArray] = None

    @property
    def kernel_variant(self) -> str:
        """'f16x2', 'bf16x3' or 'fp32': the fused kernel this chain runs, or 'layered' (a hidden
        width above 256: op by op on GEMMs and spline kernels; zf_flow_kernel_variant)."""
        v = L.load_library().zf_flow_kernel_variant(ct.c_void_p(self.handle))
        return {L.ZF_KERNEL_F16X2: "f16x2", L.ZF_KERNEL_BF16X3: "bf16x3", L.ZF_KERNEL_LAYERED: "layered"}.get(v, "fp32")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and L._lib is not None:
            L._lib.zf_flow_destroy(ct.c_void_p(h))
            self.handle = None

    # -- blob ----------------------------------------------------------------
    def _fill_blob(self, desc, blob, params, stats):
        D, Cd = self.D, self.C
        for i, op in enumerate(self.ops):
            d = desc.ops[i]
            if op.kind == L.ZF_OP_SHIFT_BOUNDS:
                st = get_path(stats, op.path) or {}
                for j, (mode, a, b) in enumerate(sb_modes(op.module, D)):
                    xmin = np.asarray(st.get(f"xmin_{j}", [np.inf]), np.float32).reshape(-1)[0]
                    xmax = np.asarray(st.get(f"xmax_{j}", [-np.inf]), np.float32).reshape(-1)[0]
                    blob[d.off_sb + 8 * j : d.off_sb + 8 * j + 6] = [mode, a, b, xmin, xmax, op.module.margin]
            elif op.kind == L.ZF_OP_NSC:
                p = get_path(params, op.path)
                s = get_path(stats, op.path)
                if p is None:
                    raise ValueError(f"missing params for NeuralSplineCoupling at {'/'.join(op.path) or '<root>'}")
                dt = D // 2
                DC = D - dt + Cd
                bnp = p.get("BatchNorm_0", {})
                bns = (s or {}).get("BatchNorm_0", {})
                o = d.off_bn
                blob[o : o + DC] = _arr(bns.get("mean", np.zeros(DC)), (DC,), "BatchNorm_0/mean")
                blob[o + DC : o + 2 * DC] = _arr(bns.get("var", np.ones(DC)), (DC,), "BatchNorm_0/var")
                blob[o + 2 * DC : o + 3 * DC] = _arr(bnp.get("scale", np.ones(DC)), (DC,), "BatchNorm_0/scale")
                blob[o + 3 * DC : o + 4 * DC] = _arr(bnp.get("bias", np.zeros(DC)), (DC,), "BatchNorm_0/bias")
                self.param_mask[o + 2 * DC : o + 4 * DC] = 1
                widths = list(op.module.layers) + [dt * (3 * op.module.knots - 1)]
                fan_in = DC
                for l, w in enumerate(widths):
                    dense = p.get(f"Dense_{l}")
                    if dense is None:
                        raise ValueError(f"missing Dense_{l} params")
                    k = _arr(dense["kernel"], (fan_in, w), f"Dense_{l}/kernel")
                    b = _arr(dense["bias"], (w,), f"Dense_{l}/bias")
                    blob[d.off_w[l] : d.off_w[l] + k.size] = k.ravel()
                    blob[d.off_b[l] : d.off_b[l] + w] = b
                    self.param_mask[d.off_w[l] : d.off_w[l] + k.size] = 1
                    self.param_mask[d.off_b[l] : d.off_b[l] + w] = 1
                    fan_in = w

    def blob_to_variables(self, blob: np.ndarray) -> Dict[str, Any]:
        """Inverse of _fill_blob: {"params": ..., "batch_stats": ...} of the
        bijector (FLAX layout) from a natural blob."""
        D, Cd = self.D, self.C
        params: Dict[str, Any] = {}
        stats: Dict[str, Any] = {}
        f32 = np.float32
        for i, op in enumerate(self.ops):
            d = self.desc.ops[i]
            if op.kind == L.ZF_OP_SHIFT_BOUNDS:
                for j, (mode, _, _) in enumerate(sb_modes(op.module, D)):
                    if mode == L.ZF_SB_BOTH:
                        continue
                    r = d.off_sb + 8 * j
                    set_path(stats, op.path + (f"xmin_{j}",), np.array([blob[r + 3]], f32))
                    set_path(stats, op.path + (f"xmax_{j}",), np.array([blob[r + 4]], f32))
            elif op.kind == L.ZF_OP_NSC:
                dt = D // 2
                DC = D - dt + Cd
                o = d.off_bn
                set_path(stats, op.path + ("BatchNorm_0", "mean"), blob[o : o + DC].astype(f32).copy())
                set_path(stats, op.path + ("BatchNorm_0", "var"), blob[o + DC : o + 2 * DC].astype(f32).copy())
                set_path(params, op.path + ("BatchNorm_0", "scale"), blob[o + 2 * DC : o + 3 * DC].astype(f32).copy())
                set_path(params, op.path + ("BatchNorm_0", "bias"), blob[o + 3 * DC : o + 4 * DC].astype(f32).copy())
                widths = list(op.module.layers) + [dt * (3 * op.module.knots - 1)]
                fan_in = DC
                for l, w in enumerate(widths):
                    k = blob[d.off_w[l] : d.off_w[l] + fan_in * w].reshape(fan_in, w).astype(f32).copy()
                    set_path(params, op.path + (f"Dense_{l}", "kernel"), k)
                    set_path(params, op.path + (f"Dense_{l}", "bias"), blob[d.off_b[l] : d.off_b[l] + w].astype(f32).copy())
                    fan_in = w
        return {"params": params, "batch_stats": stats}

    # -- helpers ---------------------------------------------------------------
    def workspace(self, N: int) -> DeviceArray:
        need = int(L.load_library().zf_flow_workspace_bytes(N))
        if self._ws is None or self._ws.nbytes < need:
            self._ws = DeviceArray((need,), np.uint8)
        return self._ws

    def _c_ptr(self, c: Optional[DeviceArray]):
        if self.C == 0:
            return None
        if c is None:
            raise ValueError(f"this flow is conditional (C={self.C}); pass c")
        return c.ptr

    def _check_x(self, x: DeviceArray):
        if x.ndim != 2 or x.shape[1] != self.D:
            raise ValueError(f"x must have shape (N, {self.D}), got {x.shape}")

    # -- launches --------------------------------------------------------------
    def forward(self, x: DeviceArray, c=None, op_begin=0, op_end=None, ld_in=None,
                y: Optional[DeviceArray] = None, ld: Optional[DeviceArray] = None):
        """Chain.__call__ in eval mode (bijectors.py:103-111)."""
        self._check_x(x)
        N = x.shape[0]
        op_end = len(self.ops) if op_end is None else op_end
        y = y if y is not None else DeviceArray((N, self.D))
        ld = ld if ld is not None else DeviceArray((N,))
        check(L.load_library().zf_flow_forward(
            self.handle, op_begin, op_end, x.ptr, self._c_ptr(c), y.ptr,
            None if ld_in is None else ld_in.ptr, ld.ptr, N, L.stream()), "zf_flow_forward")
        return y, ld

    def inverse(self, z: DeviceArray, c=None, op_begin=0, op_end=None, out=None):
        """Chain.inverse (bijectors.py:113-116)."""
        self._check_x(z)
        N = z.shape[0]
        op_end = len(self.ops) if op_end is None else op_end
        x = out if out is not None else DeviceArray((N, self.D))
        check(L.load_library().zf_flow_inverse(
            self.handle, op_begin, op_end, z.ptr, self._c_ptr(c), x.ptr, N, L.stream()),
            "zf_flow_inverse")
        return x

    def sample(self, N: int, seed: int, c=None, out=None):
        """Flow.sample (flow.py:50-78) in one launch: latent drawn on the device
        (Philox, zf_flow_sample), then Chain.inverse."""
        if self.latent is None:
            raise ValueError("flow has no latent distribution")
        x = out if out is not None else DeviceArray((N, self.D))
        check(L.load_library().zf_flow_sample(
            self.handle, int(seed) & 0xFFFFFFFFFFFFFFFF, self._c_ptr(c), x.ptr, N, L.stream()),
            "zf_flow_sample")
        return x

    def log_prob(self, x: DeviceArray, c=None, out=None, nll_sum: Optional[DeviceArray] = None,
                 op_begin=0, op_end=None, ld_in=None):
        """Flow.__call__ (flow.py:22-48) as one fused launch (+ the NLL reduce)."""
        self._check_x(x)
        N = x.shape[0]
        op_end = len(self.ops) if op_end is None else op_end
        lp = out if out is not None else DeviceArray((N,))
        ws = self.workspace(N) if nll_sum is not None else None
        check(L.load_library().zf_flow_log_prob_segment(
            self.handle, op_begin, op_end, x.ptr, self._c_ptr(c),
            None if ld_in is None else ld_in.ptr, lp.ptr,
            None if nll_sum is None else nll_sum.ptr, None if ws is None else ws.ptr,
            N, L.stream()), "zf_flow_log_prob")
        return lp

    # -- train mode --------------------------------------------------------------
    def colstats(self, x: DeviceArray, ncols, ld, col_offset, modes=None, params=None):
        N = x.shape[0]
        lib = L.load_library()
        ws = DeviceArray((int(lib.zf_colstats_workspace_bytes(N, ncols)),), np.uint8)
        cmin = DeviceArray((ncols,))
        cmax = DeviceArray((ncols,))
        csum = DeviceArray((ncols,), np.float64)
        csq = DeviceArray((ncols,), np.float64)
        m = None if modes is None else np.ascontiguousarray(modes, np.float32)
        p = None if params is None else np.ascontiguousarray(params, np.float32)
        check(lib.zf_colstats(
            x.ptr, N, ncols, ld, col_offset,
            None if m is None else m.ctypes.data, None if p is None else p.ctypes.data,
            cmin.ptr, cmax.ptr, csum.ptr, csq.ptr, ws.ptr, L.stream()), "zf_colstats")
        return cmin.numpy(), cmax.numpy(), csum.numpy(), csq.numpy()

    def train_forward(self, x: DeviceArray, c, batch_stats: Dict[str, Any], update: bool):
        """Chain.__call__ with train=True: batch statistics, op by op.

        Returns (y, log_det, new_batch_stats)."""
        self._check_x(x)
        N = x.shape[0]
        lib = L.load_library()
        new_stats = copy.deepcopy(batch_stats) if batch_stats else {}
        state = x
        ld = DeviceArray((N,)).zero_()
        f32 = np.float32
        for i, op in enumerate(self.ops):
            if op.kind == L.ZF_OP_SHIFT_BOUNDS:
                modes = sb_modes(op.module, self.D)
                mcol = [m for (m, _, _) in modes]
                pcol = [a if m == L.ZF_SB_LOWER else b for (m, a, b) in modes]
                cmin, cmax, _, _ = self.colstats(state, self.D, self.D, 0, mcol, pcol)
                old = get_path(batch_stats, op.path) or {}
                xmins = np.zeros(self.D, f32)
                xmaxs = np.zeros(self.D, f32)
                margin = f32(op.module.margin)
                for j, (mode, a, b) in enumerate(modes):
                    if mode == L.ZF_SB_BOTH:
                        continue
                    # bijectors.py:250-257
                    lo, hi = f32(cmin[j]), f32(cmax[j])
                    delta = f32(0.5) * (hi - lo) * margin
                    lo, hi = lo - delta, hi + delta
                    ra_min = f32(np.asarray(old.get(f"xmin_{j}", [np.inf]), f32).reshape(-1)[0])
                    ra_max = f32(np.asarray(old.get(f"xmax_{j}", [-np.inf]), f32).reshape(-1)[0])
                    lo = np.minimum(ra_min, lo)
                    hi = np.maximum(ra_max, hi)
                    xmins[j], xmaxs[j] = lo, hi
                    if update:
                        set_path(new_stats, op.path + (f"xmin_{j}",), np.array([lo], f32))
                        set_path(new_stats, op.path + (f"xmax_{j}",), np.array([hi], f32))
                check(lib.zf_flow_set_sb_stats(self.handle, i, xmins.ctypes.data, xmaxs.ctypes.data),
                      "zf_flow_set_sb_stats")
            elif op.kind == L.ZF_OP_NSC:
                dt = self.D // 2
                dc = self.D - dt
                _, _, s1, q1 = self.colstats(state, dc, self.D, dt)
                sums, sqs = [s1], [q1]
                if self.C:
                    _, _, s2, q2 = self.colstats(c, self.C, self.C, 0)
                    sums.append(s2)
                    sqs.append(q2)
                csum = np.concatenate(sums)
                csq = np.concatenate(sqs)
                mean = (csum / N).astype(f32)
                mean2 = (csq / N).astype(f32)
                var = np.maximum(f32(0), mean2 - mean * mean)
                check(lib.zf_flow_set_bn_stats(self.handle, i, mean.ctypes.data, var.ctypes.data),
                      "zf_flow_set_bn_stats")
                if update:
                    old = get_path(batch_stats, op.path + ("BatchNorm_0",)) or {}
                    DC = dc + self.C
                    om = np.asarray(old.get("mean", np.zeros(DC)), f32)
                    ov = np.asarray(old.get("var", np.ones(DC)), f32)
                    mom = f32(BN_MOMENTUM)
                    set_path(new_stats, op.path + ("BatchNorm_0", "mean"), mom * om + f32(1 - BN_MOMENTUM) * mean)
                    set_path(new_stats, op.path + ("BatchNorm_0", "var"), mom * ov + f32(1 - BN_MOMENTUM) * var)
            state, ld = self.forward(state, c, i, i + 1, ld_in=ld)
        return state, ld, new_stats


def _latent_code(latent) -> Tuple[int, float]:
    if latent is None:
        return L.ZF_LATENT_NONE, 0.0
    from .distributions import Beta, Normal, TruncatedNormal, Uniform

    if isinstance(latent, Normal):
        return L.ZF_LATENT_NORMAL, 0.0
    if isinstance(latent, Beta):
        return L.ZF_LATENT_BETA, float(latent.peakness)
    if isinstance(latent, TruncatedNormal):
        return L.ZF_LATENT_TRUNCNORM, 0.0
    if isinstance(latent, Uniform):
        return L.ZF_LATENT_UNIFORM, 0.0
    raise NotImplementedError(f"latent {type(latent).__name__} has no HIP implementation")


def to_host_like(arr: DeviceArray, like_device: bool):
    return arr if like_device else arr.numpy()


def _digest(tree) -> str:
    """Content digest of a variables tree: paths, shapes, dtypes and bytes."""
    h = _xxhash.xxh3_128() if _xxhash is not None else hashlib.blake2b(digest_size=16)

    def walk(node, path):
        if isinstance(node, dict):
            for k in sorted(node):
                walk(node[k], path + "/" + str(k))
            return
        a = np.ascontiguousarray(np.asarray(node))
        h.update(f"{path}:{a.dtype.str}:{a.shape};".encode())
        h.update(memoryview(a).cast("B"))

    walk(tree, "")
    return h.hexdigest()


PROGRAM_CACHE_SIZE = 4


def cached_program(owner, module, variables, D: int, C: int, latent=None, cached: bool = True) -> "Program":
    """The device program of ``module`` for these variables, cached on
    ``owner`` per (content digest of the variables, D, C, latent) so that
    repeated ``apply(variables, x)`` calls pack and upload the weights once;
    a digest (xxh3 over every leaf's bytes, ~0.1 ms/MB) rather than object
    identity, because numpy leaves can be changed in place.  Train-mode
    calls (``cached=False``) write batch statistics into their program and
    never share it."""
    if not cached:
        return Program(module, variables, D, C, latent=latent)
    key = (_digest(variables), int(D), int(C), type(latent).__name__,
           getattr(latent, "peakness", None), getattr(latent, "_dim", None))
    cache = owner.__dict__.setdefault("_programs", OrderedDict())
    prog = cache.get(key)
    if prog is None:
        prog = Program(module, variables, D, C, latent=latent)
        cache[key] = prog
        while len(cache) > PROGRAM_CACHE_SIZE:
            cache.popitem(last=False)
    else:
        cache.move_to_end(key)
    return prog
