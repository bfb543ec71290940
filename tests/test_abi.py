"""The C-ABI library loads on a CPU-only host and exports every symbol that
include/zenflow_amd.h declares; host-only entry points (planning, error
reporting) behave.  No GPU compute is called here."""

import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "zenflow_amd.h"


def header_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**\s*(zf_[a-z_0-9]+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_header_parses():
    names = header_functions()
    assert "zf_flow_log_prob" in names and "zf_rqs_forward" in names
    assert len(names) >= 40


def test_library_exports_every_header_symbol():
    from zenflow_amd import _lib

    lib = _lib.load_library()
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes binding declares exactly the header's functions
    assert sorted(_lib.SIGNATURES) == header_functions()


def test_struct_layout_matches_header():
    from zenflow_amd import _lib

    assert ctypes.sizeof(_lib.ZfOpDesc) == 4 * 22 + 8 * (1 + 17 + 17 + 1)
    assert _lib.ZfFlowDesc.ops.offset == 24
    assert ctypes.sizeof(_lib.ZfFlowDesc) == 24 + 64 * ctypes.sizeof(_lib.ZfOpDesc)


def _desc(D, C, ops):
    from zenflow_amd import _lib as L

    d = L.ZfFlowDesc()
    d.dim, d.cond_dim, d.latent, d.n_ops = D, C, L.ZF_LATENT_NORMAL, len(ops)
    for i, op in enumerate(ops):
        o = d.ops[i]
        o.kind = op[0]
        if op[0] == L.ZF_OP_NSC:
            o.knots = op[1]
            o.n_hidden = len(op[2])
            for l, w in enumerate(op[2]):
                o.hidden[l] = w
        elif op[0] == L.ZF_OP_ROLL:
            o.shift = 1
    return d


def test_flow_plan_offsets_cfg2():
    """zf_flow_plan is host-only: the natural blob of rolling_spline_coupling(4,
    K=16, (128,128)) has exactly the FLAX parameter count + BN + SB records."""
    from zenflow_amd import _lib as L

    lib = L.load_library()
    nsc = (L.ZF_OP_NSC, 16, (128, 128))
    ops = [(L.ZF_OP_SHIFT_BOUNDS,)] + [nsc, (L.ZF_OP_ROLL,)] * 3 + [nsc]
    d = _desc(4, 0, ops)
    n = ctypes.c_int64()
    assert lib.zf_flow_plan(ctypes.byref(d), ctypes.byref(n)) == 0
    per_nsc = 4 * 2 + (2 * 128 + 128) + (128 * 128 + 128) + (128 * 94 + 94)
    assert n.value == 8 * 4 + 4 * per_nsc
    assert d.ops[0].off_sb == 0
    assert d.ops[1].off_bn == 32 and d.ops[1].off_w[0] == 40


@pytest.mark.parametrize(
    "D,ops,err",
    [
        (1, [(3, 16, (128,))], ValueError),  # NSC needs D >= 2
        (4, [(3, 0, (128,))], ValueError),  # knots < 1
        (4, [(3, 16, (5000,))], NotImplementedError),  # width > 4096 (257..4096 run layered)
        (4, [(9,)], ValueError),  # unknown op
    ],
)
def test_flow_plan_rejects(D, ops, err):
    from zenflow_amd import _lib as L

    d = _desc(D, 0, ops)
    n = ctypes.c_int64()
    rc = L.load_library().zf_flow_plan(ctypes.byref(d), ctypes.byref(n))
    with pytest.raises(err):
        L.check(rc, "zf_flow_plan")
    assert L.load_library().zf_last_error()


def test_no_gpu_fails_loudly(monkeypatch):
    """Without a GPU the product path raises instead of falling back to CPU."""
    from zenflow_amd import _lib as L

    if L.device_count() > 0:
        pytest.skip("a GPU is visible")
    monkeypatch.setattr(L, "_device_ready", False)
    with pytest.raises(RuntimeError, match="no HIP device"):
        L.ensure_device()
    import zenflow_amd.utils as u

    with pytest.raises(RuntimeError):
        u.rational_quadratic_spline_forward(np.zeros((1, 1)), np.ones((1, 1, 1)), np.ones((1, 1, 1)),
                                            np.ones((1, 1, 0)))


def test_header_constants_match_python():
    """Every `#define ZF_<NAME> <int>` of include/zenflow_amd.h that the
    Python side mirrors (`zenflow_amd._lib`) has the same value there."""
    from zenflow_amd import _lib as L

    hdr = (Path(__file__).resolve().parents[1] / "include" / "zenflow_amd.h").read_text()
    defs = dict(re.findall(r"^#define (ZF_[A-Z0-9_]+)\s+(-?\d+)\b", hdr, re.M))
    assert "ZF_KERNEL_LAYERED" in defs
    mirrored = [n for n in defs if hasattr(L, n)]
    assert len(mirrored) >= 20, mirrored
    for n in mirrored:
        assert getattr(L, n) == int(defs[n]), n
