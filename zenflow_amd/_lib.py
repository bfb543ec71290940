"""ctypes binding of libzenflow_amd.so (the C ABI in include/zenflow_amd.h).

The product path has no fallback: if the HIP library is missing or no GPU is
visible, every compute entry point raises ``RuntimeError``.  Loading the
library itself needs no GPU (the ABI tests load it on a CPU-only host).
"""

from __future__ import annotations

import ctypes as C
import os
import threading
import weakref
from pathlib import Path
from typing import Optional, Sequence, Tuple, Union

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("ZF_LIB", _HERE / "libzenflow_amd.so"))

ZF_OP_SHIFT_BOUNDS = 1
ZF_OP_ROLL = 2
ZF_OP_NSC = 3
ZF_LATENT_NONE = 0
ZF_LATENT_NORMAL = 1
ZF_LATENT_BETA = 2
ZF_LATENT_TRUNCNORM = 3
ZF_LATENT_UNIFORM = 4
ZF_ACT_SWISH = 0
ZF_ACT_RELU = 1
ZF_ACT_TANH = 2
ZF_ACT_SIGMOID = 3
ZF_ACT_GELU = 4
ZF_ACT_SOFTPLUS = 5
ZF_ACT_ELU = 6
ZF_ACT_LEAKY_RELU = 7
ZF_SB_NONE = 0
ZF_SB_BOTH = 1
ZF_SB_LOWER = 2
ZF_SB_UPPER = 3
ZF_KERNEL_FP32 = 0
ZF_KERNEL_BF16X3 = 1
ZF_KERNEL_F16X2 = 2
ZF_KERNEL_LAYERED = 3


class ZfOpDesc(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("shift", C.c_int32),
        ("knots", C.c_int32),
        ("n_hidden", C.c_int32),
        ("hidden", C.c_int32 * 16),
        ("act", C.c_int32),
        ("_pad", C.c_int32),
        ("off_bn", C.c_int64),
        ("off_w", C.c_int64 * 17),
        ("off_b", C.c_int64 * 17),
        ("off_sb", C.c_int64),
    ]


class ZfOptimDesc(C.Structure):
    _fields_ = [("learning_rate", C.c_float), ("b1", C.c_float), ("b2", C.c_float), ("eps", C.c_float),
                ("weight_decay", C.c_float), ("nesterov", C.c_int)]


# zf_allgather_fn(ctx, send, recv, bytes, stream) and zf_comm_desc
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


class ZfCommDesc(C.Structure):
    _fields_ = [("rank", C.c_int), ("world", C.c_int), ("ctx", C.c_void_p), ("allgather", C.c_void_p)]


class ZfFlowDesc(C.Structure):
    _fields_ = [
        ("dim", C.c_int32),
        ("cond_dim", C.c_int32),
        ("latent", C.c_int32),
        ("latent_param", C.c_float),
        ("n_ops", C.c_int32),
        ("_pad", C.c_int32),
        ("ops", ZfOpDesc * 64),
    ]


_vp = C.c_void_p
_i64 = C.c_int64
_int = C.c_int
_u64 = C.c_uint64
_dbl = C.c_double

# name -> (restype, argtypes); mirrors include/zenflow_amd.h one-to-one.
SIGNATURES = {
    "zf_last_error": (C.c_char_p, []),
    "zf_version": (_int, []),
    "zf_device_count": (_int, [C.POINTER(_int)]),
    "zf_set_device": (_int, [_int]),
    "zf_get_device": (_int, [C.POINTER(_int)]),
    "zf_device_name": (_int, [_int, C.c_char_p, _int]),
    "zf_device_synchronize": (_int, []),
    "zf_malloc": (_int, [C.POINTER(_vp), C.c_size_t]),
    "zf_free": (_int, [_vp]),
    "zf_memset_async": (_int, [_vp, _int, C.c_size_t, _vp]),
    "zf_memcpy_htod": (_int, [_vp, _vp, C.c_size_t, _vp]),
    "zf_memcpy_dtoh": (_int, [_vp, _vp, C.c_size_t, _vp]),
    "zf_memcpy_dtod": (_int, [_vp, _vp, C.c_size_t, _vp]),
    "zf_stream_create": (_int, [C.POINTER(_vp)]),
    "zf_stream_destroy": (_int, [_vp]),
    "zf_stream_synchronize": (_int, [_vp]),
    "zf_event_create": (_int, [C.POINTER(_vp)]),
    "zf_event_destroy": (_int, [_vp]),
    "zf_event_record": (_int, [_vp, _vp]),
    "zf_stream_wait_event": (_int, [_vp, _vp]),
    "zf_event_elapsed_ms": (_int, [_vp, _vp, C.POINTER(C.c_float)]),
    "zf_event_synchronize": (_int, [_vp]),
    "zf_rqs_forward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _vp]),
    "zf_rqs_inverse": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _int, _int, _vp]),
    "zf_normalize_spline_params": (_int, [_vp, _vp, _vp, _i64, _int, _vp]),
    "zf_squareplus": (_int, [_vp, _vp, _i64, C.c_float, _vp]),
    "zf_softmax_with_threshold": (_int, [_vp, _vp, _i64, _int, C.c_double, _vp]),
    "zf_flow_plan": (_int, [C.POINTER(ZfFlowDesc), C.POINTER(_i64)]),
    "zf_flow_create": (_int, [C.POINTER(ZfFlowDesc), _vp, _i64, C.POINTER(_vp)]),
    "zf_flow_destroy": (_int, [_vp]),
    "zf_flow_kernel_variant": (_int, [_vp]),
    "zf_flow_workspace_bytes": (_i64, [_i64]),
    "zf_flow_log_prob": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "zf_flow_log_prob_segment": (_int, [_vp, _int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "zf_flow_nll_reduce": (_int, [_vp, _i64, _vp, _vp]),
    "zf_flow_forward": (_int, [_vp, _int, _int, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "zf_flow_inverse": (_int, [_vp, _int, _int, _vp, _vp, _vp, _i64, _vp]),
    "zf_flow_sample": (_int, [_vp, _u64, _vp, _vp, _i64, _vp]),
    "zf_trainer_create": (_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp]),
    "zf_trainer_destroy": (_int, [_vp]),
    "zf_trainer_loss_grad": (_int, [_vp, _vp, _vp, _i64, _int, _vp, _vp, _vp]),
    "zf_trainer_step": (_int, [_vp, _vp, _vp, _i64, _vp, _vp]),
    "zf_trainer_set_comm": (_int, [_vp, _vp]),
    "zf_trainer_loss_grad_shard": (_int, [_vp, _vp, _vp, _i64, _i64, _int, _vp, _vp, _vp]),
    "zf_trainer_step_shard": (_int, [_vp, _vp, _vp, _i64, _i64, _vp, _vp]),
    "zf_trainer_get_blob": (_int, [_vp, _vp]),
    "zf_trainer_set_blob": (_int, [_vp, _vp]),
    "zf_latent_sample": (_int, [_int, _dbl, _u64, _vp, _i64, _int, _vp]),
    "zf_flow_set_bn_stats": (_int, [_vp, _int, _vp, _vp]),
    "zf_flow_set_sb_stats": (_int, [_vp, _int, _vp, _vp]),
    "zf_colstats_workspace_bytes": (_i64, [_i64, _int]),
    "zf_colstats": (_int, [_vp, _i64, _int, _i64, _int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "zf_rccl_available": (_int, []),
    "zf_rccl_get_unique_id": (_int, [C.c_char_p]),
    "zf_rccl_comm_init": (_int, [C.POINTER(_vp), _int, C.c_char_p, _int]),
    "zf_rccl_allreduce_sum_f64": (_int, [_vp, _vp, _vp, C.c_size_t, _vp]),
    "zf_rccl_comm_destroy": (_int, [_vp]),
    "zf_rccl_allgather": (_int, [_vp, _vp, _vp, C.c_size_t, _vp]),
}

_lib: Optional[C.CDLL] = None
_lock = threading.Lock()


def load_library() -> C.CDLL:
    """Load libzenflow_amd.so (no GPU needed).  Raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"zenflow_amd: HIP library {LIB_PATH} is missing; build it with "
                "`python -m zenflow_amd.build` (hipcc --offload-arch=gfx950). "
                "There is no CPU fallback."
            )
        lib = C.CDLL(str(LIB_PATH))
        allow_missing = os.environ.get("ZF_ALLOW_MISSING_SYMBOLS") == "1"  # diagnostics only
        for name, (res, args) in SIGNATURES.items():
            if allow_missing and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


class ZfError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load_library().zf_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(f"{what}: {msg}")
        if rc == -2:
            raise NotImplementedError(f"{what}: {msg}")
        raise ZfError(f"{what}: rc={rc}: {msg}")


# ---------------------------------------------------------------------------
# Device / stream
# ---------------------------------------------------------------------------

_stream = None
_device_ready = False


def device_count() -> int:
    n = C.c_int(0)
    rc = load_library().zf_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def select_device(env, n: int) -> int:
    """The device index this process binds (one rank per GPU).

    * ``LOCAL_RANK`` (torchrun / our launcher) picks device LOCAL_RANK; when
      the scheduler masks each rank down to ONE visible device (a
      HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES mask
      is set), LOCAL_RANK >= 1 maps to that device 0 — without a mask, two
      ranks on a one-GPU node are an oversubscribed launch and raise below;
    * ``ZF_DEVICE`` (explicit) overrides it — for ranks that share one GPU on
      purpose (HostAllgather tests); with WORLD_SIZE > 1 that puts several
      ranks on one device, so it warns;
    * a LOCAL_RANK beyond the visible devices of a multi-device process
      (oversubscribed launch) raises before any RCCL call would fail."""
    zf_dev = env.get("ZF_DEVICE")
    local = env.get("LOCAL_RANK")
    if zf_dev is not None and zf_dev != "":
        dev = int(zf_dev)
        if local is not None and int(env.get("WORLD_SIZE", "1")) > 1:
            import warnings

            warnings.warn(f"zenflow_amd: ZF_DEVICE={dev} overrides LOCAL_RANK={local} in a "
                          f"{env.get('WORLD_SIZE')}-rank job (ranks sharing one GPU)", RuntimeWarning, stacklevel=3)
    else:
        dev = int(local or "0")
        masked = any(env.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"))
        if n == 1 and dev >= 1 and masked:
            dev = 0  # the scheduler masked this rank down to its one device
    if not 0 <= dev < n:
        raise RuntimeError(
            f"zenflow_amd: device {dev} (LOCAL_RANK/ZF_DEVICE) is not visible; "
            f"{n} HIP device(s) visible — launch at most one rank per GPU"
        )
    return dev


def ensure_device() -> None:
    """Fail loudly when no GPU is visible (no silent CPU path)."""
    global _device_ready
    if _device_ready:
        return
    if device_count() < 1:
        raise RuntimeError(
            "zenflow_amd: no HIP device is visible; the product path runs only on "
            "MI355X (gfx950) and has no CPU fallback."
        )
    dev = select_device(os.environ, device_count())
    check(load_library().zf_set_device(dev), "zf_set_device")
    _device_ready = True


def stream():
    """The library stream of this process (created lazily)."""
    global _stream
    if _stream is None:
        ensure_device()
        s = C.c_void_p()
        check(load_library().zf_stream_create(C.byref(s)), "zf_stream_create")
        _stream = s.value
    return _stream


def new_stream():
    """A further HIP stream on this process's device (e.g. for communication)."""
    ensure_device()
    s = C.c_void_p()
    check(load_library().zf_stream_create(C.byref(s)), "zf_stream_create")
    return s.value


def synchronize() -> None:
    check(load_library().zf_stream_synchronize(stream()), "zf_stream_synchronize")


def device_name() -> str:
    ensure_device()
    buf = C.create_string_buffer(256)
    dev = C.c_int(0)
    check(load_library().zf_get_device(C.byref(dev)), "zf_get_device")
    check(load_library().zf_device_name(dev.value, buf, 256), "zf_device_name")
    return buf.value.decode()


# ---------------------------------------------------------------------------
# Device arrays
# ---------------------------------------------------------------------------


def _free(ptr):
    if _lib is not None and ptr:
        _lib.zf_free(C.c_void_p(ptr))


class DeviceArray:
    """A contiguous device buffer with a numpy-like shape/dtype.

    Returned by the API when the inputs were DeviceArrays (device in -> device
    out); ``numpy()`` copies it to the host."""

    __slots__ = ("ptr", "shape", "dtype", "nbytes", "_fin", "__weakref__")

    def __init__(self, shape, dtype=np.float32):
        ensure_device()
        self.shape = tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        p = C.c_void_p()
        check(load_library().zf_malloc(C.byref(p), self.nbytes), "zf_malloc")
        self.ptr = p.value
        self._fin = weakref.finalize(self, _free, self.ptr)

    @classmethod
    def from_numpy(cls, a) -> "DeviceArray":
        a = np.ascontiguousarray(a)
        d = cls(a.shape, a.dtype)
        check(load_library().zf_memcpy_htod(d.ptr, a.ctypes.data, a.nbytes, stream()), "htod")
        synchronize()  # the host buffer may be freed right after
        return d

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        check(load_library().zf_memcpy_dtoh(out.ctypes.data, self.ptr, self.nbytes, stream()), "dtoh")
        synchronize()
        return out

    def copy_from(self, other: "DeviceArray") -> None:
        assert other.nbytes == self.nbytes
        check(load_library().zf_memcpy_dtod(self.ptr, other.ptr, self.nbytes, stream()), "dtod")

    def zero_(self) -> "DeviceArray":
        check(load_library().zf_memset_async(self.ptr, 0, self.nbytes, stream()), "memset")
        return self

    @property
    def ndim(self):
        return len(self.shape)

    def __len__(self):
        return self.shape[0]

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def __repr__(self):
        return f"DeviceArray(shape={self.shape}, dtype={self.dtype})"


ArrayLike = Union[np.ndarray, DeviceArray, Sequence]


def as_device(a, dtype=np.float32) -> Tuple[DeviceArray, bool]:
    """Return (device array, was_device).  Host input is converted to ``dtype``
    (integer inputs are cast to float32, as ShiftBounds does, bijectors.py:178)."""
    if isinstance(a, DeviceArray):
        if a.dtype != np.dtype(dtype):
            raise TypeError(f"expected a {np.dtype(dtype)} DeviceArray, got {a.dtype}")
        return a, True
    arr = np.asarray(a)
    return DeviceArray.from_numpy(np.ascontiguousarray(arr, dtype=dtype)), False


class Event:
    def __init__(self):
        e = C.c_void_p()
        check(load_library().zf_event_create(C.byref(e)), "zf_event_create")
        self.ptr = e.value
        self._fin = weakref.finalize(self, lambda p: _lib and _lib.zf_event_destroy(C.c_void_p(p)), self.ptr)

    def record(self, s=None):
        check(load_library().zf_event_record(self.ptr, stream() if s is None else s), "event_record")

    def synchronize(self):
        check(load_library().zf_event_synchronize(self.ptr), "event_sync")

    def wait(self, s=None):
        """Make work queued later on stream `s` (default: the library stream) wait for this event."""
        check(load_library().zf_stream_wait_event(stream() if s is None else s, self.ptr), "stream_wait_event")

    def elapsed_ms(self, end: "Event") -> float:
        ms = C.c_float()
        check(load_library().zf_event_elapsed_ms(self.ptr, end.ptr, C.byref(ms)), "elapsed")
        return float(ms.value)
