"""Data-parallel log_prob across GPUs: one process per GPU, contiguous batch
shards, and a single all-reduce of the fp64 NLL partial sum.

log_prob is a per-sample map in eval mode (BatchNorm running stats,
ShiftBounds stored min/max), so the only exchange is the scalar
``-mean(log_prob)`` of train.py:75-78.  On GPUs it goes through RCCL over
xGMI (``RcclCommunicator``, librccl via the C ABI); the CPU test suite drives
the same code with a gloo communicator."""

from __future__ import annotations

import ctypes as C
from typing import Callable, Optional, Tuple

import numpy as np

from . import _lib as L
from ._lib import DeviceArray, check


def shard_rows(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, stop) of ``n`` rows for ``rank`` of ``world``."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(int(n), world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


class RcclCommunicator:
    """RCCL communicator of one rank (ncclCommInitRank).  ``broadcast`` sends
    the 128-byte unique id from rank 0 to all ranks (any control plane)."""

    def __init__(self, rank: int, world: int, broadcast: Callable[[Optional[bytes]], bytes]):
        lib = L.load_library()
        L.ensure_device()
        if not lib.zf_rccl_available():
            raise RuntimeError("librccl is not available")
        uid = None
        if rank == 0:
            buf = C.create_string_buffer(128)
            check(lib.zf_rccl_get_unique_id(buf), "zf_rccl_get_unique_id")
            uid = buf.raw
        uid = broadcast(uid)
        comm = C.c_void_p()
        check(lib.zf_rccl_comm_init(C.byref(comm), world, C.create_string_buffer(uid, 128), rank),
              "zf_rccl_comm_init")
        self.comm = comm.value
        self.rank, self.world = rank, world

    def allreduce_sum_(self, buf: DeviceArray, stream=None) -> DeviceArray:
        """In-place fp64 sum across ranks on ``stream`` (default: the library stream)."""
        if buf.dtype != np.float64:
            raise TypeError("fp64 buffer expected")
        check(L.load_library().zf_rccl_allreduce_sum_f64(
            self.comm, buf.ptr, buf.ptr, buf.shape[0] if buf.shape else 1,
            L.stream() if stream is None else stream), "allreduce")
        return buf

    def close(self):
        if self.comm:
            L.load_library().zf_rccl_comm_destroy(self.comm)
            self.comm = None


class GlooCommunicator:
    """Host-side fp64 all-reduce through torch.distributed (gloo) — used by
    the multi-process CPU tests; same interface as RcclCommunicator."""

    def __init__(self):
        import torch.distributed as td

        self.td = td
        self.rank, self.world = td.get_rank(), td.get_world_size()

    def allreduce_sum_host(self, v: np.ndarray) -> np.ndarray:
        import torch

        t = torch.from_numpy(np.ascontiguousarray(v, np.float64))
        self.td.all_reduce(t)
        return t.numpy()


def nll_from_sum(total_sum: float, n_total: int) -> float:
    """-mean(log_prob) (train.py:78) from the all-reduced fp64 sum.

    The reference's ``jnp.mean`` sums in fp32: a sum outside the fp32 range
    (two rows at finfo.min after flow.py:47 suffice) makes its NLL infinite,
    so the fp64 sum keeps that overflow instead of returning a finite mean."""
    total_sum = float(total_sum)
    if total_sum != total_sum:
        return float("nan")
    if abs(total_sum) >= _F32_MAX_ROUND:  # ties round to even = inf
        return float("inf") if total_sum < 0 else float("-inf")
    return float(-total_sum / max(1, n_total))


# |s| above which fp32 rounding of s gives inf: FLT_MAX + half an ulp (2^103)
_F32_MAX_ROUND = float(np.finfo(np.float32).max) + 2.0 ** 103


class OverlappedAllreduce:
    """All-reduce of a per-step fp64 partial on a communication stream, off
    the compute stream's critical path: step i's reduce output (slot i of a
    ring of buffers) is handed to the comm stream by an event, and the
    compute stream waits only when it comes back to a slot — ``depth`` steps
    later — for the all-reduce that last read it.  Ranks are thus not put in
    lockstep by every step's collective; the caller synchronises the device
    at the end."""

    def __init__(self, comm: RcclCommunicator, count: int = 1, depth: int = 64):
        from ._lib import Event

        self.comm = comm
        self.depth = depth
        self.stream = L.new_stream()
        self.bufs = [DeviceArray((count,), np.float64) for _ in range(depth)]
        self.ready = [Event() for _ in range(depth)]
        self.done = [Event() for _ in range(depth)]
        self.pending = [False] * depth
        self.i = 0
        self.last = None

    def buffer(self) -> DeviceArray:
        """The buffer this step's partial goes into (on reuse of a slot the
        compute stream first waits for the slot's previous all-reduce)."""
        k = self.i % self.depth
        if self.pending[k]:
            self.done[k].wait()
        return self.bufs[k]

    def launch(self) -> None:
        """All-reduce this step's buffer once the compute stream has filled it."""
        k = self.i % self.depth
        self.ready[k].record()
        self.ready[k].wait(self.stream)
        self.comm.allreduce_sum_(self.bufs[k], stream=self.stream)
        self.done[k].record(self.stream)
        self.pending[k] = True
        self.last = self.bufs[k]
        self.i += 1


class ShardedLogProb:
    """log_prob over this rank's shard + global NLL (RCCL all-reduce)."""

    def __init__(self, bound_flow, comm: Optional[RcclCommunicator]):
        self.bf = bound_flow
        self.comm = comm
        self.nll = DeviceArray((1,), np.float64)

    def __call__(self, x_shard: DeviceArray, c_shard=None, out=None) -> DeviceArray:
        lp = self.bf.log_prob(x_shard, c_shard, out=out, nll_sum=self.nll)
        if self.comm is not None and self.comm.world > 1:
            self.comm.allreduce_sum_(self.nll)
        return lp

    def nll_value(self, n_total: int) -> float:
        return nll_from_sum(float(self.nll.numpy()[0]), n_total)
