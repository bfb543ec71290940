"""Data parallelism across GPUs, one process per GPU.

log_prob: contiguous batch shards and a single all-reduce of the fp64 NLL
partial sum.  Training: the trainer's all-gather at every
batch reduction (``RcclCommunicator.trainer_comm_desc`` / ``HostAllgather``;
zf_trainer_set_comm), with the leaf-tree schedule mirrored on the host by
``reduction_leaves`` / ``tree_sum``.

log_prob is a per-sample map in eval mode (BatchNorm running stats,
ShiftBounds stored min/max), so the only exchange is the scalar
``-mean(log_prob)`` of train.py:75-78.  On GPUs it goes through RCCL over
xGMI (``RcclCommunicator``, librccl via the C ABI).  No torch: ranks are
started by ``launch.spawn`` (or torch.distributed.run, the driver's
launcher) and exchange the RCCL unique id, barriers and timings through
``launch.FileRendezvous``.  The CPU test suite drives the same step sequence
(``DataParallelLogProb``) with a host backend and ``HostCommunicator``."""

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

    def __init__(self, rank: int, world: int, broadcast: Callable[[Optional[bytes]], bytes],
                 force: bool = False):
        self.force = force  # keep a 1-rank communicator in DataParallelLogProb (plumbing checks)
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

    def trainer_comm_desc(self) -> L.ZfCommDesc:
        """zf_comm_desc for data-parallel training (zf_trainer_set_comm):
        the trainer's all-gather is ncclAllGather on this communicator."""
        fn = C.cast(L.load_library().zf_rccl_allgather, C.c_void_p).value
        return L.ZfCommDesc(self.rank, self.world, self.comm, fn)

    def close(self):
        if self.comm:
            L.load_library().zf_rccl_comm_destroy(self.comm)
            self.comm = None


class HostAllgather:
    """zf_allgather_fn over the control-plane rendezvous (device -> host ->
    rank-order gather -> device, synchronous on the trainer's stream).  For
    data-parallel training where RCCL cannot run: several ranks sharing one
    GPU (the multi-process GPU tests; RCCL refuses two ranks on one device).
    The data path of a real multi-GPU job is ``RcclCommunicator``."""

    def __init__(self, rdzv):
        self.rdzv = rdzv
        self.rank, self.world = rdzv.rank, rdzv.world
        self._cb = L.ALLGATHER_FN(self._allgather)  # kept alive with this object

    def _allgather(self, ctx, send, recv, nbytes, stream) -> int:
        try:
            lib = L.load_library()
            buf = C.create_string_buffer(max(1, nbytes))
            check(lib.zf_stream_synchronize(stream), "allgather sync")
            check(lib.zf_memcpy_dtoh(buf, send, nbytes, stream), "allgather dtoh")
            check(lib.zf_stream_synchronize(stream), "allgather sync")
            out = b"".join(self.rdzv.allgather_bytes(buf.raw[:nbytes], "trainer_ag"))
            check(lib.zf_memcpy_htod(recv, out, len(out), stream), "allgather htod")
            check(lib.zf_stream_synchronize(stream), "allgather sync")
            return 0
        except Exception as e:  # a C caller: report, do not unwind through ctypes
            import sys

            print(f"HostAllgather rank {self.rank}: {e!r}", file=sys.stderr, flush=True)
            return 1

    def trainer_comm_desc(self) -> L.ZfCommDesc:
        return L.ZfCommDesc(self.rank, self.world, None, C.cast(self._cb, C.c_void_p).value)

    def close(self):
        pass


def reduction_leaves(rows: int, global_rows: int, world: int, cap: int = 4096) -> Tuple[int, int]:
    """(leaves on this rank, rows per leaf) of every batch reduction of the
    trainer — the host mirror of zf_train.hip ``leaves_for``: ~32 rows per
    leaf, at most ``cap`` (a power of two) leaves in the global batch, a
    power of two per rank."""
    want = max(1, min(int(global_rows) // 32, int(cap)))
    per = max(1, want // max(1, int(world)))
    n = 1 << (per.bit_length() - 1)
    return n, (int(rows) + n - 1) // n


def tree_sum(leaves: np.ndarray) -> np.ndarray:
    """The trainer's pairwise leaf tree (zf_train.hip ``tree_n``) in fp64 over
    axis 0: level s adds element i + s into i for i a multiple of 2s."""
    v = [np.asarray(x, np.float64) for x in leaves]
    n = len(v)
    s = 1
    while s < n:
        for i in range(0, n, 2 * s):
            if i + s < n:
                v[i] = v[i] + v[i + s]
        s *= 2
    return v[0]


def leaf_tree_colsum(x: np.ndarray, global_rows: int, world: int, cap: int = 4096) -> np.ndarray:
    """This rank's subtree root of the column sums of ``x`` (rows x cols,
    fp32): leaves of ``reduction_leaves`` rows summed in row order in fp64,
    then ``tree_sum`` — the schedule of the trainer's BatchNorm sums."""
    n, rows = reduction_leaves(x.shape[0], global_rows, world, cap)
    parts = []
    for z in range(n):
        acc = np.zeros(x.shape[1:], np.float64)
        for b in range(min(x.shape[0], z * rows), min(x.shape[0], (z + 1) * rows)):
            acc = acc + x[b].astype(np.float64)
        parts.append(acc)
    return tree_sum(parts)


class HostCommunicator:
    """Host-side fp64 all-reduce over the control-plane rendezvous
    (``launch.FileRendezvous``): the same ``allreduce_sum_`` interface as
    ``RcclCommunicator`` on numpy buffers, summed in rank order so every rank
    gets the same bits.  Used where there is no GPU (the multi-process CPU
    tests) — the GPU data path uses RCCL."""

    def __init__(self, rdzv):
        self.rdzv = rdzv
        self.rank, self.world = rdzv.rank, rdzv.world

    def allreduce_sum_(self, buf: np.ndarray, stream=None) -> np.ndarray:
        vals = self.rdzv.allgather([float(v) for v in np.asarray(buf, np.float64).ravel()], "allreduce")
        acc = np.zeros(np.asarray(buf).size, np.float64)
        for v in vals:
            acc = acc + np.asarray(v, np.float64)
        buf[...] = acc.reshape(np.shape(buf))
        return buf

    def close(self):
        pass


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


class DeviceLogProbStep:
    """The product backend of a data-parallel log_prob step on this rank's
    GPU: the fused kernel over the resident shard (ShiftBounds -> couplings
    -> latent -> flow.py:47 -> per-block fp64 partials) and the fixed-order
    NLL reduce of those partials, both on the library stream."""

    def __init__(self, program, n_rows: int):
        self.lib = L.load_library()
        self.program = program
        self.n_rows = int(n_rows)
        self.ws = program.workspace(self.n_rows)

    def new_partial(self) -> DeviceArray:
        return DeviceArray((1,), np.float64)

    def kernel(self, x: DeviceArray, c, out: DeviceArray) -> None:
        p = self.program
        check(self.lib.zf_flow_log_prob_segment(p.handle, 0, len(p.ops), x.ptr, p._c_ptr(c), None, out.ptr,
                                                None, self.ws.ptr, self.n_rows, L.stream()), "log_prob")

    def reduce(self, partial: DeviceArray) -> None:
        check(self.lib.zf_flow_nll_reduce(self.ws.ptr, self.n_rows, partial.ptr, L.stream()), "nll_reduce")

    def read(self, partial: DeviceArray) -> float:
        return float(partial.numpy()[0])


class DataParallelLogProb:
    """One rank's step of the data-parallel log_prob: the
    backend's kernel over this rank's shard, its fp64 partial sum of
    log_prob, and the all-reduce of that partial — overlapped on a
    communication stream (``OverlappedAllreduce``, device backends) or in
    order after the reduce.  ``nll(n_total)`` is train.py:78's -mean over the
    global batch.  bench.py drives the device backend with RCCL; the CPU
    tests drive this same sequence with a host backend and
    ``HostCommunicator``."""

    def __init__(self, backend, comm=None, overlap: bool = True, depth: int = 64):
        self.backend = backend
        self.comm = comm if comm is not None and comm.world > 1 or _force(comm) else None
        self.ar = (OverlappedAllreduce(self.comm, depth=depth)
                   if self.comm is not None and overlap else None)
        self.partial = backend.new_partial()
        self.last = None

    def step(self, x, c, out, ev=None) -> None:
        if ev is not None:
            ev[0].record()
        self.backend.kernel(x, c, out)
        if ev is not None:
            ev[1].record()
        if self.ar is not None:
            buf = self.ar.buffer()
            self.backend.reduce(buf)
            self.ar.launch()
            self.last = buf
        else:
            self.backend.reduce(self.partial)
            if self.comm is not None:
                self.comm.allreduce_sum_(self.partial)
            self.last = self.partial

    def nll(self, n_total: int) -> float:
        if self.last is None:
            raise RuntimeError("no step has run")
        return nll_from_sum(self.backend.read(self.last), n_total)


def _force(comm) -> bool:
    """A 1-rank communicator is kept only when asked for (plumbing checks)."""
    return comm is not None and getattr(comm, "force", False)
