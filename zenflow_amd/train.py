"""Training (zenflow.train, src/zenflow/train.py:18-138) on the GPU.

``loss_fn`` (train.py:64-72) is -mean(log_prob) of a train-mode forward —
ShiftBounds and BatchNorm on batch statistics — and ``step`` (:80-86) applies
its gradient with an optax-style (n)adamw update.  Both run in the library's
trainer (include/zenflow_amd.h, zf_trainer_*): the forward with stored
activations, the reverse pass through RQ splines, conditioner MLPs and
BatchNorm, and the optimiser, all on the device in the natural FLAX blob
layout.  ``metric_fn`` (:74-78) is the eval-mode log_prob of the fused
kernels.

Not reproducible offline (no JAX / optax here): jax.random's init and
permutation streams (seeded numpy generators stand in) and optax's exact
floating-point order; the optimiser restates optax's published update
(scale_by_adam with nesterov for nadamw -> add_decayed_weights -> scale by
-learning_rate).  Every gradient element is checked against float64
autograd of the oracle's loss (oracle/zf_oracle_torch.py,
tests/test_gpu_train.py::test_train_gradient_per_parameter)."""

from __future__ import annotations

import ctypes as ct
import warnings
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import _lib as L
from ._lib import DeviceArray, check
from .dist import shard_rows
from .random import PRNGKey


@dataclass
class Optimizer:
    """optax.adamw / optax.nadamw hyper-parameters (optax defaults)."""

    learning_rate: float = 1e-3
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8
    weight_decay: float = 1e-4
    nesterov: bool = True

    def desc(self) -> L.ZfOptimDesc:
        return L.ZfOptimDesc(self.learning_rate, self.b1, self.b2, self.eps, self.weight_decay,
                             1 if self.nesterov else 0)


def nadamw(learning_rate: float = 1e-3, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
           weight_decay: float = 1e-4) -> Optimizer:
    return Optimizer(learning_rate, b1, b2, eps, weight_decay, True)


def adamw(learning_rate: float = 1e-3, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
          weight_decay: float = 1e-4) -> Optimizer:
    return Optimizer(learning_rate, b1, b2, eps, weight_decay, False)


# |sum(lp)| from which the fp32 sum of the reference's jnp.mean is infinite
_F32_SUM_LIMIT = float(np.finfo(np.float32).max)

DEFAULT_OPTIMIZER = nadamw  # train.py:13-16 (optax.nadamw when available)


class Trainer:
    """Device-resident training state of one Flow: natural blob (params +
    batch statistics), gradient, optimiser moments, activation arena for
    batches of up to ``batch_max`` rows."""

    def __init__(self, flow, variables: Dict[str, Any], D: int, C: int, batch_max: int,
                 optimizer: Optional[Optimizer] = None, comm=None):
        """``comm``: data parallelism — an object with ``rank``, ``world`` and
        ``trainer_comm_desc()`` (``dist.RcclCommunicator``, or
        ``dist.HostAllgather`` for ranks sharing a GPU); each rank then passes
        its shard of every global batch."""
        L.ensure_device()
        self.flow = flow
        self.D, self.C = int(D), int(C)
        self.batch_max = int(batch_max)
        self.optimizer = optimizer or DEFAULT_OPTIMIZER()
        self.program = flow._program(variables, self.D, self.C)
        prog = self.program
        opt = self.optimizer.desc()
        h = ct.c_void_p()
        check(L.load_library().zf_trainer_create(
            ct.byref(prog.desc), prog.blob.ctypes.data, prog.blob.size, prog.param_mask.ctypes.data,
            self.batch_max, ct.byref(opt), ct.byref(h)), "zf_trainer_create")
        self.handle = h.value
        self._loss = DeviceArray((1,), np.float64)
        self.comm = comm
        self.world = 1
        if comm is not None and comm.world > 1:
            self._comm_desc = comm.trainer_comm_desc()  # kept alive: the C side holds its pointers
            check(L.load_library().zf_trainer_set_comm(self.handle, ct.byref(self._comm_desc)), "zf_trainer_set_comm")
            self.world = comm.world

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and L._lib is not None:
            L._lib.zf_trainer_destroy(ct.c_void_p(h))
            self.handle = None

    def _dev(self, x, cols):
        if x is None:
            return None
        if isinstance(x, DeviceArray):
            return x
        a = np.asarray(x, np.float32)
        if a.ndim == 1:
            a = a.reshape(-1, 1)
        return DeviceArray.from_numpy(np.ascontiguousarray(a))

    def _global(self, rows: int, global_rows: Optional[int]) -> int:
        return int(global_rows) if global_rows is not None else int(rows) * self.world

    def loss_grad(self, x, c=None, update_stats: bool = False,
                  global_rows: Optional[int] = None) -> Tuple[float, np.ndarray]:
        """(loss, gradient in the natural blob layout) — loss_fn + jax.grad.
        Data parallel: ``x`` is this rank's shard of a global batch of
        ``global_rows`` rows (default: equal shards); both results are global."""
        xd, cd = self._dev(x, self.D), self._dev(c, self.C)
        g = DeviceArray((self.program.blob.size,))
        check(L.load_library().zf_trainer_loss_grad_shard(
            self.handle, xd.ptr, None if cd is None else cd.ptr, xd.shape[0], self._global(xd.shape[0], global_rows),
            1 if update_stats else 0, self._loss.ptr, g.ptr, L.stream()), "zf_trainer_loss_grad")
        self._last_rows = self._global(xd.shape[0], global_rows)
        return self._fp32_mean(float(self._loss.numpy()[0])), g.numpy()

    def grad_tree(self, grad_blob: np.ndarray) -> Dict[str, Any]:
        """Gradient blob -> FLAX ``params`` tree (like jax.grad's output)."""
        return {"bijector": self.program.blob_to_variables(grad_blob)["params"]}

    def step(self, x, c=None, global_rows: Optional[int] = None) -> None:
        xd, cd = self._dev(x, self.D), self._dev(c, self.C)
        self._step_rows(xd.ptr, None if cd is None else cd.ptr, xd.shape[0], global_rows)

    def _step_rows(self, xptr: int, cptr: Optional[int], rows: int, global_rows: Optional[int] = None) -> None:
        """One step on ``rows`` device-resident rows (raw pointers; async)."""
        self._last_rows = self._global(rows, global_rows)
        check(L.load_library().zf_trainer_step_shard(self.handle, xptr, cptr, rows, self._global(rows, global_rows),
                                                     self._loss.ptr, L.stream()), "zf_trainer_step")

    def _step_local(self, xptr: int, cptr: Optional[int], rows: int) -> None:
        """One step on the whole batch without the cross-rank reductions:
        every rank holds the same batch, so each computes the one-device
        step itself (a batch with fewer rows than ranks)."""
        lib = L.load_library()
        if self.world > 1:
            check(lib.zf_trainer_set_comm(self.handle, None), "zf_trainer_set_comm")
        try:
            self._last_rows = rows
            check(lib.zf_trainer_step_shard(self.handle, xptr, cptr, rows, rows, self._loss.ptr, L.stream()),
                  "zf_trainer_step")
        finally:
            if self.world > 1:
                check(lib.zf_trainer_set_comm(self.handle, ct.byref(self._comm_desc)), "zf_trainer_set_comm")

    def last_loss(self) -> float:
        return self._fp32_mean(float(self._loss.numpy()[0]))

    def _fp32_mean(self, loss: float) -> float:
        """The device loss is -sum(lp / B) in fp64; the reference's loss_fn
        (train.py:70-72) is jnp.mean in fp32, whose sum overflows to +-inf once
        |sum(lp)| leaves the fp32 range (two rows at finfo.min) — the same rule
        as dist.nll_from_sum, applied to the global batch of the last call."""
        from .dist import nll_from_sum

        B = getattr(self, "_last_rows", None)
        if B is None or loss != loss:
            return loss
        return nll_from_sum(-loss * B, B) if abs(loss * B) >= _F32_SUM_LIMIT else loss

    def variables(self) -> Dict[str, Any]:
        blob = np.empty_like(self.program.blob)
        check(L.load_library().zf_trainer_get_blob(self.handle, blob.ctypes.data), "zf_trainer_get_blob")
        v = self.program.blob_to_variables(blob)
        return {"params": {"bijector": v["params"]}, "batch_stats": {"bijector": v["batch_stats"]}}


def _metric(flow, variables, x, c) -> float:
    """metric_fn (train.py:74-78): -mean(log_prob), eval mode."""
    from .dist import nll_from_sum

    lp = np.asarray(flow.apply(variables, x, c), np.float64)
    return nll_from_sum(lp.sum(), lp.shape[0])


def train(
    flow,
    X_train,
    X_test,
    C_train=None,
    C_test=None,
    *,
    epochs: int = 1000,
    batch_size: int = 1024,
    optimizer: Optional[Optimizer] = None,
    patience: float = 0.05,
    warmup: float = 0.2,
    seed: int = 0,
    progress: bool = True,
    initial_variables=None,
    comm=None,
) -> Tuple[Dict[str, Any], int, List[float], List[float]]:
    """Trains the normalizing flow on the provided inputs (train.py:18-138).

    Same arguments, defaults, early stopping and return value
    ``(best_variables, best_epoch, loss_train, loss_test)`` as the reference;
    ``optimizer`` is an :class:`Optimizer` (``nadamw(...)`` / ``adamw(...)``).

    ``comm`` (data parallelism, one process per GPU, every rank calling with
    the same data and seed): each global batch of ``batch_size`` rows is cut
    into contiguous per-rank shards (``dist.shard_rows``); the trainer's
    reductions make every rank's parameters identical after every step, and
    equal to one device's when every batch splits evenly.  A batch with fewer
    rows than ranks is stepped by every rank on the whole batch, without
    reductions (the one-device step)."""
    if warmup < 1:
        warmup = warmup * epochs
    warmup = int(warmup)
    if patience < 1:
        patience = patience * epochs
    patience = int(patience)

    X_train = np.asarray(X_train, np.float32)
    X_test = np.asarray(X_test, np.float32)
    C_train = None if C_train is None else np.asarray(C_train, np.float32)
    C_test = None if C_test is None else np.asarray(C_test, np.float32)
    if C_train is not None and C_train.ndim == 1:
        C_train = C_train.reshape(-1, 1)
    if C_test is not None and C_test.ndim == 1:
        C_test = C_test.reshape(-1, 1)

    if initial_variables is None:
        variables = flow.init(PRNGKey(seed), X_train[:1], None if C_train is None else C_train[:1])
    else:
        variables = initial_variables
    D = X_train.shape[1]
    Cd = 0 if C_train is None else C_train.shape[1]
    world = 1 if comm is None else int(comm.world)
    rank = 0 if comm is None else int(comm.rank)
    shard_max = -(-min(batch_size, X_train.shape[0]) // world)
    trainer = Trainer(flow, variables, D, Cd, shard_max, optimizer, comm=comm)

    loop = range(epochs)
    if progress:
        try:
            from tqdm import tqdm

            loop = tqdm(loop)
        except ModuleNotFoundError:  # pragma: no cover
            pass

    loss_train: List[float] = []
    loss_test: List[float] = []
    best_epoch = 0
    best_variables = variables
    X = C = None
    n = X_train.shape[0]
    for epoch in loop:
        perm = np.random.default_rng([seed, epoch]).permutation(n)
        X_perm = X_train[perm]
        C_perm = None if C_train is None else C_train[perm]
        # one upload per epoch; batches are row ranges of the resident copy
        X_dev = DeviceArray.from_numpy(X_perm)
        C_dev = None if C_perm is None else DeviceArray.from_numpy(C_perm)
        for batch_idx in range(0, n, batch_size):
            rows = min(batch_size, n - batch_idx)
            if rows < world:
                trainer._step_local(X_dev.ptr + batch_idx * D * 4,
                                    None if C_dev is None else C_dev.ptr + batch_idx * Cd * 4, rows)
                continue
            if rows % world and epoch == 0:
                warnings.warn(f"batch of {rows} rows does not split evenly over {world} ranks: ranks stay "
                              "identical but their fp64 reduction order differs from one device's", RuntimeWarning)
            lo, hi = shard_rows(rows, rank, world)
            trainer._step_rows(X_dev.ptr + (batch_idx + lo) * D * 4,
                               None if C_dev is None else C_dev.ptr + (batch_idx + lo) * Cd * 4, hi - lo, rows)
        X = X_perm[batch_idx : batch_idx + batch_size]
        C = None if C_perm is None else C_perm[batch_idx : batch_idx + batch_size]

        variables = trainer.variables()
        loss_train.append(_metric(flow, variables, X, C))  # last batch, as train.py:122
        loss_test.append(_metric(flow, variables, X_test, C_test))

        if not np.isfinite(loss_train[-1]):
            warnings.warn(f"epoch {epoch}: loss[train] not finite, abort training", RuntimeWarning)
            break

        if loss_test[-1] <= loss_test[best_epoch]:
            best_epoch = epoch
            best_variables = variables

        if epoch >= warmup and epoch >= 2 * patience and epoch % patience == 0:
            if not np.min(loss_test[-patience:]) < np.min(loss_test[-2 * patience : -patience]):
                break
    return best_variables, best_epoch, loss_train, loss_test
