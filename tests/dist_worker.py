"""Rank program for the multi-process tests (tests/test_dist_launch.py on
CPU; tests/test_gpu_train_dp.py: ranks sharing the GPU):
started by zenflow_amd.launch.spawn or by the tests' own torchrun-style
launcher.  ``python tests/dist_worker.py <mode> <outdir>``; writes
<outdir>/rank<r>.json."""

import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


class OracleLogProbStep:
    """Host backend of dist.DataParallelLogProb: the CPU oracle stands in for
    the GPU kernel (the tests run without a GPU); partials are fp64 arrays."""

    def __init__(self, case):
        self.case = case

    def new_partial(self):
        return np.zeros(1, np.float64)

    def kernel(self, x, c, out):
        from oracle import zf_oracle as O

        lp, _ = O.flow_log_prob(self.case["model"], self.case["variables"], x, c)
        out[...] = lp
        self._last = out

    def reduce(self, partial):
        partial[0] = self._last.astype(np.float64).sum()

    def read(self, partial):
        return float(partial[0])


def tree_data(rows):
    """fp32 rows spanning 2^-40..2^40: fp64 sums of them depend on the order."""
    rng = np.random.default_rng(3)
    return (rng.standard_normal((rows, 5)) * np.exp2(rng.integers(-40, 40, (rows, 5)))).astype(np.float32)


def main(mode, outdir):
    from tests.flowcases import make_case
    from zenflow_amd.dist import DataParallelLogProb, HostCommunicator, shard_rows
    from zenflow_amd.launch import FileRendezvous

    rdzv = FileRendezvous.from_env(timeout=120)
    rank, world = rdzv.rank, rdzv.world
    res = {"rank": rank, "world": world, "dir": str(rdzv.path)}
    if mode == "prims":
        res["gather"] = rdzv.allgather({"r": rank, "sq": rank * rank}, "g")
        res["bcast"] = rdzv.broadcast_bytes(b"uid-%d" % 7 if rank == 0 else None, tag="uid").decode()
        res["max"] = rdzv.max(1.5 * rank, "m")
        res["sum"] = rdzv.sum(0.1 * (rank + 1), "s")
        rdzv.barrier("b")
    elif mode == "nll":
        n = 1001
        case = make_case("cfg2", N=n, seed=5)
        a, b = shard_rows(n, rank, world)
        be = OracleLogProbStep(case)
        dp = DataParallelLogProb(be, HostCommunicator(rdzv), overlap=False)
        out = np.empty(b - a, np.float32)
        dp.step(case["x"][a:b], None, out)
        res["rows"] = b - a
        res["nll"] = dp.nll(n)
        res["lp"] = out.tolist()
    elif mode == "tree":
        # the trainer's reduction schedule on host data: this rank's subtree
        # root, all-gathered, combined by the top of the tree
        from zenflow_amd.dist import leaf_tree_colsum, tree_sum

        Bg = int(os.environ.get("ZF_TEST_ROWS", "1024"))
        x = tree_data(Bg)
        a, b = shard_rows(Bg, rank, world)
        root = leaf_tree_colsum(x[a:b], Bg, world)
        parts = [np.frombuffer(p, np.float64) for p in rdzv.allgather_bytes(root.tobytes(), "roots")]
        res["sum"] = tree_sum(parts).tobytes().hex()
    elif mode == "train_dp":
        _train_dp(rdzv, res, outdir)
    elif mode == "train_fn":
        _train_fn(rdzv, res, outdir)
    elif mode == "train_rccl":
        _train_dp(rdzv, res, outdir, rccl=True)
    rdzv.close()
    Path(outdir, f"rank{rank}.json").write_text(json.dumps(res))


def _train_dp(rdzv, res, outdir, rccl=False):
    """One rank of data-parallel training: loss_grad on this rank's shard,
    then ZF_TEST_STEPS optimiser steps; the gradient, loss and final blob go
    to <outdir>/rank<r>.npz.  Ranks share one GPU through HostAllgather, or
    (``rccl``) each rank drives its own GPU (LOCAL_RANK) over RCCL."""
    from tests.flowcases import build_flow, make_case
    from zenflow_amd.dist import HostAllgather, RcclCommunicator, shard_rows
    from zenflow_amd.train import Trainer

    name, N, seed = os.environ["ZF_TEST_CASE"].split(":")
    N, seed = int(N), int(seed)
    steps = int(os.environ.get("ZF_TEST_STEPS", "3"))
    case = make_case(name, N=N, seed=seed)
    cfg = case["cfg"]
    flow = build_flow(cfg)
    flow.latent._dim = cfg["D"]
    if rccl:
        comm = RcclCommunicator(rdzv.rank, rdzv.world, lambda u: rdzv.broadcast_bytes(u, tag="rccl_uid"))
    else:
        comm = HostAllgather(rdzv)
    a, b = shard_rows(N, rdzv.rank, rdzv.world)
    x = case["x"][a:b]
    c = None if case["c"] is None else case["c"][a:b]
    tr = Trainer(flow, case["variables"], cfg["D"], cfg["C"], b - a, comm=comm)
    loss, g = tr.loss_grad(x, c, global_rows=N)
    for _ in range(steps):
        tr.step(x, c, global_rows=N)
    blob = np.empty_like(tr.program.blob)
    from zenflow_amd import _lib as L

    L.check(L.load_library().zf_trainer_get_blob(tr.handle, blob.ctypes.data), "get_blob")
    np.savez(Path(outdir, f"rank{rdzv.rank}.npz"), grad=g, loss=np.float64(loss), blob=blob,
             last_loss=np.float64(tr.last_loss()))
    res["rows"] = b - a
    if rccl:
        comm.close()


def two_moons_flow():
    import zenflow_amd as zf
    from zenflow_amd import bijectors as bi
    from zenflow_amd import distributions as dist

    return zf.Flow(bi.rolling_spline_coupling(2, knots=8, layers=(64, 64)), latent=dist.Beta())


def two_moons_data():
    from sklearn.datasets import make_moons

    X, _ = make_moons(3000, noise=0.05, random_state=2)
    return X.astype(np.float32)


def _train_fn(rdzv, res, outdir):
    """zenflow_amd.train(..., comm=HostAllgather) on every rank: the same
    data and seed, each rank stepping on its shard of every batch."""
    import zenflow_amd as zf
    from zenflow_amd.dist import HostAllgather
    from zenflow_amd.io import flatten_variables

    X = two_moons_data()
    n = int(os.environ.get("ZF_TEST_NTRAIN", "2400"))
    best, best_epoch, lt, ls = zf.train(two_moons_flow(), X[:n], X[2400:], epochs=int(os.environ.get("ZF_TEST_EPOCHS", "20")),
                                        batch_size=512, progress=False, comm=HostAllgather(rdzv))
    np.savez(Path(outdir, f"rank{rdzv.rank}.npz"), best_epoch=best_epoch, lt=np.asarray(lt), ls=np.asarray(ls),
             **{"v:" + k: v for k, v in flatten_variables(best).items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
