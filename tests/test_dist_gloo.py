"""N>1 data-parallel path on CPU over gloo (world size 2): the ranks shard
the batch with zenflow_amd.dist.shard_rows and run dist.DataParallelLogProb
— the step sequence bench.py runs with RCCL — with the oracle as the per-rank
stand-in for the GPU kernel (tests/dist_worker.py) and a gloo communicator
(test-only; the product is torch-free).  The global NLL must equal the
single-process NLL."""

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class GlooCommunicator:
    """fp64 all-reduce through torch.distributed (gloo), with the
    ``allreduce_sum_`` interface of dist.RcclCommunicator (test-only)."""

    def __init__(self):
        import torch.distributed as td

        self.td = td
        self.rank, self.world = td.get_rank(), td.get_world_size()

    def allreduce_sum_(self, buf, stream=None):
        import torch

        t = torch.from_numpy(np.ascontiguousarray(buf, np.float64))
        self.td.all_reduce(t)
        buf[...] = t.numpy()
        return buf


def _worker(rank, world, port, q):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as td

    from tests.dist_worker import OracleLogProbStep
    from tests.flowcases import make_case
    from zenflow_amd.dist import DataParallelLogProb, shard_rows

    td.init_process_group("gloo", rank=rank, world_size=world)
    case = make_case("cfg2", N=1001, seed=5)
    a, b = shard_rows(1001, rank, world)
    dp = DataParallelLogProb(OracleLogProbStep(case), GlooCommunicator(), overlap=False)
    out = np.empty(b - a, np.float32)
    dp.step(case["x"][a:b], None, out)
    q.put((rank, b - a, dp.nll(1001)))
    td.barrier()
    td.destroy_process_group()


def test_two_rank_nll_allreduce():
    from oracle import zf_oracle as O
    from tests.flowcases import make_case

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(world))
    case = make_case("cfg2", N=1001, seed=5)
    lp, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], None)
    ref = O.nll(lp)
    assert sum(r[1] for r in res) == 1001
    for _, _, nll in res:
        assert nll == pytest.approx(ref, rel=1e-12)
