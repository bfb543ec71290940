"""Rank program for the multi-process CPU tests (tests/test_dist_launch.py):
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
    rdzv.close()
    Path(outdir, f"rank{rank}.json").write_text(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
