"""The N>1 control plane without torch (zenflow_amd.launch) and the
data-parallel step sequence (zenflow_amd.dist.DataParallelLogProb) on CPU:
ranks started by launch.spawn and by a torchrun-style env (no
ZF_RDZV_DIR), exchanging through the file rendezvous; and bench.py
--gpus 2 spawning its own ranks."""

import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
WORKER = str(ROOT / "tests" / "dist_worker.py")


def _results(d, world):
    return [json.loads((Path(d) / f"rank{r}.json").read_text()) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3])
def test_spawn_rendezvous_primitives(tmp_path, world):
    from zenflow_amd.launch import spawn

    assert spawn(world, [WORKER, "prims", str(tmp_path)], timeout=120) == 0
    res = _results(tmp_path, world)
    for r in res:
        assert r["world"] == world
        assert r["gather"] == [{"r": k, "sq": k * k} for k in range(world)]
        assert r["bcast"] == "uid-7"
        assert r["max"] == 1.5 * (world - 1)
        assert r["sum"] == res[0]["sum"]  # same bits on every rank (rank-order sum)
    assert len({r["dir"] for r in res}) == 1
    assert not Path(res[0]["dir"]).exists()  # spawn removed its rendezvous directory


def test_spawn_reports_failing_rank(tmp_path):
    from zenflow_amd.launch import spawn

    code = "import os,sys; sys.exit(3 if os.environ['RANK']=='1' else 0)"
    assert spawn(2, ["-c", code], timeout=60) == 3


def test_two_rank_nll_step(tmp_path):
    """DataParallelLogProb over 2 spawned ranks (host backend + host
    communicator) = the single-process NLL over the whole batch."""
    from oracle import zf_oracle as O
    from tests.flowcases import make_case
    from zenflow_amd.launch import spawn

    assert spawn(2, [WORKER, "nll", str(tmp_path)], timeout=180) == 0
    res = _results(tmp_path, 2)
    case = make_case("cfg2", N=1001, seed=5)
    lp, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], None)
    assert sum(r["rows"] for r in res) == 1001
    assert np.array_equal(np.concatenate([np.asarray(r["lp"], np.float32) for r in res]), lp)
    assert res[0]["nll"] == res[1]["nll"]
    assert res[0]["nll"] == pytest.approx(O.nll(lp), rel=1e-12)


def test_torchrun_style_env(tmp_path):
    """Ranks launched with RANK/WORLD_SIZE/MASTER_PORT only (as
    torch.distributed.run does, one parent) derive one shared directory."""
    env = {k: v for k, v in os.environ.items() if k != "ZF_RDZV_DIR"}
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                 MASTER_PORT="29517")
        procs.append(subprocess.Popen([sys.executable, WORKER, "prims", str(tmp_path)], env=e))
    assert [p.wait(timeout=120) for p in procs] == [0, 0]
    res = _results(tmp_path, 2)
    assert res[0]["dir"] == res[1]["dir"] and "29517" in res[0]["dir"]
    assert res[1]["bcast"] == "uid-7"
    assert not Path(res[0]["dir"]).exists()  # rank 0 cleaned up


@pytest.mark.parametrize("world", [2, 8])
def test_bench_spawns_ranks(world):
    """`python bench.py --gpus N` with no launcher starts N ranks itself;
    on this GPU-less host each reaches the no-device error of the product
    path (no CPU fallback)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ZF_RDZV_DIR")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert p.stderr.count("no HIP device is visible") == world, p.stderr[-2000:]


@pytest.mark.parametrize("config,world,batch", [("cfg5", 8, 1 << 23), ("cfg2", 8, 1 << 23), ("cfg2", 1, 1 << 20),
                                                ("cfg5", 2, 1 << 21)])
def test_bench_dry_run_global_batch(config, world, batch):
    """The scaling run's shapes: cfg5 at --gpus 8 is
    BASELINE's 2^23-row batch sharded 2^20 rows per GPU (weak scaling); the
    ranks rendezvous, rank 0 prints the config, no GPU is touched."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ZF_RDZV_DIR")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--config", config, "--dry-run"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["config"]["global_batch"] == batch
    assert out["config"]["rows_per_gpu"] == 1 << 20


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr


@pytest.mark.parametrize("world,rows", [(2, 1024), (4, 1024), (2, 4096), (8, 2048)])
def test_trainer_reduction_schedule_rank_invariant(tmp_path, world, rows):
    """The trainer's batch-reduction schedule (leaves of ~32 rows whose count
    depends on the global batch only, a pairwise fp64 tree, ranks combining
    their subtree roots by the top of the tree; zenflow_amd.dist mirrors
    zf_train.hip's leaves_for / tree_n): `world` ranks produce bit for bit the
    one-device sum of the whole batch, on every rank."""
    from zenflow_amd.dist import leaf_tree_colsum, reduction_leaves
    from zenflow_amd.launch import spawn

    n1, r1 = reduction_leaves(rows, rows, 1)
    nw, rw = reduction_leaves(rows // world, rows, world)
    assert n1 == nw * world and r1 == rw
    env = dict(os.environ, ZF_TEST_ROWS=str(rows))
    assert spawn(world, [WORKER, "tree", str(tmp_path)], env=env, timeout=120) == 0
    res = _results(tmp_path, world)
    from tests.dist_worker import tree_data

    x = tree_data(rows)
    one = leaf_tree_colsum(x, rows, 1).tobytes().hex()
    assert all(r["sum"] == one for r in res)
    # a different schedule (sequential fp64 sum) differs in the last bits here,
    # so the equality above is not vacuous
    assert np.asarray(x, np.float64).sum(axis=0).tobytes().hex() != one
