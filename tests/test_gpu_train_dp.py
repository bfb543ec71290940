"""Data-parallel training (train() with the cross-GPU
reductions of ShiftBounds min/max, BatchNorm sums and the gradient;
train.py:64-86, bijectors.py:250-257, :342).

Two ranks share this box's one GPU (tests/dist_worker.py ``train_dp``; the
trainer's all-gather goes through dist.HostAllgather, since RCCL refuses two
ranks on one device), each on its half of every batch.  The trainer's batch
reductions are fixed leaf trees whose shape depends on the global batch only,
so both ranks must end with the bits ONE device gets on the whole batch:
the same loss, the same gradient, and after three optimiser steps the same
parameters and statistics — compared with ``array_equal``, not a tolerance.
65536 rows is past the batch at which the forward GEMMs switch to 128-row
tiles (chosen by the global batch, so a 32768-row shard switches too)."""

import os
from pathlib import Path

import numpy as np
import pytest

from tests.test_gpu_train import _setup

pytestmark = pytest.mark.gpu
WORKER = str(Path(__file__).resolve().parent / "dist_worker.py")


@pytest.mark.parametrize("name,N,seed", [("cfg2", 1024, 81), ("cfg4", 2048, 82), ("d8", 1024, 83),
                                         ("cfg2", 16384, 84), ("cfg2", 65536, 85)])
def test_two_ranks_match_one_device_bitwise(tmp_path, name, N, seed):
    from zenflow_amd import _lib as L
    from zenflow_amd.launch import spawn

    env = dict(os.environ, ZF_TEST_CASE=f"{name}:{N}:{seed}", ZF_TEST_STEPS="3", ZF_DEVICE="0")
    assert spawn(2, [WORKER, "train_dp", str(tmp_path)], env=env, timeout=240) == 0
    ranks = [np.load(tmp_path / f"rank{k}.npz") for k in range(2)]

    case, flow, tr = _setup(name, N, seed)  # one device, the whole batch
    loss, g = tr.loss_grad(case["x"], case["c"])
    for _ in range(3):
        tr.step(case["x"], case["c"])
    blob = np.empty_like(tr.program.blob)
    L.check(L.load_library().zf_trainer_get_blob(tr.handle, blob.ctypes.data), "get_blob")
    for k, r in enumerate(ranks):
        assert float(r["loss"]) == loss, f"rank {k} loss"
        assert np.array_equal(r["grad"], g), f"rank {k}: {np.sum(r['grad'] != g)} gradient entries differ"
        assert float(r["last_loss"]) == tr.last_loss(), f"rank {k} last loss"
        assert np.array_equal(r["blob"], blob, equal_nan=True), f"rank {k}: {np.sum(r['blob'] != blob)} blob entries"


def test_train_function_two_ranks_match_one_device(tmp_path):
    """zenflow_amd.train(..., comm=...) (train.py:18-138's loop, batches cut
    into per-rank shards; 2400 rows in batches of 512, the last one ragged):
    both ranks return the one-device result — the same losses per epoch, the
    same best epoch and the same best variables, bit for bit."""
    import zenflow_amd as zf
    from tests.dist_worker import two_moons_data, two_moons_flow
    from zenflow_amd.io import flatten_variables
    from zenflow_amd.launch import spawn

    env = dict(os.environ, ZF_TEST_EPOCHS="20", ZF_DEVICE="0")
    assert spawn(2, [WORKER, "train_fn", str(tmp_path)], env=env, timeout=300) == 0
    X = two_moons_data()
    best, best_epoch, lt, ls = zf.train(two_moons_flow(), X[:2400], X[2400:], epochs=20, batch_size=512,
                                        progress=False)
    flat = flatten_variables(best)
    for k in range(2):
        r = np.load(tmp_path / f"rank{k}.npz")
        assert int(r["best_epoch"]) == best_epoch
        assert np.array_equal(r["lt"], np.asarray(lt)) and np.array_equal(r["ls"], np.asarray(ls))
        for name, v in flat.items():
            assert np.array_equal(r["v:" + name], v), f"rank {k}: {name}"


def _train_fn_ranks(tmp_path, ntrain, epochs=20):
    from tests.dist_worker import two_moons_data, two_moons_flow
    from zenflow_amd.launch import spawn
    import zenflow_amd as zf

    env = dict(os.environ, ZF_TEST_EPOCHS=str(epochs), ZF_TEST_NTRAIN=str(ntrain), ZF_DEVICE="0")
    assert spawn(2, [WORKER, "train_fn", str(tmp_path)], env=env, timeout=300) == 0
    X = two_moons_data()
    one = zf.train(two_moons_flow(), X[:ntrain], X[2400:], epochs=epochs, batch_size=512, progress=False)
    return [np.load(tmp_path / f"rank{k}.npz") for k in range(2)], one


def test_train_function_batch_smaller_than_world(tmp_path):
    """2049 rows in batches of 512: the last batch has 1 row, fewer than the
    2 ranks.  The reference trains on it (train.py:111-117); every rank steps
    it on the whole batch without reductions, so both ranks still return the
    one-device result bit for bit."""
    from zenflow_amd.io import flatten_variables

    ranks, (best, best_epoch, lt, ls) = _train_fn_ranks(tmp_path, 2049)
    flat = flatten_variables(best)
    for k, r in enumerate(ranks):
        assert int(r["best_epoch"]) == best_epoch
        assert np.array_equal(r["lt"], np.asarray(lt)) and np.array_equal(r["ls"], np.asarray(ls)), f"rank {k}"
        for name, v in flat.items():
            assert np.array_equal(r["v:" + name], v), f"rank {k}: {name}"


def test_train_function_uneven_shards(tmp_path):
    """2401 rows: the last batch (353 rows) splits 177/176.  The documented
    guarantee is that the ranks stay identical to each other (their fp64
    reduction order then differs from one device's, so only closeness to the
    one-device losses is asserted)."""
    ranks, (_, _, lt, _) = _train_fn_ranks(tmp_path, 2401)
    a, b = ranks
    assert int(a["best_epoch"]) == int(b["best_epoch"])
    assert np.array_equal(a["lt"], b["lt"]) and np.array_equal(a["ls"], b["ls"])
    for name in a.files:
        if name.startswith("v:"):
            assert np.array_equal(a[name], b[name]), name
    np.testing.assert_allclose(a["lt"], np.asarray(lt), rtol=1e-2)


def test_rccl_two_ranks_match_one_device_bitwise(tmp_path):
    """The product DP training path: Trainer(comm=RcclCommunicator), one rank
    per GPU, every batch reduction an ncclAllGather of the ranks' fp64 tree
    roots.  Needs two visible GPUs (the driver's multi-GPU node); both ranks
    must end with one device's loss, gradient and parameters, bit for bit."""
    from zenflow_amd import _lib as L
    from zenflow_amd.launch import spawn

    if L.device_count() < 2:
        pytest.skip("needs 2 GPUs (RCCL refuses two ranks on one device)")
    if not L.load_library().zf_rccl_available():
        pytest.skip("librccl not present on this box")
    env = dict(os.environ, ZF_TEST_CASE="cfg2:4096:91", ZF_TEST_STEPS="3")
    env.pop("ZF_DEVICE", None)  # one GPU per rank (LOCAL_RANK)
    assert spawn(2, [WORKER, "train_rccl", str(tmp_path)], env=env, timeout=240) == 0
    ranks = [np.load(tmp_path / f"rank{k}.npz") for k in range(2)]
    case, flow, tr = _setup("cfg2", 4096, 91)
    loss, g = tr.loss_grad(case["x"], case["c"])
    for _ in range(3):
        tr.step(case["x"], case["c"])
    blob = np.empty_like(tr.program.blob)
    L.check(L.load_library().zf_trainer_get_blob(tr.handle, blob.ctypes.data), "get_blob")
    for k, r in enumerate(ranks):
        assert float(r["loss"]) == loss, f"rank {k} loss"
        assert np.array_equal(r["grad"], g), f"rank {k} gradient"
        assert np.array_equal(r["blob"], blob, equal_nan=True), f"rank {k} blob"
