"""RCCL plumbing on one GPU (the 8-GPU path itself only runs on the driver's
node): librccl loads, a 1-rank communicator initialises, the fp64 NLL
all-reduce runs on the library stream and returns the rank's own sum."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_single_rank_allreduce():
    from zenflow_amd import _lib as L
    from zenflow_amd.dist import RcclCommunicator, nll_from_sum

    lib = L.load_library()
    if not lib.zf_rccl_available():
        pytest.skip("librccl not present on this box")
    comm = RcclCommunicator(0, 1, lambda b: b)
    buf = L.DeviceArray.from_numpy(np.array([-1234.5678], np.float64))
    comm.allreduce_sum_(buf)
    L.synchronize()
    assert buf.numpy()[0] == -1234.5678
    assert nll_from_sum(buf.numpy()[0], 10) == pytest.approx(123.45678)
    comm.close()


def test_overlapped_allreduce_ring():
    """dist.OverlappedAllreduce: partials written on the compute stream,
    all-reduced on the comm stream, across more steps than the ring holds
    (slot reuse waits on the slot's previous all-reduce)."""
    from zenflow_amd import _lib as L
    from zenflow_amd.dist import OverlappedAllreduce, RcclCommunicator

    lib = L.load_library()
    if not lib.zf_rccl_available():
        pytest.skip("librccl not present on this box")
    comm = RcclCommunicator(0, 1, lambda b: b)
    ar = OverlappedAllreduce(comm, depth=4)
    vals = np.arange(11, dtype=np.float64) * 1.5 - 3.0
    srcs = [L.DeviceArray.from_numpy(np.array([v], np.float64)) for v in vals]
    L.synchronize()
    for s in srcs:
        buf = ar.buffer()
        L.check(lib.zf_memcpy_dtod(buf.ptr, s.ptr, 8, L.stream()), "dtod")
        ar.launch()
    L.check(lib.zf_device_synchronize(), "sync")
    assert ar.last.numpy()[0] == vals[-1]
    # the ring's slots hold the last `depth` steps' all-reduced partials
    assert sorted(float(b.numpy()[0]) for b in ar.bufs) == sorted(vals[-4:].tolist())
    comm.close()


def test_rccl_allgather_one_rank():
    """zf_rccl_allgather (the trainer's zf_allgather_fn over RCCL) on a
    one-rank communicator: recv = send."""
    from zenflow_amd import _lib as L
    from zenflow_amd._lib import DeviceArray
    from zenflow_amd.dist import RcclCommunicator

    comm = RcclCommunicator(0, 1, lambda b: b, force=True)
    try:
        src = DeviceArray.from_numpy(np.arange(37, dtype=np.float64))
        dst = DeviceArray((37,), np.float64)
        L.check(L.load_library().zf_rccl_allgather(comm.comm, src.ptr, dst.ptr, 37 * 8, L.stream()), "allgather")
        assert np.array_equal(dst.numpy(), np.arange(37, dtype=np.float64))
        d = comm.trainer_comm_desc()
        assert d.world == 1 and d.allgather
    finally:
        comm.close()
