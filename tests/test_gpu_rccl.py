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
