"""Bit-identity check of the fused split-set combine (ZF_TRAIN_FUSED_COMBINE,
zf_train.hip mgemm_body): run N training steps at small batches (the
split-set GEMMs' regime) and save every parameter; run once with and once
without the switch (it is read once per process) and compare the files.
GPU box only.

    ZF_TRAIN_FUSED_COMBINE=1 python scripts/fused_combine_check.py out_fused.npz
    python scripts/fused_combine_check.py out_plain.npz
    python scripts/fused_combine_check.py --compare out_fused.npz out_plain.npz
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def run(out, steps=40):
    from tests.flowcases import build_flow, make_case
    from zenflow_amd._lib import DeviceArray
    from zenflow_amd.io import flatten_variables
    from zenflow_amd.train import Trainer

    res = {}
    for name in ("cfg1", "cfg2", "cfg4", "cfg5"):
        for B in (1024, 4096):
            case = make_case(name, N=B, seed=7)
            cfg = case["cfg"]
            flow = build_flow(cfg)
            flow.latent._dim = cfg["D"]
            tr = Trainer(flow, case["variables"], cfg["D"], cfg["C"], B)
            xd = DeviceArray.from_numpy(np.ascontiguousarray(case["x"]))
            cd = None if case["c"] is None else DeviceArray.from_numpy(np.ascontiguousarray(case["c"]))
            losses = []
            for _ in range(steps):
                tr.step(xd, cd)
                losses.append(tr.last_loss())
            for k, v in flatten_variables(tr.variables()).items():
                res[f"{name}/{B}/{k}"] = np.asarray(v)
            res[f"{name}/{B}/losses"] = np.asarray(losses, np.float64)
            del tr
    np.savez(out, **res)
    print("saved", out, len(res))


def compare(a, b):
    A, B = np.load(a), np.load(b)
    assert sorted(A.files) == sorted(B.files)
    bad = [k for k in A.files if not np.array_equal(A[k], B[k], equal_nan=True)]
    print(f"{len(A.files)} arrays, {len(bad)} differ" + (f": {bad[:8]}" if bad else " (bit-identical)"))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    run(sys.argv[1])
