"""Training-step throughput: samples/s of
``Trainer.step`` (train-mode forward + reverse pass + nadamw update) for a
few batch sizes on the BASELINE configs.  GPU box only; not part of bench.py's
contract (the headline metric is the eval-mode log_prob).

    python scripts/train_bench.py [--configs cfg1,cfg2,cfg5] [--batches 1024,16384,65536]
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg1,cfg2,cfg5")
    ap.add_argument("--batches", default="1024,16384,65536")
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()

    from tests.flowcases import build_flow, make_case
    from zenflow_amd import _lib as L
    from zenflow_amd._lib import DeviceArray
    from zenflow_amd.train import Trainer

    for name in args.configs.split(","):
        for B in [int(b) for b in args.batches.split(",")]:
            case = make_case(name, N=B, seed=5)
            cfg = case["cfg"]
            flow = build_flow(cfg)
            flow.latent._dim = cfg["D"]
            tr = Trainer(flow, case["variables"], cfg["D"], cfg["C"], B)
            xd = DeviceArray.from_numpy(np.ascontiguousarray(case["x"]))
            cd = None if case["c"] is None else DeviceArray.from_numpy(np.ascontiguousarray(case["c"]))
            for _ in range(3):
                tr.step(xd, cd)
            L.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.step(xd, cd)
            L.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            print(json.dumps({"config": name, "batch": B, "ms_per_step": round(dt * 1e3, 4),
                              "samples_per_s": round(B / dt), "loss": tr.last_loss()}), flush=True)
            del tr


if __name__ == "__main__":
    main()
