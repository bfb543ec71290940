"""Throughput of the layered eval path (hidden widths > 256, zf_layered.hip):
log_prob and inverse over 2^20 rows with inputs resident in HBM, HIP-event
timed, flops = 2 * sum of the Dense layers' in x out per row.  GPU box only.

    python scripts/layered_bench.py [--configs h512,h1024] [--rows 1048576]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

SHAPES = {  # (D, C, K, layers, latent)
    "h512": dict(D=4, C=0, K=16, layers=(512, 512), latent="normal"),
    "h1024": dict(D=4, C=0, K=16, layers=(1024, 1024), latent="normal"),
    "h384c2": dict(D=3, C=2, K=8, layers=(384,), latent="beta", act="gelu"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="h512,h1024")
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()

    from tests import flowcases
    from zenflow_amd import _lib as L

    for name in args.configs.split(","):
        flowcases.CONFIGS.setdefault(name, SHAPES[name])
        case = flowcases.make_case(name, N=args.rows, seed=3)
        cfg = case["cfg"]
        flow = flowcases.build_flow(cfg)
        bf = flow.bind(case["variables"], cfg["D"], cfg["C"])
        prog = bf.program
        D, C = cfg["D"], cfg["C"]
        dt, dc = D // 2, D - D // 2
        dims = [dc + C] + list(cfg["layers"]) + [dt * (3 * cfg["K"] - 1)]
        flops_row = 2 * sum(a * b for a, b in zip(dims[:-1], dims[1:])) * cfg.get("couplings", D)
        x = L.DeviceArray.from_numpy(case["x"])
        c = None if case["c"] is None else L.DeviceArray.from_numpy(case["c"])
        out = {}
        for mode in ("log_prob", "inverse"):
            lp = L.DeviceArray((args.rows,))
            y = L.DeviceArray((args.rows, D))
            run = (lambda: prog.log_prob(x, c, out=lp)) if mode == "log_prob" else (lambda: prog.inverse(x, c, out=y))
            run()
            L.synchronize()
            e0, e1 = L.Event(), L.Event()
            e0.record()
            for _ in range(args.steps):
                run()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_ms(e1) / args.steps
            out[mode] = {"ms": ms, "samples_per_s": args.rows / ms * 1e3,
                         "tflops": flops_row * args.rows / ms * 1e-9}
        print(json.dumps({"config": name, "variant": prog.kernel_variant, "rows": args.rows,
                          "flops_per_row": flops_row, **out}), flush=True)


if __name__ == "__main__":
    main()
