"""Diagnostic: strict parity per config x kernel scheme, with the worst rows'
conditioning (row_sensitivity) and latent value, over several seeds.

    python scripts/diag_strict.py [cfg ...]   -> gpurun_out/diag_strict.jsonl
"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import zf_oracle as O  # noqa: E402
from tests.flowcases import build_flow, make_case  # noqa: E402

names = sys.argv[1:] or ["cfg4"]
out = ROOT / "gpurun_out" / "diag_strict.jsonl"
out.parent.mkdir(exist_ok=True)
for scheme in ["f16x2", "bf16x3", "fp32"]:
    if scheme == "fp32":
        os.environ["ZF_DISABLE_X3"] = "1"
    else:
        os.environ.pop("ZF_DISABLE_X3", None)
        os.environ["ZF_X3_SCHEME"] = scheme
    for name in names:
        for seed in (41, 42, 43):
            case = make_case(name, N=4096, seed=seed)
            flow = build_flow(case["cfg"])
            lp = flow.apply(case["variables"], case["x"], case["c"])
            r32, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"])
            r64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
            sens = O.row_sensitivity(case["model"], case["variables"], case["x"], case["c"])
            f = (np.abs(lp) < 1e38) & (np.abs(r32) < 1e38) & np.isfinite(r64) & (np.abs(r64) < 1e300)
            sc = np.maximum(1, np.abs(r64))
            eg = np.where(f, np.abs(lp - r64) / sc, 0)
            eo = np.where(f, np.abs(r32 - r64) / sc, 0)
            es = np.where(f, sens / sc, 0)
            worst = np.argsort(-eg)[:5]
            rec = dict(scheme=scheme, config=name, seed=seed, gpu64_max=float(eg.max()), o32_max=float(eo.max()),
                       gpu64_mean=float(eg[f].mean()), o32_mean=float(eo[f].mean()),
                       strict=float((np.abs(lp - r32) / np.maximum(1, np.abs(r32)))[f].max()),
                       worst=[dict(row=int(i), eg=float(eg[i]), eo=float(eo[i]), sens=float(es[i]),
                                   lp64=float(r64[i])) for i in worst])
            with open(out, "a") as fh:
                fh.write(json.dumps(rec) + "\n")
            print(json.dumps({k: v for k, v in rec.items() if k != "worst"}), flush=True)
