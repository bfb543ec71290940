"""Diagnostic: error of each library variant vs the fp64 / fp32 oracle."""
import os, sys, json
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import zf_oracle as O
from tests.flowcases import build_flow, make_case

res = {"lib": os.environ.get("ZF_LIB", "default")}
for name, N, seed in [("cfg2", 4096, 11), ("cfg4", 4096, 11), ("deep", 4096, 11), ("cfg2", 65536, 3)]:
    case = make_case(name, N=N, seed=seed)
    lp = build_flow(case["cfg"]).apply(case["variables"], case["x"], case["c"])
    r32, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"])
    r64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
    f = np.isfinite(lp) & np.isfinite(r32) & np.isfinite(r64) & (np.abs(r32) < 1e38)
    sc = np.maximum(1, np.abs(r64[f]))
    eg = np.abs(lp[f] - r64[f]) / sc
    eo = np.abs(r32[f] - r64[f]) / sc
    d = np.abs(lp[f] - r32[f]) / sc
    res[f"{name}/{N}"] = dict(gpu64_max=float(eg.max()), gpu64_p999=float(np.quantile(eg, .999)),
                              gpu64_mean=float(eg.mean()), o32_max=float(eo.max()), o32_mean=float(eo.mean()),
                              gpu_vs_o32_max=float(d.max()))
print(json.dumps(res))
