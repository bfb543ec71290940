"""Diagnostic: tiny-activation regime (tests/test_gpu_flow.py
test_split_scaling_extremes_other_acts) under f16x2 and the fp32 kernel:
max / mean error vs fp64 next to the fp32 oracle's, and the worst rows."""
import json, os, sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import zf_oracle as O
from tests.flowcases import build_flow, make_case
F32 = np.float32
out = {}
for name in ["sigmoid", "softplus"]:
    case = make_case(name, N=1500, seed=36)
    for key, p in case["variables"]["params"]["bijector"].items():
        p["Dense_0"]["kernel"] = (p["Dense_0"]["kernel"] * 1e-6).astype(F32)
        p["Dense_0"]["bias"] = (p["Dense_0"]["bias"] * 1e-6).astype(F32)
        p["Dense_1"]["kernel"] = (p["Dense_1"]["kernel"] * 1e4).astype(F32)
    r32, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"])
    r64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
    sc = np.maximum(1, np.abs(r64))
    eo = np.abs(r32 - r64) / sc
    rec = {"oracle32_max": float(eo.max()), "oracle32_mean": float(eo.mean()), "oracle32_argmax": int(eo.argmax())}
    for scheme in ["f16x2", "fp32"]:
        os.environ.pop("ZF_DISABLE_X3", None)
        if scheme == "fp32":
            os.environ["ZF_DISABLE_X3"] = "1"
        flow = build_flow(case["cfg"])
        bf = flow.bind(case["variables"], case["cfg"]["D"], case["cfg"]["C"])
        lp = flow.apply(case["variables"], case["x"], case["c"])
        e = np.abs(lp - r64) / sc
        top = np.argsort(-e)[:5]
        rec[scheme] = {"variant": bf.program.kernel_variant, "max": float(e.max()), "mean": float(e.mean()),
                       "top": [(int(i), float(e[i]), float(eo[i])) for i in top]}
    out[name] = rec
print(json.dumps(out, indent=1))
