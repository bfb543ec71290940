"""Diagnostic (GPU box): the tiny-activation regime of
test_split_scaling_extremes_other_acts for one activation under each kernel
(fp32 K2, bf16x3, f16x2 where eligible): GPU vs fp64 against the fp32
oracle vs fp64 and the conditioned tolerance.
    python scripts/diag_acts.py [softplus|sigmoid] -> stdout JSON lines"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import zf_oracle as O  # noqa: E402
from tests.flowcases import build_flow, make_case  # noqa: E402

F32 = np.float32
name = sys.argv[1] if len(sys.argv) > 1 else "softplus"
for scheme in ("fp32", "bf16x3", "f16x2"):
    os.environ.pop("ZF_DISABLE_X3", None)
    os.environ.pop("ZF_X3_SCHEME", None)
    if scheme == "fp32":
        os.environ["ZF_DISABLE_X3"] = "1"
    else:
        os.environ["ZF_X3_SCHEME"] = scheme
    for regime in ("tiny_activations", "none"):
        case = make_case(name, N=1500, seed=36)
        if regime != "none":
            for key, p in case["variables"]["params"]["bijector"].items():
                if "Dense_1" not in p:
                    continue
                p["Dense_0"]["kernel"] = (p["Dense_0"]["kernel"] * 1e-6).astype(F32)
                p["Dense_0"]["bias"] = (p["Dense_0"]["bias"] * 1e-6).astype(F32)
                p["Dense_1"]["kernel"] = (p["Dense_1"]["kernel"] * 1e4).astype(F32)
        flow = build_flow(case["cfg"])
        bf = flow.bind(case["variables"], case["cfg"]["D"], case["cfg"]["C"])
        lp = np.asarray(flow.apply(case["variables"], case["x"], case["c"]), np.float64)
        r32, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"])
        r64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
        sens = O.row_sensitivity(case["model"], case["variables"], case["x"], case["c"])
        f = np.isfinite(r64) & np.isfinite(lp)
        sc = np.maximum(1, np.abs(r64[f]))
        eg = np.abs(lp[f] - r64[f]) / sc
        eo = np.abs(r32[f] - r64[f]) / sc
        print(json.dumps({"act": name, "scheme": scheme, "kernel": bf.program.kernel_variant, "regime": regime,
                          "gpu_max": float(eg.max()), "o32_max": float(eo.max()), "gpu_mean": float(eg.mean()),
                          "o32_mean": float(eo.mean()), "sens_med": float(np.median(sens[f])),
                          "worst": int(np.argmax(eg))}), flush=True)
