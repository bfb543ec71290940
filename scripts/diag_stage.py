"""Diagnostic (GPU box): where a config's worst rows against fp64 pick up
their error — stage by stage (after each bijector: state y and log-det, then
the latent), the GPU's one-op segments against the fp64 oracle fed the SAME
fp64 input at every stage (so each stage's own error shows, not what it
inherits), next to the fp32 oracle's error at that stage.

    python scripts/diag_stage.py [cfg4] [f16x2|bf16x3|fp32]  -> stdout JSON lines
"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
name = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
scheme = sys.argv[2] if len(sys.argv) > 2 else "f16x2"
if scheme == "fp32":
    os.environ["ZF_DISABLE_X3"] = "1"
else:
    os.environ["ZF_X3_SCHEME"] = scheme

from oracle import zf_oracle as O  # noqa: E402
from tests.flowcases import build_flow, make_case  # noqa: E402
from zenflow_amd._lib import DeviceArray  # noqa: E402

for seed in (41, 42, 43):
    case = make_case(name, N=4096, seed=seed)
    flow = build_flow(case["cfg"])
    v, x, c = case["variables"], case["x"], case["c"]
    spec = case["model"]["bijector"]
    lp = flow.apply(v, x, c)
    r32, _ = O.flow_log_prob(case["model"], v, x, c)
    r64, _ = O.flow_log_prob(case["model"], v, x, c, dtype=np.float64)
    f = np.isfinite(r64) & (np.abs(lp) < 1e38) & (np.abs(r32) < 1e38)
    sc = np.maximum(1, np.abs(r64))
    eg = np.where(f, np.abs(lp - r64) / sc, 0)
    worst = np.argsort(-eg)[:4]
    prog = flow.bind(v, case["cfg"]["D"], case["cfg"]["C"]).program
    params = v["params"]["bijector"]
    stats = v["batch_stats"]["bijector"]
    cd = None if c is None else DeviceArray.from_numpy(c)
    # stage-by-stage: input of stage i = the fp64 oracle's output of stage i-1
    x64 = x.astype(np.float64)
    stages = []
    for i, b in enumerate(spec["bijectors"]):
        key = f"bijectors_{i}"
        y64, ld64, _ = O.bijector_forward(b, params.get(key), stats.get(key), x64, None if c is None else c.astype(np.float64),
                                          False, np.float64)
        xin32 = x64.astype(np.float32)
        y32, ld32, _ = O.bijector_forward(b, params.get(key), stats.get(key), xin32, c, False, np.float32)
        yg, ldg = prog.forward(DeviceArray.from_numpy(xin32), cd, i, i + 1)
        yg, ldg = yg.numpy(), ldg.numpy()
        rec = {"stage": f"{i}:{b['type']}"}
        for r in worst:
            rec[int(r)] = {
                "y_gpu": float(np.abs(yg[r] - y64[r]).max()), "y_o32": float(np.abs(y32[r] - y64[r]).max()),
                "ld_gpu": float(abs(ldg[r] - ld64[r])), "ld_o32": float(abs(ld32[r] - ld64[r])),
                "y64": [float(t) for t in y64[r]],
            }
        stages.append(rec)
        x64 = y64
    # latent on the fp64 final state
    z32 = x64.astype(np.float32)
    lat64 = O.latent_log_prob(case["model"]["latent"], x64)
    lat32 = O.latent_log_prob(case["model"]["latent"], z32)
    n = len(prog.ops)
    lpg = prog.log_prob(DeviceArray.from_numpy(z32), cd, op_begin=n, op_end=n).numpy()
    stages.append({"stage": "latent", **{int(r): {"lat_gpu": float(abs(lpg[r] - lat64[r])),
                                                  "lat_o32": float(abs(lat32[r] - lat64[r])),
                                                  "lat64": float(lat64[r])} for r in worst}})
    print(json.dumps({"config": name, "scheme": scheme, "seed": seed,
                      "worst": [{"row": int(r), "eg": float(eg[r]), "eo": float(abs(r32[r] - r64[r]) / sc[r]),
                                 "lp64": float(r64[r])} for r in worst],
                      "stages": stages}), flush=True)
