"""Diagnostic: cfg4 (seed 41, 4096 rows) per-row error vs fp64 under the three
kernel schemes, on the rows where the f16x2 error exceeds the fp32 oracle's
largest error (writes gpurun_out/cfg4_rows.json)."""
import json, os, sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import zf_oracle as O
from tests.flowcases import build_flow, make_case

case = make_case("cfg4", N=4096, seed=41)
lp = {}
for scheme in ["f16x2", "bf16x3", "fp32"]:
    os.environ.pop("ZF_DISABLE_X3", None)
    os.environ.pop("ZF_X3_SCHEME", None)
    if scheme == "fp32":
        os.environ["ZF_DISABLE_X3"] = "1"
    else:
        os.environ["ZF_X3_SCHEME"] = scheme
    flow = build_flow(case["cfg"])
    bf = flow.bind(case["variables"], case["cfg"]["D"], case["cfg"]["C"])
    assert bf.program.kernel_variant == scheme, bf.program.kernel_variant
    lp[scheme] = flow.apply(case["variables"], case["x"], case["c"])
r32, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"])
r64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
sens = O.row_sensitivity(case["model"], case["variables"], case["x"], case["c"])
sc = np.maximum(1, np.abs(r64))
e = {k: np.abs(v - r64) / sc for k, v in lp.items()}
eo = np.abs(r32 - r64) / sc
order = np.argsort(-e["f16x2"])[:12]
rows = [dict(row=int(i), lp64=float(r64[i]), sens=float(sens[i] / sc[i]), oracle32=float(eo[i]),
             **{k: float(e[k][i]) for k in e}) for i in order]
out = dict(oracle32_max=float(eo.max()), **{f"{k}_max": float(e[k].max()) for k in e},
           **{f"{k}_argmax": int(e[k].argmax()) for k in e}, top_rows_by_f16x2=rows)
print(json.dumps(out, indent=1))
