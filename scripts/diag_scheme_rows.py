"""Diagnostic: per-row error vs fp64 under the three kernel schemes (f16x2,
bf16x3, the unsplit fp32 kernel), with each row's conditioning, on the rows
where f16x2 leaves 1e-5 of the fp32 oracle or exceeds the oracle's largest
error vs fp64.  Cases: cfg4 (seed 41, 4096 rows) or trained_<cfg> (the
tests/golden trained weights and held-out data).  Prints JSON.

    python scripts/diag_scheme_rows.py trained_cfg1
"""
import json, os, sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import zf_oracle as O
from tests.flowcases import build_flow, make_case
from zenflow_amd.io import load_variables

name = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
if name.startswith("trained_"):
    g = ROOT / "tests" / "golden"
    d = np.load(g / f"{name}_data.npz")
    base = make_case(name[len("trained_"):], N=1, seed=0)
    case = dict(base, variables=load_variables(g / f"{name}.npz"), x=d["x"], c=d["c"] if "c" in d.files else None)
else:
    case = make_case(name, N=4096, seed=41)
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
f = np.isfinite(r64) & np.isfinite(r32) & np.all([np.isfinite(v) for v in lp.values()], axis=0)
sc = np.maximum(1, np.abs(r64))
e = {k: np.where(f, np.abs(v - r64) / sc, 0) for k, v in lp.items()}
s = {k: np.where(f, np.abs(v.astype(np.float64) - r32) / np.maximum(1, np.abs(r32)), 0) for k, v in lp.items()}
eo = np.where(f, np.abs(r32 - r64) / sc, 0)
pick = np.union1d(np.where(s["f16x2"] > 1e-5)[0], np.where(e["f16x2"] > eo.max())[0])
pick = pick[np.argsort(-s["f16x2"][pick])][:40]
rows = [dict(row=int(i), lp64=float(r64[i]), sens=float(sens[i] / sc[i]), oracle32=float(eo[i]),
             **{k: float(e[k][i]) for k in e}, **{f"strict_{k}": float(s[k][i]) for k in s}) for i in pick]
out = dict(case=name, rows=int(f.sum()), oracle32_max=float(eo.max()), oracle32_mean=float(eo[f].mean()),
           **{f"{k}_max": float(e[k].max()) for k in e}, **{f"{k}_mean": float(e[k][f].mean()) for k in e},
           **{f"strict_{k}_max": float(s[k].max()) for k in s}, **{f"{k}_argmax": int(e[k].argmax()) for k in e},
           rows_f16x2_strict_over_1e5_or_over_oracle_max=rows)
print(json.dumps(out, indent=1))
