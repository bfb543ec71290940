"""A/B parity diagnosis (GPU box): log_prob of ab/lib{A,B}.so vs the fp64
oracle on one test case; prints error stats and the worst rows.
usage: ZF_LIB=ab/libB.so python scripts/diag_ab_parity.py cfg2 4096"""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import zf_oracle as O
from tests.flowcases import build_flow, make_case

name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
case = make_case(name, N=N, seed=11)
lp = build_flow(case["cfg"]).apply(case["variables"], case["x"], case["c"])
r64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
r32, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float32)
sc = np.maximum(1, np.abs(r64))
e = np.abs(lp - r64) / sc
e32 = np.abs(r32 - r64) / sc
ok = np.isfinite(e)
print(f"{name} N={N}: gpu max {e[ok].max():.3g} mean {e[ok].mean():.3g} | o32 max {e32[ok].max():.3g} mean {e32[ok].mean():.3g}")
for i in np.argsort(-np.where(ok, e, 0))[:5]:
    print(f"  row {i}: gpu {lp[i]:.7g} o64 {r64[i]:.7g} o32 {r32[i]:.7g} x {case['x'][i]}")
