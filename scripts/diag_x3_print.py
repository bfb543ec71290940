"""Debug aid (GPU box, printf build in ab/libC.so): oracle intermediates of
row 0 in the first coupling, to compare with the kernel's DBG lines."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import zf_oracle as O
from tests.flowcases import build_flow, make_case

case = make_case("cfg2", N=1, seed=11)
orig = O.nsc_params
calls = []
def hooked(spec, params, stats, x, c, train, dt):
    if not calls and dt == np.float32:
        u = x[:, x.shape[1] // 2:]
        u, _ = O._batchnorm(u, params["BatchNorm_0"], stats["BatchNorm_0"], False, dt)
        for li in range(3):
            d = params[f"Dense_{li}"]
            v = u @ np.asarray(d["kernel"], dt) + np.asarray(d["bias"], dt)
            print(f"ORACLE L{li} v*log2e {v[0,:4] * 1.4426950408889634}  raw {v[0,:4]}")
            u = O.swish(v)
    calls.append(1)
    return orig(spec, params, stats, x, c, train, dt)
O.nsc_params = hooked
O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float32)
lp = build_flow(case["cfg"]).apply(case["variables"], case["x"], case["c"])
print("gpu", lp)
