"""Print GPU (f16x2 / bf16x3 / fp32 kernels) vs oracle log_prob on the first
rows of a tests/flowcases case: python scripts/diag_case.py NAME N SEED."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import zf_oracle as O  # noqa: E402
from tests.flowcases import build_flow, make_case  # noqa: E402

name, N, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
case = make_case(name, N=N, seed=seed)
ref32, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"])
ref64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
out = {}
for tag, env in (("f16x2", {}), ("bf16x3", {"ZF_X3_SCHEME": "bf16x3"}), ("fp32", {"ZF_DISABLE_X3": "1"})):
    for k in ("ZF_X3_SCHEME", "ZF_DISABLE_X3"):
        os.environ.pop(k, None)
    os.environ.update(env)
    flow = build_flow(case["cfg"])
    bf = flow.bind(case["variables"], case["cfg"]["D"], case["cfg"]["C"])
    print(tag, "kernel", bf.program.kernel_variant)
    out[tag] = build_flow(case["cfg"]).apply(case["variables"], case["x"], case["c"])
bad = np.zeros(N, bool)
for tag, lp in out.items():
    bad |= np.isfinite(lp) != np.isfinite(ref32)
    f = np.isfinite(lp) & np.isfinite(ref32)
    e = np.abs(lp[f] - ref32[f]) / np.maximum(1, np.abs(ref32[f]))
    print(tag, "finite mismatches", int((np.isfinite(lp) != np.isfinite(ref32)).sum()), "max rel", e.max() if e.size else None)
for i in np.flatnonzero(bad)[:10]:
    print(i, "x", case["x"][i], "c", None if case["c"] is None else case["c"][i], "ref32", ref32[i], "ref64", ref64[i],
          {t: float(v[i]) for t, v in out.items()})
