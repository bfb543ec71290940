"""Where the time of one drop-in ``flow.apply(variables, x)`` call goes at
config 1 (two_moons, 4096 rows, host in / host out): program lookup (the
content digest), upload, kernel, download.  GPU box; prints one JSON line."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from zenflow_amd import flow as F  # noqa: E402
from zenflow_amd.random import PRNGKey  # noqa: E402


def best(fn, n=200):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


flow = bench.build_model("cfg1")
x = np.random.default_rng(0).standard_normal((4096, 2)).astype(np.float32)
v = flow.init(PRNGKey(1), x[:1])
flow.apply(v, x)
sub = {k: vv["bijector"] for k, vv in v.items()}
out = {
    "apply_us": best(lambda: flow.apply(v, x)),
    "digest_us": best(lambda: F._digest(sub)),
}
from zenflow_amd._lib import DeviceArray  # noqa: E402

bound = flow.bind(v, 2, 0)
xd = DeviceArray.from_numpy(x)
out["upload_us"] = best(lambda: DeviceArray.from_numpy(x))
out["bound_device_in_host_out_us"] = best(lambda: bound.log_prob(xd).numpy())
print(json.dumps(out))
