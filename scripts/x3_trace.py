"""Phase timing of the bf16x3 kernel from s_memtime stamps (tuning only).

Needs a library built with -DZF_X3_TRACE=1 (scripts/x3_trace.sh) passed as
ZF_LIB.  Prints, per wave, where the cycles of one block go: barrier waits,
group MFMA phases, layer 0, hidden epilogue, spline."""
import ctypes as ct
import os
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from zenflow_amd import _lib as L  # noqa: E402
from zenflow_amd._lib import DeviceArray  # noqa: E402
from zenflow_amd.random import PRNGKey  # noqa: E402

L.ensure_device()
name = os.environ.get("CFG", "cfg2")
D, C, K, layers, nL, latent, mode = bench.WORKLOADS[name]
flow = bench.build_model(name)
x0 = np.random.default_rng(3).standard_normal((1 << 14, D)).astype(np.float32)
v = flow.init(PRNGKey(1), x0[:1])
_, upd = flow.apply(v, x0, train=True, mutable=["batch_stats"])
v = {"params": v["params"], "batch_stats": upd["batch_stats"]}
N = 1 << 20
x = np.random.default_rng(5).standard_normal((N, D)).astype(np.float32)
bf = flow.bind(v, D, C)
print("kernel", bf.program.kernel_variant, "variant", os.environ.get("ZF_X3_VARIANT", "0"))
xd = DeviceArray.from_numpy(x)
lib = L.load_library()
buf = (ct.c_ulonglong * (4 * 8 * 256))()
cnt = (ct.c_int * 32)()
for _ in range(3):
    bf.log_prob(xd)
L.synchronize()
lib.zf_debug_x3_trace(buf, cnt)
bf.log_prob(xd)
L.synchronize()
lib.zf_debug_x3_trace(buf, cnt)
a = np.frombuffer(buf, dtype=np.uint64).reshape(4, 8, 256)
n = np.frombuffer(cnt, dtype=np.int32).reshape(4, 8)
names = {0: "start", 1: "arrive", 2: "depart", 3: "nsc", 4: "l0_done", 5: "hid_done", 6: "epi_done",
         7: "last_done", 8: "spline_done", 9: "ops_done", 10: "end"}
for tb in range(4):
    tot = defaultdict(float)
    waves = [w for w in range(8) if n[tb, w] > 0]
    for w in waves:
        k = min(int(n[tb, w]), 256)
        ev = (a[tb, w, :k] >> 48).astype(int)
        t = (a[tb, w, :k] & ((1 << 48) - 1)).astype(np.int64)
        t = t - t[0]
        for i in range(1, k):
            tot[(names[ev[i - 1]], names[ev[i]])] += (t[i] - t[i - 1]) / len(waves)
    span = sum(tot.values())
    print(f"block#{tb}: avg wave span {span:.0f} ticks; segments (avg per wave, ticks):")
    for key, val in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"   {key[0]:>12s} -> {key[1]:<12s} {val:9.0f}  {100 * val / span:5.1f}%")
