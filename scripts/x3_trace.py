"""Tuning: per-wave phase breakdown of the split-MFMA kernel from a
-DZF_X3_TRACE=1 build (python -m zenflow_amd.build --out tune/libtrace.so
-DZF_X3_TRACE=1), run on the GPU box as

    ZF_LIB=tune/libtrace.so python scripts/x3_trace.py [cfg2] [rows_log2]

Prints mean s_memtime ticks per wave-coupling for each phase."""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("ZF_ALLOW_MISSING_SYMBOLS", "1")
import bench  # noqa: E402
from zenflow_amd import _lib as L  # noqa: E402
from zenflow_amd._lib import DeviceArray  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
N = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 20)
D, Cd, K, layers, nL, latent, mode, act = bench.workload(name)
flow, variables, x, c = bench.make_workload(name, N)
prog = flow.bind(variables, D, Cd).program
lib = L.load_library()
nwaves = (N + 127) // 128 * 4
buf = DeviceArray((nwaves * 16,), np.uint64)
fn = getattr(lib, f"zf_x3_trace_set_k{K}")
fn.argtypes = [C.c_void_p]
assert fn(buf.ptr) == 0
xd = DeviceArray.from_numpy(x)
cd = DeviceArray.from_numpy(c) if c is not None else None  # conditional flows (cfg4)
out = DeviceArray((N,))
for _ in range(5):
    prog.log_prob(xd, cd, out=out)
L.synchronize()
t = buf.numpy().reshape(nwaves, 16).astype(np.float64)
names = ["start->nsc", "layer0", "hidden", "hid->last", "last", "spline", "epilogue", "barrier_wait", "total",
         "couplings", "sb", "plain_step_dma_issue", "plain_step_group"]
ncoup = t[:, 9].mean()
res = {"config": name, "rows": N, "kernel": prog.kernel_variant, "couplings": ncoup}
for k, nm in enumerate(names):
    if k == 9:
        continue
    v = t[:, k] / (ncoup if k not in (8, 6) else 1)
    res[nm] = {"mean": float(v.mean()), "p10": float(np.percentile(v, 10)), "p90": float(np.percentile(v, 90))}
print(json.dumps(res, indent=1))
