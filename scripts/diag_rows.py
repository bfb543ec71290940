"""Diagnostic: rows of a flow case where the GPU log_prob leaves the parity
band of tests/test_gpu_flow.py (per library variant, ZF_LIB)."""
import os, sys, json
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import zf_oracle as O
from tests.flowcases import build_flow, make_case

for name in sys.argv[1:] or ["cfg1", "cfg2"]:
    case = make_case(name, N=4096, seed=5)
    lp = build_flow(case["cfg"]).apply(case["variables"], case["x"], case["c"])
    r32, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"])
    r64, _ = O.flow_log_prob(case["model"], case["variables"], case["x"], case["c"], dtype=np.float64)
    sc = np.maximum(1, np.abs(r64))
    err = np.abs(lp - r64) / sc
    bad = np.where(~(err <= 1e-5 + 2 * np.abs(r32 - r64) / sc))[0]
    print(os.environ.get("ZF_LIB", "default"), name, "bad rows", len(bad), "of", len(lp), "first", bad[:16].tolist(),
          "lanes", sorted(set((bad % 32).tolist()))[:32], flush=True)
