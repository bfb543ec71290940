"""Standalone K1 (rational_quadratic_spline_forward/inverse) timing at one
cfg2 coupling's shapes; prints GB/s vs the HBM peak."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import json
from bench import spline_kernel_roofline
M = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 16
print(json.dumps(spline_kernel_roofline(M, 2, K, 20)))
