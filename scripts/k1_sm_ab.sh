#!/bin/bash
# A/B of the K1 slope-fetch forms (ZF_K1_SM) + K1 parity tests under each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for SM in 1 2; do
  ZF_K1_SM=$SM timeout -k 10 300 python -m pytest tests/test_gpu_rqs.py -m gpu -q -p no:cacheprovider --timeout 120 > gpurun_out/k1_test_$SM.log 2>&1 || { tail -20 gpurun_out/k1_test_$SM.log; exit 1; }
  tail -1 gpurun_out/k1_test_$SM.log
done
for K in 8 16 32; do
  for SM in 0 1 2 0 1 2; do
    ZF_K1_SM=$SM timeout -k 10 200 python scripts/bench_rqs.py 20 $K > gpurun_out/k1_$SM.log 2>&1 || { tail -5 gpurun_out/k1_$SM.log; exit 1; }
    python - "$SM" "$K" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/k1_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(f"SM={sys.argv[1]} K={sys.argv[2]:>2s}  " + "  ".join(f"{k} {v['achieved']:.0f} GB/s ({v['frac']:.3f})" for k, v in d.items()))
PY
  done
done
