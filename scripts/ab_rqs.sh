#!/bin/bash
# A/B the K1 spline kernels (LIBS from tune/) at one coupling's shapes for K in $KS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for K in ${KS:-8 16 32}; do
  for v in ${LIBS:-A B}; do
    ZF_LIB=tune/lib$v.so timeout -k 10 200 python scripts/bench_rqs.py 20 $K > gpurun_out/abr_$v.log 2>&1 || { tail -5 gpurun_out/abr_$v.log; exit 1; }
    python - "$v" "$K" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/abr_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>8s} K={sys.argv[2]:>2s}  " + "  ".join(f"{k} {v['achieved']:.0f} GB/s ({v['frac']:.3f})" for k, v in d.items() if isinstance(v, dict) and 'achieved' in v))
PY
  done
done
